# round-5 call J: parity of the scalar-factor solves; same-box A/B (Llama, Mixtral) against round 4
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05j_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/r05j_parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  (cd ab_r04 && timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline) > gpurun_out/r05j_r04_$i.log 2>&1 || exit 1
  grep '^{"metric' gpurun_out/r05j_r04_$i.log | cut -c100-180 | sed 's/^/r04 /'
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r05j_cur_$i.log 2>&1 || exit 1
  grep '^{"metric' gpurun_out/r05j_cur_$i.log | cut -c100-180 | sed 's/^/cur /'
done
(cd ab_r04 && timeout -k 10 300 python bench.py --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 --no-cpu-baseline) > gpurun_out/r05j_r04_mx.log 2>&1 || exit 1
grep '^{"metric' gpurun_out/r05j_r04_mx.log | cut -c150-260 | sed 's/^/r04 mx /'
timeout -k 10 300 python bench.py --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r05j_cur_mx.log 2>&1 || exit 1
grep '^{"metric' gpurun_out/r05j_cur_mx.log | cut -c150-260 | sed 's/^/cur mx /'
