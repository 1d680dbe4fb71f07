# round-5 call B: parity of the LDS trsm, then a same-box A/B of the round-4 tree (ab_r04/) against
# HEAD on the Llama and Mixtral bench lines, and the phase-cost diagnostic
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tp.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05b_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/r05b_parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  (cd ab_r04 && timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline) > gpurun_out/r05b_r04_$i.log 2>&1 || exit 1
  grep '^{"metric' gpurun_out/r05b_r04_$i.log | cut -c1-150 | sed 's/^/r04 /'
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r05b_cur_$i.log 2>&1 || exit 1
  grep '^{"metric' gpurun_out/r05b_cur_$i.log | cut -c1-150 | sed 's/^/cur /'
done
(cd ab_r04 && timeout -k 10 300 python bench.py --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 --no-cpu-baseline) > gpurun_out/r05b_r04_mx.log 2>&1 || exit 1
grep '^{"metric' gpurun_out/r05b_r04_mx.log | cut -c150-330 | sed 's/^/r04 mx /'
timeout -k 10 300 python bench.py --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r05b_cur_mx.log 2>&1 || exit 1
grep '^{"metric' gpurun_out/r05b_cur_mx.log | cut -c150-330 | sed 's/^/cur mx /'
timeout -k 10 400 python scripts/dev/r05/diag_phases.py > gpurun_out/r05b_diag.log 2>&1
echo "diag rc=$?"; cat gpurun_out/r05b_diag.log | grep '^{'
