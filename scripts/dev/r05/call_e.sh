# round-5 call E: parity of the fused orthonormalisation tail, then A/B against the round-4 tree
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_bf16.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05e_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/r05e_parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  (cd ab_r04 && timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline) > gpurun_out/r05e_r04_$i.log 2>&1 || exit 1
  grep '^{"metric' gpurun_out/r05e_r04_$i.log | cut -c100-180 | sed 's/^/r04 /'
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r05e_cur_$i.log 2>&1 || exit 1
  grep '^{"metric' gpurun_out/r05e_cur_$i.log | cut -c100-180 | sed 's/^/cur /'
done
timeout -k 10 300 python scripts/dev/r05/diag_phases.py --streams 2 --modes base,no_ortho,no_fixup,only_streaming > gpurun_out/r05e_diag.log 2>&1
grep '^{"streams' gpurun_out/r05e_diag.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/r05e_prof" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --probe-steps 0 --no-cpu-baseline --streams 1 > gpurun_out/r05e_prof.log 2>&1
echo "prof rc=$?"
