# ortho kernel change: parity tests that exercise RCQR, then kernel stats + bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tp.py tests/test_gpu_fullsize.py tests/test_gpu_bf16.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ortho.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ortho.log
if [ $rc -ne 0 ]; then grep -a -B5 "Error\|assert" gpurun_out/pytest_ortho.log | head -60; exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_ortho" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --streams 1 > gpurun_out/prof_ortho.log 2>&1
rc=$?; echo "prof rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/prof_ortho.log; exit $rc; fi
f=$(find gpurun_out/prof_ortho -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | grep -v "at::native" | head -25
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_ortho.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_ortho.log | cut -c1-300
exit $rc
