# ortho chain: RCQR-heavy parity tests, ortho kernel stats (ortho_bench under rocprofv3), kernel trace of the bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_bf16.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ortho.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ortho.log
if [ $rc -ne 0 ]; then grep -a -B5 "Error\|assert" gpurun_out/pytest_ortho.log | head -60; exit $rc; fi
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/ob" -o run --output-format csv -- python scripts/dev/ortho_bench.py > gpurun_out/ob.log 2>&1 || exit $?
f=$(find gpurun_out/ob -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | grep -v "at::native" | sed 's/(.*)"/"/'
bash scripts/gpu_r03_trace.sh
