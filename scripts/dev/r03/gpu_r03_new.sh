# round 3: the new GPU tests (configs 1 / dense / Llama W=2, bf16 FS/TP, mixed state dtypes, update precision)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_fs.py tests/test_gpu_tp.py tests/test_gpu_bf16.py tests/test_gpu_update_precision.py -v -rf --timeout 600 --timeout-method thread > gpurun_out/pytest_new.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -a -E "PASSED|FAILED|Error|passed|failed" gpurun_out/pytest_new.log | tail -60
exit $rc
