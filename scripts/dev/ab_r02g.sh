# bf16 state mode: the update on b16_stream_kernel vs b16_update_kernel (b16old): GPU bf16
export DION_DEV_ALLOW_LIB_PATH=1
# tests, then the bf16-state bench line with each library
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_bf16.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_bf16.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --state-dtype bf16 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_bf16.log 2>&1; echo "bf16 rc=$?"; tail -n 1 gpurun_out/bench_bf16.log | cut -c1-200
DION_LIB_PATH=$PWD/megatron-dion_amd/csrc/variants/libdion_codec_b16old.so timeout -k 10 600 python bench.py --state-dtype bf16 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_bf16_old.log 2>&1; echo "bf16 old rc=$?"; tail -n 1 gpurun_out/bench_bf16_old.log | cut -c1-200
