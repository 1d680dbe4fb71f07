# bf16-state projections: GPU tests of the bf16 mode, then same-box bench A/B (new lib vs HEAD lib)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py -x -v --timeout 200 --timeout-method thread > gpurun_out/b16_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -a -E "passed|failed|FAILED|Error" gpurun_out/b16_tests.log | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
AB_LIB=megatron-dion_amd/csrc/variants/libdion_head.so BENCH_ARGS="--state-dtype bf16" bash scripts/gpu_r03_ab.sh
