# bf16 GPU tests and bf16 bench (tiled thin transpose), then the N = 2 launcher rehearsed over gloo
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_fstp.py -x -q --timeout 200 --timeout-method thread > gpurun_out/misc_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/misc_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --state-dtype bf16 > gpurun_out/b16_thin.log 2>&1 || exit 1
tail -1 gpurun_out/b16_thin.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bf16', d['value'], d['ms_per_step'])"
timeout -k 10 400 python bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --layers 4 --no-cpu-baseline > gpurun_out/gloo2.log 2>&1
rc=$?; echo "gloo2 rc=$rc"; tail -1 gpurun_out/gloo2.log | cut -c1-300; exit $rc
