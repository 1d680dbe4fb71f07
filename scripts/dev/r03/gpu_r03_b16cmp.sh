# bf16-state: GPU tests of the bf16 mode, then per-kernel bench comparison new lib vs HEAD lib
export DION_DEV_ALLOW_LIB_PATH=1
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread > gpurun_out/b16_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/b16_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for f in new old new; do
  if [ $f = old ]; then export DION_LIB_PATH=$PWD/megatron-dion_amd/csrc/variants/${OLD_LIB:-libdion_head.so}; else unset DION_LIB_PATH; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --state-dtype bf16 ${BENCH_ARGS:-} > gpurun_out/b16_$f.log 2>&1 || exit 1
  tail -1 gpurun_out/b16_$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step']); [print('  ', k, v['avg_launch_ms'], v['GB/s']) for k,v in d['roofline']['kernels'].items()]"
done
