# r = 128 (Mixtral experts): r = 128 GPU parity tests, then Mixtral bench A/B (new lib vs $OLD_LIB)
export DION_DEV_ALLOW_LIB_PATH=1
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q -k "128 or mixtral" --timeout 300 --timeout-method thread > gpurun_out/mix_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/mix_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for f in new old; do
  if [ $f = old ]; then export DION_LIB_PATH=$PWD/megatron-dion_amd/csrc/variants/${OLD_LIB}; else unset DION_LIB_PATH; fi
  timeout -k 10 400 python bench.py --steps 4 --warmup 2 --no-cpu-baseline --workload mixtral-8x7b-experts-r128 > gpurun_out/mix_$f.log 2>&1 || exit 1
  tail -1 gpurun_out/mix_$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step']); [print('  ', k, v['avg_launch_ms'], v['GB/s']) for k,v in d['roofline']['kernels'].items()]"
done
