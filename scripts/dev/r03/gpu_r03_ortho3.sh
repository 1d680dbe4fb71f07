# ortho chain (trsm factor in LDS, 1024-thread r = 128 Cholesky): parity tests, Mixtral + Llama A/B vs $OLD_LIB
export DION_DEV_ALLOW_LIB_PATH=1
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_tp.py -x -q --timeout 300 --timeout-method thread > gpurun_out/o3_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/o3_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for wl in mixtral-8x7b-experts-r128 llama3-8b-2d-grad-set-r64; do
for f in new old; do
  if [ $f = old ]; then export DION_LIB_PATH=$PWD/megatron-dion_amd/csrc/variants/${OLD_LIB}; else unset DION_LIB_PATH; fi
  timeout -k 10 400 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --workload $wl > gpurun_out/o3_$f.log 2>&1 || exit 1
  tail -1 gpurun_out/o3_$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl $f', d['value'], d['ms_per_step'])"
done
done
