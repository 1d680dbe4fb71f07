# round-5 call V: the ordered partial-sum reductions with eight loads in flight (slab reduction,
# column-norm partials, pass B + fix-up); parity; A/B against call U's tree (variants/lib_u.so)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_bf16.py tests/test_gpu_configs.py -x -q -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05v_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; grep "P maxrel vs oracle" gpurun_out/r05v_parity.log; tail -2 gpurun_out/r05v_parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
export DION_DEV_ALLOW_LIB_PATH=1
run() {  # label, lib ("" = this tree), extra bench args
  local label=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then
    DION_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/r05v_$label.log 2>&1 || return 1
  else
    timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/r05v_$label.log 2>&1 || return 1
  fi
  python - "$label" gpurun_out/r05v_$label.log <<'PY'
import json, sys
line = next(l for l in open(sys.argv[2]) if l.startswith('{"metric'))
d = json.loads(line)
print(f"{sys.argv[1]:>12s} {d['value']:8.2f} {d['unit']} {d['ms_per_step']:8.3f} ms")
PY
}
for i in 1 2; do
  run u_$i variants/lib_u.so --steps 20 --warmup 3 || exit 1
  run new_$i "" --steps 20 --warmup 3 || exit 1
done
run u_mx variants/lib_u.so --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
run new_mx "" --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05v_prof_llama1 -o run -- python scripts/dev/r05/diag_phases.py --streams 1 --modes base --steps 2 > gpurun_out/r05v_prof_llama1.log 2>&1
echo "prof llama rc=$?"
