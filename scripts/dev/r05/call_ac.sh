# round-5 call AC: 512-row update blocks at r > 64 (DION_RSL128) against the final tree's library
# (variants/lib_final.so, 256 rows at every r): Mixtral three samples each, Llama one (same kernels)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export DION_DEV_ALLOW_LIB_PATH=1
run() {  # label, lib ("" = this tree), extra bench args
  local label=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then
    DION_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/r05ac_$label.log 2>&1 || return 1
  else
    timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/r05ac_$label.log 2>&1 || return 1
  fi
  python - "$label" gpurun_out/r05ac_$label.log <<'PY'
import json, sys
line = next(l for l in open(sys.argv[2]) if l.startswith('{"metric'))
d = json.loads(line)
print(f"{sys.argv[1]:>12s} {d['value']:8.2f} {d['unit']} {d['ms_per_step']:8.3f} ms")
PY
}
timeout -k 10 300 python -u -m pytest tests/test_gpu_update_precision.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "update or r128 or fixup" > gpurun_out/r05ac_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/r05ac_parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2 3; do
  run mx_final_$i variants/lib_final.so --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
  run mx_new_$i "" --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
done
run final_1 variants/lib_final.so --steps 20 --warmup 3 || exit 1
run new_1 "" --steps 20 --warmup 3 || exit 1
