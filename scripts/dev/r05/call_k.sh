# round-5 call K: parity of the fp16x3 Gram, the LDS-staged sketch and the fused r = 128 fix-up;
# solve variants (ubench); same-box A/B: J tree (variants/lib_j.so) vs this tree vs this tree
# with LDS factors (variants/lib_ldsR.so); a Mixtral kernel-stats profile of this tree
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/ubench/trsm_ab > gpurun_out/r05k_trsm.log 2>&1
echo "trsm rc=$?"; cat gpurun_out/r05k_trsm.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05k_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; grep "P maxrel vs oracle" gpurun_out/r05k_parity.log; tail -2 gpurun_out/r05k_parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
export DION_DEV_ALLOW_LIB_PATH=1
run() {  # label, lib ("" = this tree), extra bench args
  local label=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then
    DION_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/r05k_$label.log 2>&1 || return 1
  else
    timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/r05k_$label.log 2>&1 || return 1
  fi
  python - "$label" gpurun_out/r05k_$label.log <<'PY'
import json, sys
line = next(l for l in open(sys.argv[2]) if l.startswith('{"metric'))
d = json.loads(line)
print(f"{sys.argv[1]:>12s} {d['value']:8.2f} {d['unit']} {d['ms_per_step']:8.3f} ms")
PY
}
for i in 1 2; do
  run j_$i variants/lib_j.so --steps 20 --warmup 3 || exit 1
  run new_$i "" --steps 20 --warmup 3 || exit 1
  run ldsR_$i variants/lib_ldsR.so --steps 20 --warmup 3 || exit 1
done
run j_mx variants/lib_j.so --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
run new_mx "" --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05k_prof_mx -o run -- python bench.py --workload mixtral-8x7b-experts-r128 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05k_prof_mx.log 2>&1
echo "prof rc=$?"
