# round-5 call L: the GPU suite with LDS factors by default and pass B carrying the fix-up
# (dion_project_r_fixup); same-box A/B against call K's best (variants/lib_ldsR.so); Mixtral
# kernel costs with one stream, and its step with 2 / 3 streams
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05l_pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -2 gpurun_out/r05l_pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
export DION_DEV_ALLOW_LIB_PATH=1
run() {  # label, lib ("" = this tree), extra bench args
  local label=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then
    DION_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/r05l_$label.log 2>&1 || return 1
  else
    timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/r05l_$label.log 2>&1 || return 1
  fi
  python - "$label" gpurun_out/r05l_$label.log <<'PY'
import json, sys
line = next(l for l in open(sys.argv[2]) if l.startswith('{"metric'))
d = json.loads(line)
print(f"{sys.argv[1]:>12s} {d['value']:8.2f} {d['unit']} {d['ms_per_step']:8.3f} ms")
PY
}
for i in 1 2; do
  run k_$i variants/lib_ldsR.so --steps 20 --warmup 3 || exit 1
  run new_$i "" --steps 20 --warmup 3 || exit 1
done
run k_mx variants/lib_ldsR.so --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
run new_mx "" --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
timeout -k 10 300 python scripts/dev/r05/diag_phases.py --workload mixtral-8x7b-experts-r128 --streams 2,3 --modes base,no_ortho --steps 8 > gpurun_out/r05l_diag_mx.log 2>&1
echo "diag rc=$?"; grep '^{' gpurun_out/r05l_diag_mx.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05l_prof_mx1 -o run -- python scripts/dev/r05/diag_phases.py --workload mixtral-8x7b-experts-r128 --streams 1 --modes base --steps 2 > gpurun_out/r05l_prof_mx1.log 2>&1
echo "prof rc=$?"
