# round-5 call N: the GPU suite with the GEMM solves on (tri_inv_kernel inverses, chol 512
# threads at r = 64); same-box A/B against call M's GEMM variant (inverses from the factor
# kernels); one-stream kernel profiles of the Llama and Mixtral steps
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05n_pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -2 gpurun_out/r05n_pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
export DION_DEV_ALLOW_LIB_PATH=1
run() {  # label, lib ("" = this tree), extra bench args
  local label=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then
    DION_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/r05n_$label.log 2>&1 || return 1
  else
    timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/r05n_$label.log 2>&1 || return 1
  fi
  python - "$label" gpurun_out/r05n_$label.log <<'PY'
import json, sys
line = next(l for l in open(sys.argv[2]) if l.startswith('{"metric'))
d = json.loads(line)
print(f"{sys.argv[1]:>12s} {d['value']:8.2f} {d['unit']} {d['ms_per_step']:8.3f} ms")
PY
}
run m_1 variants/lib_gemm.so --steps 20 --warmup 3 || exit 1
run new_1 "" --steps 20 --warmup 3 || exit 1
run m_mx variants/lib_gemm.so --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
run new_mx "" --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05n_prof_llama1 -o run -- python scripts/dev/r05/diag_phases.py --streams 1 --modes base --steps 2 > gpurun_out/r05n_prof_llama1.log 2>&1
echo "prof llama rc=$?"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05n_prof_mx1 -o run -- python scripts/dev/r05/diag_phases.py --workload mixtral-8x7b-experts-r128 --streams 1 --modes base --steps 2 > gpurun_out/r05n_prof_mx1.log 2>&1
echo "prof mx rc=$?"
