# round-5 call M: solve variants beside a streaming kernel (ubench), Cholesky block sizes; the GPU
# suite; parity of the GEMM solves (variants/lib_gemm.so: -DDION_TSOLVE_GEMM=1); same-box A/B
# (variants/lib_l.so = call L's tree vs lib_gemm); Mixtral with 2 / 3 streams; a one-stream
# Mixtral kernel profile of lib_gemm
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/ubench/trsm_conc > gpurun_out/r05m_trsm_conc.log 2>&1
echo "trsm_conc rc=$?"; cat gpurun_out/r05m_trsm_conc.log
timeout -k 10 60 ./scripts/ubench/chol_ab > gpurun_out/r05m_chol.log 2>&1
echo "chol rc=$?"; cat gpurun_out/r05m_chol.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05m_pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -2 gpurun_out/r05m_pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
export DION_DEV_ALLOW_LIB_PATH=1
DION_LIB_PATH=$PWD/variants/lib_gemm.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py -x -q -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05m_parity_gemm.log 2>&1
rc=$?; echo "parity gemm rc=$rc"; grep "P maxrel vs oracle" gpurun_out/r05m_parity_gemm.log; tail -2 gpurun_out/r05m_parity_gemm.log
run() {  # label, lib ("" = this tree), extra bench args
  local label=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then
    DION_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/r05m_$label.log 2>&1 || return 1
  else
    timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/r05m_$label.log 2>&1 || return 1
  fi
  python - "$label" gpurun_out/r05m_$label.log <<'PY'
import json, sys
line = next(l for l in open(sys.argv[2]) if l.startswith('{"metric'))
d = json.loads(line)
print(f"{sys.argv[1]:>12s} {d['value']:8.2f} {d['unit']} {d['ms_per_step']:8.3f} ms")
PY
}
for i in 1 2; do
  run l_$i variants/lib_l.so --steps 20 --warmup 3 || exit 1
  run gemm_$i variants/lib_gemm.so --steps 20 --warmup 3 || exit 1
done
run l_mx variants/lib_l.so --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
run gemm_mx variants/lib_gemm.so --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
DION_LIB_PATH=$PWD/variants/lib_gemm.so timeout -k 10 300 python scripts/dev/r05/diag_phases.py --workload mixtral-8x7b-experts-r128 --streams 2,3 --modes base,no_ortho --steps 8 > gpurun_out/r05m_diag_mx.log 2>&1
echo "diag rc=$?"; grep '^{' gpurun_out/r05m_diag_mx.log
DION_LIB_PATH=$PWD/variants/lib_gemm.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05m_prof_mx1 -o run -- python scripts/dev/r05/diag_phases.py --workload mixtral-8x7b-experts-r128 --streams 1 --modes base --steps 2 > gpurun_out/r05m_prof_mx1.log 2>&1
echo "prof rc=$?"
