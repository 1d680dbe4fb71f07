# elementwise GPU parity (incl. the mixed moment-dtype cases); A/B: split-operand staging loads
# issued before the big operand's prefetch (sf1)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_elementwise.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_ew.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_ew.log; if [ $rc -ne 0 ]; then exit $rc; fi
OPS="pa_ef pa_ef_T pbf pbf_T" bash scripts/dev/ab_kernels.sh default sf1 default sf1 || exit $?
KB_R=128 OPS="pa_ef pa_ef_T pbf pbf_T" bash scripts/dev/ab_kernels.sh default sf1 || exit $?
