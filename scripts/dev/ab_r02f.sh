# A/B: split-operand staging loads issued before the big operand's prefetch (sf1)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
OPS="pa_ef pa_ef_T pbf pbf_T" bash scripts/dev/ab_kernels.sh default sf1 default sf1 || exit $?
KB_R=128 OPS="pa_ef pa_ef_T pbf pbf_T" bash scripts/dev/ab_kernels.sh default sf1 || exit $?
