# A/B: pass A row kernel 3-deep pipeline (bf16 G), pass-B row kernel at 3 blocks per CU
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
OPS="pa_ef pbf_T" bash scripts/dev/ab_kernels.sh default pd3 pbr3 default || exit $?
