# kbench A/B: fused pass A with 2-wave blocks (4 blocks per CU) vs 4-wave blocks
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
OPS="pa_ef" bash scripts/dev/ab_kernels.sh default panw2 default panw2 || exit $?
KB_R=128 OPS="pa_ef" bash scripts/dev/ab_kernels.sh default panw2 || exit $?
