# kbench A/B: the KR-templated row pass A (default) vs the library before that change (prekr)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
OPS="pa_ef pa_ef_T pbf w" bash scripts/dev/ab_kernels.sh default prekr default prekr || exit $?
