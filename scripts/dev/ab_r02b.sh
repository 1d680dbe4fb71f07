# A/B of round-2 knobs (kbench, Llama-size batches): waves per block of the pass-B kernels and
# pass A, the LDS transpose swizzle; then the swizzle variant's LDS counters on pass A
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__" || exit 1
OPS="pa_ef pa_ef_T pbf pbf_T" bash scripts/dev/ab_kernels.sh default || exit $?
OPS="pbf" bash scripts/dev/ab_kernels.sh nw8 || exit $?
OPS="pa_ef" bash scripts/dev/ab_kernels.sh panw8 || exit $?
OPS="pbf_T" bash scripts/dev/ab_kernels.sh pbrnw8 || exit $?
OPS="pa_ef pbf_T" bash scripts/dev/ab_kernels.sh swz5 || exit $?
VARIANT=swz5 OPS="pa_ef" bash scripts/dev/pmc_variant.sh || exit $?
