# A/B of round-2 knobs (kbench, Llama-size batches): waves per block of the pass-B row kernel,
# the LDS transpose swizzle (+ its LDS counters on pass A); the Mixtral r = 128 bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
OPS="pa_ef pbf_T" bash scripts/dev/ab_kernels.sh default pbrnw8 swz5 || exit $?
VARIANT=swz5 OPS="pa_ef" bash scripts/dev/pmc_variant.sh || exit $?
timeout -k 10 600 python bench.py --workload mixtral-8x7b-experts-r128 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_mixtral.log 2>&1; echo "mixtral rc=$?"; tail -n 1 gpurun_out/bench_mixtral.log
