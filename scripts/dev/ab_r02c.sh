# A/B: r = 128 pass-B kernels with the split P two cb at a time (two waves per SIMD) vs all
# RB at once (one wave per SIMD); the r = 64 kernels are unchanged (control)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
KB_R=128 OPS="pbf pbf_T" bash scripts/dev/ab_kernels.sh default nopairs || exit $?
OPS="pbf pbf_T" bash scripts/dev/ab_kernels.sh default nopairs || exit $?
timeout -k 10 600 python bench.py --workload mixtral-8x7b-experts-r128 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_mixtral.log 2>&1; echo "mixtral rc=$?"; tail -n 1 gpurun_out/bench_mixtral.log
