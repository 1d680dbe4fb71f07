# one GPU box call: the round's committed profiles
#  (1) rocprofv3 --kernel-trace --stats of the bench on one stream (the roofline probe's
#      configuration, so the per-kernel averages compare with the bench's HIP-event probe)
#  (2) HBM traffic per kernel: FETCH_SIZE and WRITE_SIZE passes (scripts/gpu_pmc.sh)
#  (3) SQ issue / MFMA-busy counters of the streaming kernels (scripts/gpu_pmc_sq.sh)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --streams 1 > gpurun_out/prof.log 2>&1
rc=$?; echo "stats rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/prof.log; exit $rc; fi
find gpurun_out/prof -name "*kernel_trace.csv" -delete  # per-launch rows: large, the stats keep the summary
bash scripts/gpu_pmc.sh || exit $?
OPS="${OPS:-pa_ef pa_ef_T pbf pb_T w w_T}" bash scripts/gpu_pmc_sq.sh || exit $?
