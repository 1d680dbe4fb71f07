# per-dispatch kernel trace of the bench (single stream and the default two), round 4 baseline
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04_base_bench.log 2>&1 || exit 1
tail -1 gpurun_out/r04_base_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/r04_trace1" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --probe-steps 0 --no-cpu-baseline --streams 1 > gpurun_out/r04_trace1.log 2>&1
echo "trace1 rc=$?"
