# per-dispatch kernel trace of the default two-stream bench step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$PWD/gpurun_out/r04_trace2" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --probe-steps 0 --no-cpu-baseline --streams 2 > gpurun_out/r04_trace2.log 2>&1
echo "trace2 rc=$?"
