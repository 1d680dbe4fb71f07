# kernel trace of the default two-stream Mixtral step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$PWD/gpurun_out/r04_trace_mx" -o run --output-format csv -- python bench.py --workload mixtral-8x7b-experts-r128 --steps 3 --warmup 1 --probe-steps 0 --no-cpu-baseline > gpurun_out/r04_trace_mx.log 2>&1
echo "trace rc=$?"
