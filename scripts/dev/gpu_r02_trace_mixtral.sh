# kernel trace of the Mixtral r=128 bench (2 streams): time without a streaming kernel, and
# the per-kernel totals of the timed steps
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$PWD/gpurun_out/trace_mx" -o run --output-format csv -- python bench.py --workload mixtral-8x7b-experts-r128 --steps 3 --warmup 1 --no-cpu-baseline --probe-steps 0 > gpurun_out/trace_mx.log 2>&1
rc=$?; echo "trace rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/trace_mx.log; exit $rc; fi
f=$(find gpurun_out/trace_mx -name "*kernel_trace.csv" | head -1)
python scripts/dev/trace_uncovered.py "$f" 1.0 > gpurun_out/trace_mx_uncovered.txt; cat gpurun_out/trace_mx_uncovered.txt
