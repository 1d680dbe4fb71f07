# kernel trace of the bench (2 streams): time without a streaming kernel, by cause
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$PWD/gpurun_out/trace_s2" -o run --output-format csv -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/trace_s2.log 2>&1
rc=$?; echo "trace rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/trace_s2.log; exit $rc; fi
f=$(find gpurun_out/trace_s2 -name "*kernel_trace.csv" | head -1)
python scripts/dev/trace_uncovered.py "$f" 0.45 | tee gpurun_out/trace_uncovered.txt
cp "$f" gpurun_out/trace_s2_kernels.csv
