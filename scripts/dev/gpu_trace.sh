# dev: kernel trace of the bench at 1 and 2 streams, gap accounting
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for S in ${STREAMS_LIST:-1 2}; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$PWD/gpurun_out/trace_s$S" -o run --output-format csv -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline --streams $S ${BENCH_ARGS:-} > gpurun_out/trace_s$S.log 2>&1
  rc=$?; echo "trace streams=$S rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/trace_s$S.log; exit $rc; fi
  f=$(find gpurun_out/trace_s$S -name "*kernel_trace.csv" | head -1)
  python scripts/dev/trace_gaps.py "$f" 0.45 > gpurun_out/trace_s$S.txt; cat gpurun_out/trace_s$S.txt | head -30
done
