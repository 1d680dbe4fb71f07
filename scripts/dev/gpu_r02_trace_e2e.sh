# one call: kernel trace of the default bench (2 streams) with the uncovered-time accounting,
# then the end-to-end rate with host copies (scripts/e2e_pcie.py) on the current build
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$PWD/gpurun_out/trace_s2" -o run --output-format csv -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline --probe-steps 0 > gpurun_out/trace_s2.log 2>&1
rc=$?; echo "trace rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/trace_s2.log; exit $rc; fi
f=$(find gpurun_out/trace_s2 -name "*kernel_trace.csv" | head -1)
python scripts/dev/trace_uncovered.py "$f" 1.0 > gpurun_out/trace_uncovered.txt; cat gpurun_out/trace_uncovered.txt


