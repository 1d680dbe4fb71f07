# round-5 call C: CU-masked latency stream experiment; single-stream rocprof of HEAD (LDS trsm)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python scripts/dev/r05/diag_cumask.py > gpurun_out/r05c_cumask.log 2>&1
echo "cumask rc=$?"; grep '^{' gpurun_out/r05c_cumask.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/r05c_prof" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --probe-steps 0 --no-cpu-baseline --streams 1 > gpurun_out/r05c_prof.log 2>&1
echo "prof rc=$?"
