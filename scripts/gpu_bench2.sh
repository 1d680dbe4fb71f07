# bench in both error-feedback schedules + single-stream profile of the default one
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_def.log 2>&1
echo "bench deferred rc=$?"
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --eager-ef > gpurun_out/bench_eager.log 2>&1
echo "bench eager rc=$?"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --streams 1 > gpurun_out/prof.log 2>&1
echo "prof rc=$?"
