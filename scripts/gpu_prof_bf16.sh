# kernel-trace profile of the bf16-state bench (one GPU box call)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_bf16" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --streams 1 --state-dtype bf16 > gpurun_out/prof_bf16.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 gpurun_out/prof_bf16.log | cut -c1-300
exit $rc
