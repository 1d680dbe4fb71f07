# kernel-trace profile of the bench (one GPU box call)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --streams ${STREAMS:-2} > gpurun_out/prof.log 2>&1
echo "prof rc=$?"
