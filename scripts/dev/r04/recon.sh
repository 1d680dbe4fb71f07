# probe vs rocprof reconciliation: one single-stream bench under the kernel trace, the bench's
# own probe in the same process (WL = workload, default Mixtral r = 128)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
WL=${WL:-mixtral-8x7b-experts-r128}
TAG=${TAG:-mixtral}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/r04_recon_$TAG" -o run --output-format csv -- python bench.py --workload $WL --steps 2 --warmup 1 --probe-steps 2 --no-cpu-baseline --streams 1 $EXTRA > gpurun_out/r04_recon_$TAG.log 2>&1
echo "recon rc=$?"
grep "^{\"metric" gpurun_out/r04_recon_$TAG.log | tail -1 > gpurun_out/r04_recon_$TAG.json
python scripts/dev/r04/recon.py gpurun_out/r04_recon_$TAG.json gpurun_out/r04_recon_$TAG/run_kernel_trace.csv
