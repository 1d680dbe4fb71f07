# one GPU box call: the N = 2 bench launch rehearsed over gloo on one GPU, then a
# single-stream rocprofv3 kernel trace of the default bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --gpus 2 --backend gloo --layers ${GLOO_LAYERS:-4} --steps 3 --warmup 1 > gpurun_out/bench_gloo2.log 2>&1
rc=$?; echo "gloo bench rc=$rc"; grep -a '"metric"' gpurun_out/bench_gloo2.log | tail -1
if [ $rc -ne 0 ]; then tail -20 gpurun_out/bench_gloo2.log; exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --streams 1 > gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 gpurun_out/prof.log
exit $rc
