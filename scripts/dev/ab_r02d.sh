# weight update on h3 products (rank_stream_kernel<..., H3>) vs bf16x6: GPU suite, kbench A/B
# at r = 64 and r = 128, Llama and Mixtral bench lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu.log; if [ $rc -ne 0 ]; then exit $rc; fi
OPS="w w_T" bash scripts/dev/ab_kernels.sh default rankx6 || exit $?
KB_R=128 OPS="w w_T" bash scripts/dev/ab_kernels.sh default rankx6 || exit $?
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; tail -n 1 gpurun_out/bench.log | cut -c1-400
timeout -k 10 600 python bench.py --workload mixtral-8x7b-experts-r128 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_mixtral.log 2>&1; echo "mixtral rc=$?"; tail -n 1 gpurun_out/bench_mixtral.log | cut -c1-400
