# one call: the GPU suite, smoke, the default bench line, the bf16-state and Mixtral lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 1 gpurun_out/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; tail -n 1 gpurun_out/bench.log | cut -c1-300
timeout -k 10 600 python bench.py --state-dtype bf16 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_bf16.log 2>&1; echo "bf16 rc=$?"; tail -n 1 gpurun_out/bench_bf16.log | cut -c1-300
timeout -k 10 600 python bench.py --workload mixtral-8x7b-experts-r128 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_mixtral.log 2>&1; echo "mixtral rc=$?"; tail -n 1 gpurun_out/bench_mixtral.log | cut -c1-300
