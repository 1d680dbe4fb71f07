# final round-3 tree: the whole GPU suite, smoke, the default bench line, the Mixtral and bf16-state lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > gpurun_out/final_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -a -E "passed|failed|FAILED|Error" gpurun_out/final_pytest_gpu.log | tail -5
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/final_smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/final_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/final_bench.log | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --no-cpu-baseline --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 3 > gpurun_out/final_bench_mixtral.log 2>&1
rc=$?; echo "mixtral rc=$rc"; tail -1 gpurun_out/final_bench_mixtral.log | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --no-cpu-baseline --state-dtype bf16 --steps 20 --warmup 3 > gpurun_out/final_bench_bf16.log 2>&1
rc=$?; echo "bf16 rc=$rc"; tail -1 gpurun_out/final_bench_bf16.log | cut -c1-200; exit $rc
