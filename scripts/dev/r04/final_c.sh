# round-4 closing call C (after the r = 128 LDS-DMA pass A): the whole GPU suite, smoke, the three
# bench lines, and the Mixtral probe/rocprof reconciliation
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r04c_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -a -E "passed|failed" gpurun_out/r04c_pytest_gpu.log | tail -3
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04c_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r04c_smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > gpurun_out/r04c_bench.log 2>&1 || exit 1
grep '^{"metric' gpurun_out/r04c_bench.log | cut -c1-160
timeout -k 10 300 python bench.py --state-dtype bf16 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04c_bench_bf16.log 2>&1 || exit 1
grep '^{"metric' gpurun_out/r04c_bench_bf16.log | cut -c1-160
timeout -k 10 300 python bench.py --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r04c_bench_mixtral.log 2>&1 || exit 1
grep '^{"metric' gpurun_out/r04c_bench_mixtral.log | cut -c1-160
TAG=mixtral_c bash scripts/dev/r04/recon.sh
