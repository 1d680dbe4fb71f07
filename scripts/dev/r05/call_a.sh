# round-5 call A: the whole GPU suite (new W = 4 / 8, generated-sketch full-size, 12-decade tests),
# smoke, the Llama and Mixtral bench lines, and the Mixtral PMC traffic (efgl kernels)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --durations=30 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05a_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -a -E "passed|failed" gpurun_out/r05a_pytest_gpu.log | tail -3
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05a_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r05a_smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > gpurun_out/r05a_bench.log 2>&1 || exit 1
grep '^{"metric' gpurun_out/r05a_bench.log | cut -c1-200
timeout -k 10 300 python bench.py --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r05a_bench_mixtral.log 2>&1 || exit 1
grep '^{"metric' gpurun_out/r05a_bench_mixtral.log | cut -c1-200
WL=mixtral-8x7b-experts-r128 TAG=r05a_mixtral bash scripts/dev/r04/pmc_wl.sh
