# round-4 LDS-DMA r = 128 pass A: the whole GPU suite, the Mixtral bench line, the probe/rocprof
# reconciliation of the Mixtral line (single stream)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r04g_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -a -E "passed|failed" gpurun_out/r04g_pytest_gpu.log | tail -3
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r04g_bench_mixtral.log 2>&1 || exit 1
grep '^{"metric' gpurun_out/r04g_bench_mixtral.log | cut -c1-200
TAG=mixtral_gl bash scripts/dev/r04/recon.sh
bash scripts/dev/r04/probe_ab.sh "--workload mixtral-8x7b-experts-r128 --steps 4 --warmup 2" glc ef3
