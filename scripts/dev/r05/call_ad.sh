# round-5 call AD (the round's final tree: pipelined schedule, 512-row update blocks at r > 64): the GPU suite, smoke, the default bench line
# (with cpu_baseline), bf16-state and Mixtral lines, and a rocprofv3 kernel-stats pass of the
# default Llama command
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider --durations=15 > gpurun_out/r05ad_pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -1 gpurun_out/r05ad_pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05ad_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r05ad_smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/r05ad_bench_llama.log 2>&1 || exit 1
grep '^{"metric' gpurun_out/r05ad_bench_llama.log > gpurun_out/r05ad_bench_llama.json
python -c "import json; d=json.load(open('gpurun_out/r05ad_bench_llama.json')); print('llama', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 python bench.py --state-dtype bf16 --no-cpu-baseline > gpurun_out/r05ad_bench_bf16.log 2>&1 || exit 1
grep '^{"metric' gpurun_out/r05ad_bench_bf16.log > gpurun_out/r05ad_bench_bf16.json
python -c "import json; d=json.load(open('gpurun_out/r05ad_bench_bf16.json')); print('bf16', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 python bench.py --workload mixtral-8x7b-experts-r128 --no-cpu-baseline > gpurun_out/r05ad_bench_mixtral.log 2>&1 || exit 1
grep '^{"metric' gpurun_out/r05ad_bench_mixtral.log > gpurun_out/r05ad_bench_mixtral.json
python -c "import json; d=json.load(open('gpurun_out/r05ad_bench_mixtral.json')); print('mixtral', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05ad_prof_llama -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r05ad_prof_llama.log 2>&1
echo "prof rc=$?"
