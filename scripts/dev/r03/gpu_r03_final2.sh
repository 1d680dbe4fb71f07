# final tree of the round: every GPU test, smoke, and the three bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v7_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/v7_pytest_gpu.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v7_smoke.log 2>&1 || exit 1
tail -2 gpurun_out/v7_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/v7_bench.log 2>&1 || exit 1
tail -1 gpurun_out/v7_bench.log > gpurun_out/v7_bench.json
timeout -k 10 400 python bench.py --workload mixtral-8x7b-experts-r128 --no-cpu-baseline > gpurun_out/v7_bench_mixtral.log 2>&1 || exit 1
tail -1 gpurun_out/v7_bench_mixtral.log > gpurun_out/v7_bench_mixtral.json
timeout -k 10 400 python bench.py --state-dtype bf16 --no-cpu-baseline > gpurun_out/v7_bench_bf16.log 2>&1 || exit 1
tail -1 gpurun_out/v7_bench_bf16.log > gpurun_out/v7_bench_bf16_state.json
for f in gpurun_out/v7_bench.json gpurun_out/v7_bench_mixtral.json gpurun_out/v7_bench_bf16_state.json; do
  python -c "import json,sys; d=json.load(open('$f')); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['kernel'], r['frac'], ' '.join(f'{k.split(\"<\")[0]}={v[\"GB/s\"]:.0f}' for k, v in r['kernels'].items()))"
done
