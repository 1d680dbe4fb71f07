# bench A/B, alternating new / $OLD_LIB, three rounds (BENCH_ARGS picks the workload)
export DION_DEV_ALLOW_LIB_PATH=1
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
for f in new old; do
  if [ $f = old ]; then export DION_LIB_PATH=$PWD/megatron-dion_amd/csrc/variants/${OLD_LIB}; else unset DION_LIB_PATH; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/llab.log 2>&1 || exit 1
  tail -1 gpurun_out/llab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], ' '.join(f'{k.split(\"<\")[0]}={v[\"GB/s\"]:.0f}' for k, v in r['kernels'].items()))"
done
done
