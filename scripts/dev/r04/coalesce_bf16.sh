# bf16-state bench at launch groups of 8 / 16 / 24 / 32 matrices (one box, two rounds)
set -o pipefail
mkdir -p gpurun_out
for rnd in 1 2; do
  for c in 16 24 32 8; do
    timeout -k 10 300 python bench.py --state-dtype bf16 --steps 20 --warmup 3 --no-cpu-baseline --probe-steps 0 --coalesce $c > gpurun_out/r04_coal_$c.log 2>&1 || exit 1
    echo "$rnd coalesce $c $(grep '^{"metric' gpurun_out/r04_coal_$c.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
