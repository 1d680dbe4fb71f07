# Mixtral r = 128: one vs two vs three streams, lookahead, coalesce (one box, two rounds)
set -o pipefail
mkdir -p gpurun_out
for rnd in 1 2; do
  for v in "--streams 2" "--streams 1" "--streams 3" "--streams 2 --coalesce 8" "--streams 2 --coalesce 32"; do
    tag=$(echo "$v" | tr -d ' -')
    timeout -k 10 300 python bench.py --workload mixtral-8x7b-experts-r128 --steps 6 --warmup 2 --no-cpu-baseline --probe-steps 0 $v > gpurun_out/r04_mx_$tag.log 2>&1 || exit 1
    echo "$rnd [$v] $(grep '^{"metric' gpurun_out/r04_mx_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
