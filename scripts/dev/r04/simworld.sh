# compute side of the W-rank schedule on one GPU (loopback collectives): N = 1 and W = 2, 4, 8
set -o pipefail
mkdir -p gpurun_out
for w in 1 2 4 8; do
  if [ $w = 1 ]; then extra=""; else extra="--simulate-world $w"; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --probe-steps 0 --no-cpu-baseline $extra > gpurun_out/r04_sim_w$w.log 2>&1 || exit 1
  tail -1 gpurun_out/r04_sim_w$w.log > gpurun_out/r04_sim_w$w.json
  python -c "import json; d=json.load(open('gpurun_out/r04_sim_w$w.json')); print('W=$w', d['value'], d['ms_per_step'])"
done
