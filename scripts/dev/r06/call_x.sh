# round-6 call X: within-box spread of the final tree's bench lines (the driver's default
# command three times, Mixtral twice, on one box)
set -o pipefail
mkdir -p gpurun_out/r06x
export TMPDIR=/tmp
O=gpurun_out/r06x
for i in 1 2 3; do
  timeout -k 10 600 python bench.py --no-cpu-baseline > $O/llama_$i.log 2>&1 || exit 1
  grep '^{"metric' $O/llama_$i.log > $O/llama_$i.json && python -c "import json,sys; d=json.load(open(sys.argv[1])); print('llama', sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['step']['frac'])" $O/llama_$i.json $i
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload mixtral-8x7b-experts-r128 --steps 20 --warmup 3 --no-cpu-baseline > $O/mixtral_$i.log 2>&1 || exit 1
  grep '^{"metric' $O/mixtral_$i.log > $O/mixtral_$i.json && python -c "import json,sys; d=json.load(open(sys.argv[1])); print('mixtral', sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['step']['frac'])" $O/mixtral_$i.json $i
done
