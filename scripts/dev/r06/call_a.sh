# round-6 call A: baseline of the round-5 tree on this box (probe with a single-stream warm-up
# step), single-stream rocprofv3 kernel stats of the Llama and Mixtral steps, the W = 8 schedule
# simulated on one GPU for both workloads, and the --gpus 2 gloo rehearsal of the child launcher
set -o pipefail
mkdir -p gpurun_out/r06a
export TMPDIR=/tmp
O=gpurun_out/r06a
line() { grep '^{"metric' "$1" > "$2" && python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['step']['frac'] if 'step' in r else '')" "$2"; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_llama.log 2>&1 || exit 1
line $O/bench_llama.log $O/bench_llama.json || exit 1
timeout -k 10 300 python bench.py --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_mixtral.log 2>&1 || exit 1
line $O/bench_mixtral.log $O/bench_mixtral.json || exit 1
timeout -k 10 300 python bench.py --simulate-world 8 --steps 20 --warmup 3 --no-cpu-baseline > $O/sim8_llama.log 2>&1 || exit 1
line $O/sim8_llama.log $O/sim8_llama.json || exit 1
timeout -k 10 300 python bench.py --simulate-world 8 --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 --no-cpu-baseline > $O/sim8_mixtral.log 2>&1 || exit 1
line $O/sim8_mixtral.log $O/sim8_mixtral.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_llama1 -o run -- python bench.py --streams 1 --steps 3 --warmup 2 --no-cpu-baseline > $O/prof_llama1.log 2>&1 || exit 1
echo "prof llama rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mx1 -o run -- python bench.py --workload mixtral-8x7b-experts-r128 --streams 1 --steps 3 --warmup 2 --no-cpu-baseline > $O/prof_mx1.log 2>&1 || exit 1
echo "prof mixtral rc=$?"
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --layers 4 --steps 3 --warmup 1 > $O/gloo2.log 2>&1 || exit 1
line $O/gloo2.log $O/gloo2.json
