# round-6 call J2: the final tree's bench lines (the driver's default command with cpu_baseline;
# Mixtral r = 128; bf16 state), single-stream rocprofv3 kernel stats of the Llama and Mixtral
# steps, W = 8 simulated on the replicated pipeline for both workloads, and the --gpus 2 gloo
# rehearsal (child launcher, replicated pipeline over real collectives)
set -o pipefail
mkdir -p gpurun_out/r06j
export TMPDIR=/tmp
O=gpurun_out/r06j
line() { grep '^{"metric' "$1" > "$2" && python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['step']['frac'] if 'step' in r else '')" "$2"; }
timeout -k 10 600 python bench.py > $O/bench_llama.log 2>&1 || exit 1
line $O/bench_llama.log $O/bench_llama.json || exit 1
timeout -k 10 300 python bench.py --workload mixtral-8x7b-experts-r128 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_mixtral.log 2>&1 || exit 1
line $O/bench_mixtral.log $O/bench_mixtral.json || exit 1
timeout -k 10 300 python bench.py --state-dtype bf16 --no-cpu-baseline > $O/bench_bf16.log 2>&1 || exit 1
line $O/bench_bf16.log $O/bench_bf16.json || exit 1
timeout -k 10 300 python bench.py --simulate-world 8 --steps 20 --warmup 3 --no-cpu-baseline > $O/sim8_llama.log 2>&1 || exit 1
line $O/sim8_llama.log $O/sim8_llama.json || exit 1
timeout -k 10 300 python bench.py --workload mixtral-8x7b-experts-r128 --simulate-world 8 --steps 20 --warmup 3 --no-cpu-baseline > $O/sim8_mixtral.log 2>&1 || exit 1
line $O/sim8_mixtral.log $O/sim8_mixtral.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_llama1 -o run -- python bench.py --streams 1 --no-cpu-baseline --steps 3 --warmup 2 > $O/prof_llama1.log 2>&1 || exit 1
echo "prof llama ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mx1 -o run -- python bench.py --workload mixtral-8x7b-experts-r128 --streams 1 --no-cpu-baseline --steps 3 --warmup 2 > $O/prof_mx1.log 2>&1 || exit 1
echo "prof mixtral ok"
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --layers 4 --steps 3 --warmup 1 > $O/gloo2.log 2>&1 || exit 1
line $O/gloo2.log $O/gloo2.json
