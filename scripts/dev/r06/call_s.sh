# round-6 call S: closing validation of the final tree: GPU suite, smoke, the driver's default
# bench command (with cpu_baseline), Mixtral r = 128, bf16 state, simulated W = 8 (Llama), and a
# single-stream rocprofv3 kernel trace of the Llama step
set -o pipefail
mkdir -p gpurun_out/r06s
export TMPDIR=/tmp
O=gpurun_out/r06s
line() { grep '^{"metric' "$1" > "$2" && python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['step']['frac'] if 'step' in r else '')" "$2"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider --durations=10 > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > $O/bench_llama.log 2>&1 || exit 1
line $O/bench_llama.log $O/bench_llama.json || exit 1
timeout -k 10 300 python bench.py --workload mixtral-8x7b-experts-r128 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_mixtral.log 2>&1 || exit 1
line $O/bench_mixtral.log $O/bench_mixtral.json || exit 1
timeout -k 10 300 python bench.py --state-dtype bf16 --no-cpu-baseline > $O/bench_bf16.log 2>&1 || exit 1
line $O/bench_bf16.log $O/bench_bf16.json || exit 1
timeout -k 10 300 python bench.py --simulate-world 8 --steps 20 --warmup 3 --no-cpu-baseline > $O/sim8_llama.log 2>&1 || exit 1
line $O/sim8_llama.log $O/sim8_llama.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_llama1 -o run -- python bench.py --streams 1 --no-cpu-baseline --steps 3 --warmup 2 > $O/prof_llama1.log 2>&1 || exit 1
echo "prof llama ok"
