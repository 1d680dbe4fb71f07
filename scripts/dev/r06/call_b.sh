# round-6 call B: the GPU suite on the W > 1 fused tail (dion_pfix_split, ABI 16; r = 128 split
# after the last solve) with the new fused-tail and config-5 W = 4/8 tests, then the Llama and
# Mixtral lines of this tree
set -o pipefail
mkdir -p gpurun_out/r06b
export TMPDIR=/tmp
O=gpurun_out/r06b
line() { grep '^{"metric' "$1" > "$2" && python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['step']['frac'] if 'step' in r else '')" "$2"; }
timeout -k 10 240 python -u -m pytest tests/test_gpu_fused_tail.py tests/test_gpu_configs.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "fused_tail or config5 or config4" > $O/pytest_new.log 2>&1
rc=$?; echo "pytest new rc=$rc"; tail -3 $O/pytest_new.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider --durations=10 > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_llama.log 2>&1 || exit 1
line $O/bench_llama.log $O/bench_llama.json || exit 1
timeout -k 10 300 python bench.py --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_mixtral.log 2>&1 || exit 1
line $O/bench_mixtral.log $O/bench_mixtral.json || exit 1
