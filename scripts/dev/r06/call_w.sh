# round-6 call W: the exact final tree (build options added since call S are off by default):
# GPU suite, smoke, the driver's default bench command
set -o pipefail
mkdir -p gpurun_out/r06w
export TMPDIR=/tmp
O=gpurun_out/r06w
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider --durations=5 > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > $O/bench_llama.log 2>&1 || exit 1
grep '^{"metric' $O/bench_llama.log > $O/bench_llama.json && python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['step']['frac'], r.get('traffic'))" $O/bench_llama.json
