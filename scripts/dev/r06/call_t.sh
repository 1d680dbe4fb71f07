# round-6 call T: PMC HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the final tree's
# Llama step (pass A's split-K target is now 1024), then the driver's default bench command
set -o pipefail
mkdir -p gpurun_out/r06t
export TMPDIR=/tmp
O=gpurun_out/r06t
wl=llama3-8b-2d-grad-set-r64
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c -d "$PWD/$O/pmc_${wl}_$c" -o run --output-format csv -- python bench.py --workload $wl --steps 1 --warmup 1 --probe-steps 0 --no-cpu-baseline --streams 1 > $O/pmc_${wl}_$c.log 2>&1
  rc=$?; echo "pmc $wl $c rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/pmc_${wl}_$c.log; exit $rc; fi
done
python scripts/pmc_traffic.py $O/pmc_${wl}_FETCH_SIZE $O/pmc_${wl}_WRITE_SIZE > $O/pmc_traffic_$wl.json || exit 1
timeout -k 10 600 python bench.py > $O/bench_llama.log 2>&1 || exit 1
grep '^{"metric' $O/bench_llama.log > $O/bench_llama.json && python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['step']['frac'], r.get('traffic'))" $O/bench_llama.json
