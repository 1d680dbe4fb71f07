# HBM traffic of every kernel from PMC counters (one GPU box call).
# FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950 (MI355X_MICROARCH.md,
# "rocprofv3 PMC slots"), so each gets its own run; counters are collected with
# nothing but the counter pass itself (no sys/runtime trace).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD="python bench.py --steps 1 --warmup 1 --probe-steps 0 --no-cpu-baseline --streams 1"
timeout -k 10 300 rocprofv3 -L > gpurun_out/pmc_counters.txt 2>&1 || true
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c -d "$PWD/gpurun_out/pmc_$c" -o run --output-format csv -- $CMD > gpurun_out/pmc_$c.log 2>&1
  rc=$?
  echo "pmc $c rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python scripts/pmc_traffic.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE > gpurun_out/pmc_traffic.json
echo "traffic rc=$?"
