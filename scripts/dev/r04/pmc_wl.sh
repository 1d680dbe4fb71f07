# PMC HBM traffic (FETCH_SIZE, WRITE_SIZE: separate passes) of one single-stream bench step of a
# workload: WL=<workload> TAG=<name> EXTRA="<bench args>" bash scripts/dev/r04/pmc_wl.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD="python bench.py --workload ${WL:-llama3-8b-2d-grad-set-r64} --steps 1 --warmup 1 --probe-steps 0 --no-cpu-baseline --streams 1 $EXTRA"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d "$PWD/gpurun_out/pmc_${TAG}_$c" -o run --output-format csv -- $CMD > gpurun_out/pmc_${TAG}_$c.log 2>&1
  rc=$?; echo "pmc $TAG $c rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
python scripts/pmc_traffic.py gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE > gpurun_out/pmc_traffic_$TAG.json
