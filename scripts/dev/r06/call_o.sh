# round-6 call O: PMC FETCH_SIZE / WRITE_SIZE of the r = 128 LDS-DMA pass A with G in step pairs
# (this tree) and without (variant gp0) on the same box: call L's write rise (1.036x -> 1.092x)
# was measured across boxes
set -o pipefail
mkdir -p gpurun_out/r06o
export TMPDIR=/tmp
O=gpurun_out/r06o
export DION_DEV_ALLOW_LIB_PATH=1
V=$PWD/megatron-dion_amd/csrc/variants
MX="--workload mixtral-8x7b-experts-r128"
for lab in gp1 gp0; do
  for c in FETCH_SIZE WRITE_SIZE; do
    if [ $lab = gp0 ]; then export DION_LIB_PATH=$V/libdion_codec_gp0.so; else unset DION_LIB_PATH; fi
    timeout -s KILL 300 rocprofv3 --pmc $c -d "$PWD/$O/pmc_${lab}_$c" -o run --output-format csv -- python bench.py $MX --steps 1 --warmup 1 --probe-steps 0 --no-cpu-baseline --streams 1 > $O/pmc_${lab}_$c.log 2>&1
    rc=$?; echo "pmc $lab $c rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/pmc_${lab}_$c.log; exit $rc; fi
  done
  unset DION_LIB_PATH
  python scripts/pmc_traffic.py $O/pmc_${lab}_FETCH_SIZE $O/pmc_${lab}_WRITE_SIZE > $O/pmc_traffic_$lab.json || exit 1
  python - $O/pmc_traffic_$lab.json <<'PY'
import json, sys
k = json.load(open(sys.argv[1]))["kernels"]
for n, v in k.items():
    if "efgl" in n:
        print(sys.argv[1], n, round(v["hbm_bytes_per_launch"] / 1e9, 3), "GB/launch, fetch raw", round(v["fetch_bytes_raw"] / 1e9, 3), "write", round(v["write_bytes"] / 1e9, 3))
PY
done
