# round-6 call L: the r = 128 LDS-DMA pass A with its bf16 G in step pairs (variant gp1 =
# DION_PAGL_GPAIR=1; this tree's library = the previous kernel): parity subset on gp1, PMC traffic
# of the Mixtral step on gp1, a same-box bench A/B, and pass A's split-K block target
set -o pipefail
mkdir -p gpurun_out/r06l
export TMPDIR=/tmp
O=gpurun_out/r06l
export DION_DEV_ALLOW_LIB_PATH=1
V=$PWD/megatron-dion_amd/csrc/variants
MX="--workload mixtral-8x7b-experts-r128"
DION_LIB_PATH=$V/libdion_codec_gp1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "deferred_ef or fixed_scale" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for c in FETCH_SIZE WRITE_SIZE; do
  DION_LIB_PATH=$V/libdion_codec_gp1.so timeout -s KILL 300 rocprofv3 --pmc $c -d "$PWD/$O/pmc_gp_$c" -o run --output-format csv -- python bench.py $MX --steps 1 --warmup 1 --probe-steps 0 --no-cpu-baseline --streams 1 > $O/pmc_gp_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/pmc_gp_$c.log; exit $rc; fi
done
python scripts/pmc_traffic.py $O/pmc_gp_FETCH_SIZE $O/pmc_gp_WRITE_SIZE > $O/pmc_traffic_gp.json || exit 1
python - $O/pmc_traffic_gp.json <<'PY'
import json, sys
k = json.load(open(sys.argv[1]))["kernels"]
for n, v in k.items():
    if "efgl" in n:
        print(n, round(v["hbm_bytes_per_launch"] / 1e9, 3), "GB/launch, fetch raw", round(v["fetch_bytes_raw"] / 1e9, 3), "write", round(v["write_bytes"] / 1e9, 3))
PY
run() {  # label, lib ("" = this tree), bench args
  local label=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then
    DION_LIB_PATH=$V/$lib timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > $O/$label.log 2>&1 || return 1
  else
    timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > $O/$label.log 2>&1 || return 1
  fi
  python - "$label" $O/$label.log <<'PY'
import json, sys
line = next(l for l in open(sys.argv[2]) if l.startswith('{"metric'))
d = json.loads(line)
k = d["roofline"]["kernels"]
pa = {n[:14]: round(v["avg_launch_ms"], 4) for n, v in k.items() if "ef" in n}
print(f"{sys.argv[1]:>12s} {d['value']:8.2f} GiB/s {d['ms_per_step']:8.3f} ms  pass A {pa}")
PY
}
run mx_gp1 libdion_codec_gp1.so $MX --steps 10 --warmup 2 || exit 1
run mx_gp0 "" $MX --steps 10 --warmup 2 || exit 1
run mx_gp1_b libdion_codec_gp1.so $MX --steps 10 --warmup 2 || exit 1
run mx_gp0_b "" $MX --steps 10 --warmup 2 || exit 1
run llama "" --steps 20 --warmup 3 || exit 1
