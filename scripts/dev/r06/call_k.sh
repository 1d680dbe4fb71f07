# round-6 call K: the r = 128 LDS-DMA pass A's 1.12x HBM traffic (Mixtral).  A/B of its bf16 G
# loads under the nt policy (DION_PAGL_GNT=1, variant pagnt) by PMC FETCH_SIZE / WRITE_SIZE and
# the Mixtral bench; the HBM ceiling of pass A's traffic mix on this box (scripts/ubench/hbm_mix)
set -o pipefail
mkdir -p gpurun_out/r06k
export TMPDIR=/tmp
O=gpurun_out/r06k
export DION_DEV_ALLOW_LIB_PATH=1
MX="--workload mixtral-8x7b-experts-r128"
timeout -k 10 120 ./scripts/ubench/hbm_mix > $O/hbm_mix.txt 2>&1 || exit 1
grep best $O/hbm_mix.txt
pmc() {  # label, lib ("" = this tree)
  local label=$1 lib=$2
  for c in FETCH_SIZE WRITE_SIZE; do
    if [ -n "$lib" ]; then export DION_LIB_PATH=$PWD/megatron-dion_amd/csrc/variants/$lib; else unset DION_LIB_PATH; fi
    timeout -s KILL 300 rocprofv3 --pmc $c -d "$PWD/$O/pmc_${label}_$c" -o run --output-format csv -- python bench.py $MX --steps 1 --warmup 1 --probe-steps 0 --no-cpu-baseline --streams 1 > $O/pmc_${label}_$c.log 2>&1
    rc=$?; echo "pmc $label $c rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/pmc_${label}_$c.log; exit $rc; fi
  done
  unset DION_LIB_PATH
  python scripts/pmc_traffic.py $O/pmc_${label}_FETCH_SIZE $O/pmc_${label}_WRITE_SIZE > $O/pmc_traffic_$label.json || exit 1
  python - $O/pmc_traffic_$label.json <<'PY'
import json, sys
k = json.load(open(sys.argv[1]))["kernels"]
for n, v in k.items():
    if "efgl" in n:
        print(sys.argv[1], n, round(v["hbm_bytes_per_launch"] / 1e9, 3), "GB/launch, fetch raw", round(v["fetch_bytes_raw"] / 1e9, 3), "write", round(v["write_bytes"] / 1e9, 3))
PY
}
pmc def "" || exit 1
pmc pagnt libdion_codec_pagnt.so || exit 1
run() {  # label, lib ("" = this tree), bench args
  local label=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then
    DION_LIB_PATH=$PWD/megatron-dion_amd/csrc/variants/$lib timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > $O/$label.log 2>&1 || return 1
  else
    timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > $O/$label.log 2>&1 || return 1
  fi
  python - "$label" $O/$label.log <<'PY'
import json, sys
line = next(l for l in open(sys.argv[2]) if l.startswith('{"metric'))
d = json.loads(line)
k = d["roofline"]["kernels"]
pa = {n[:14]: round(v["avg_launch_ms"], 4) for n, v in k.items() if "ef" in n}
print(f"{sys.argv[1]:>10s} {d['value']:8.2f} GiB/s {d['ms_per_step']:8.3f} ms  pass A {pa}")
PY
}
run mx_def "" $MX --steps 10 --warmup 2 || exit 1
run mx_pagnt libdion_codec_pagnt.so $MX --steps 10 --warmup 2 || exit 1
run mx_def2 "" $MX --steps 10 --warmup 2 || exit 1
run mx_pagnt2 libdion_codec_pagnt.so $MX --steps 10 --warmup 2 || exit 1
