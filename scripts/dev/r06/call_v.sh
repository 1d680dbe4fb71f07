# round-6 call V: priority 1 for waves 4-7 of the 8-wave LDS-DMA kernels (variant prio,
# DION_GL_PRIO=1) against this tree, both workloads, two alternations
set -o pipefail
mkdir -p gpurun_out/r06v
export TMPDIR=/tmp
O=gpurun_out/r06v
export DION_DEV_ALLOW_LIB_PATH=1
V=$PWD/megatron-dion_amd/csrc/variants
MX="--workload mixtral-8x7b-experts-r128"
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
ks = {n[:14]: round(v["avg_launch_ms"], 4) for n, v in k.items() if "gl" in n}
print(f"{sys.argv[1]:>12s} {d['value']:8.2f} GiB/s {d['ms_per_step']:8.3f} ms  {ks}")
PY
}
for pass in a b; do
  run llama_$pass "" --steps 20 --warmup 3 || exit 1
  run llama_prio_$pass libdion_codec_prio.so --steps 20 --warmup 3 || exit 1
  run mx_$pass "" $MX --steps 10 --warmup 2 || exit 1
  run mx_prio_$pass libdion_codec_prio.so $MX --steps 10 --warmup 2 || exit 1
done
