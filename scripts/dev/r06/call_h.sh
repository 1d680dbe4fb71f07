# round-6 call H: the r <= 64 pass-A row kernel with 16-row waves (KR 1: 122 VGPRs, four waves
# per SIMD) against the default (KR 2, 166 VGPRs, three per SIMD): parity subset on the default
# build first, then same-box bench A/B
set -o pipefail
mkdir -p gpurun_out/r06h
export TMPDIR=/tmp
O=gpurun_out/r06h
export DION_DEV_ALLOW_LIB_PATH=1
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
pa = [v for n, v in k.items() if n.startswith("rowproj_efh3")]
print(f"{sys.argv[1]:>10s} {d['value']:8.2f} GiB/s {d['ms_per_step']:8.3f} ms  pass-A {pa[0]['avg_launch_ms'] if pa else 0:.4f} ms {pa[0]['GB/s'] if pa else 0:.0f} GB/s")
PY
}
run def_a "" --steps 20 --warmup 3 || exit 1
run kr1m4_a libdion_codec_pakr1m4.so --steps 20 --warmup 3 || exit 1
run kr1m3 libdion_codec_pakr1m3.so --steps 20 --warmup 3 || exit 1
run kr1nw8 libdion_codec_pakr1nw8.so --steps 20 --warmup 3 || exit 1
run def_b "" --steps 20 --warmup 3 || exit 1
run kr1m4_b libdion_codec_pakr1m4.so --steps 20 --warmup 3 || exit 1
