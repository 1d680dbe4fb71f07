# round-6 call R: two more block-count knobs re-measured under the two-stream schedule on the
# Llama set: the r = 64 pass B's split-K target (DION_TB_PBC 512 default; 256 / 1024) and the
# update's rows per block (DION_RSL 256 default; 128 / 512)
set -o pipefail
mkdir -p gpurun_out/r06r
export TMPDIR=/tmp
O=gpurun_out/r06r
export DION_DEV_ALLOW_LIB_PATH=1
V=$PWD/megatron-dion_amd/csrc/variants
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
ks = {n[:14]: round(v["avg_launch_ms"], 4) for n, v in k.items() if "colproj_h3" in n or "rank_stream" in n}
print(f"{sys.argv[1]:>12s} {d['value']:8.2f} GiB/s {d['ms_per_step']:8.3f} ms  {ks}")
PY
}
for pass in a b; do
  run def_$pass "" --steps 20 --warmup 3 || exit 1
  run pbc256_$pass libdion_codec_pbc256.so --steps 20 --warmup 3 || exit 1
  run pbc1024_$pass libdion_codec_pbc1024.so --steps 20 --warmup 3 || exit 1
  run rsl512_$pass libdion_codec_rsl512.so --steps 20 --warmup 3 || exit 1
  run rsl128_$pass libdion_codec_rsl128.so --steps 20 --warmup 3 || exit 1
done
