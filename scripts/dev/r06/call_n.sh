# round-6 call N: the LDS-DMA pass A (rowproj_efgl / colproj_efgl, with G in step pairs) at r = 64
# (variants gl64r: row kernel only, gl64: both orientations) against this tree's register kernels
# on the Llama set; parity subset on gl64 first
set -o pipefail
mkdir -p gpurun_out/r06n
export TMPDIR=/tmp
O=gpurun_out/r06n
export DION_DEV_ALLOW_LIB_PATH=1
V=$PWD/megatron-dion_amd/csrc/variants
DION_LIB_PATH=$V/libdion_codec_gl64.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "deferred_ef or fixed_scale" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
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
print(f"{sys.argv[1]:>10s} {d['value']:8.2f} GiB/s {d['ms_per_step']:8.3f} ms  pass A {pa}")
PY
}
run def "" --steps 20 --warmup 3 || exit 1
run gl64r libdion_codec_gl64r.so --steps 20 --warmup 3 || exit 1
run gl64 libdion_codec_gl64.so --steps 20 --warmup 3 || exit 1
run def_b "" --steps 20 --warmup 3 || exit 1
run gl64r_b libdion_codec_gl64r.so --steps 20 --warmup 3 || exit 1
run gl64_b libdion_codec_gl64.so --steps 20 --warmup 3 || exit 1
