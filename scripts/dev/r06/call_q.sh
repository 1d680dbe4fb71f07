# round-6 call Q: pass A's split-K block target (DION_TB_PA: 2048 default, 1024, 512) on the
# Llama set.  Fewer K chunks for qkv / proj (3 / 4 at 2048) drop their partial slabs, the slab
# reduction and the P' re-reads (~0.43 GB of the step's ~15 GB); the grid's tail is what they cost
set -o pipefail
mkdir -p gpurun_out/r06q
export TMPDIR=/tmp
O=gpurun_out/r06q
export DION_DEV_ALLOW_LIB_PATH=1
V=$PWD/megatron-dion_amd/csrc/variants
DION_LIB_PATH=$V/libdion_codec_tbpa512.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "deferred_ef" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
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
print(f"{sys.argv[1]:>12s} {d['value']:8.2f} GiB/s {d['ms_per_step']:8.3f} ms  pass A {pa}")
PY
}
run tb2048 "" --steps 20 --warmup 3 || exit 1
run tb1024 libdion_codec_tbpa1024.so --steps 20 --warmup 3 || exit 1
run tb512 libdion_codec_tbpa512.so --steps 20 --warmup 3 || exit 1
run tb2048_b "" --steps 20 --warmup 3 || exit 1
run tb1024_b libdion_codec_tbpa1024.so --steps 20 --warmup 3 || exit 1
run tb512_b libdion_codec_tbpa512.so --steps 20 --warmup 3 || exit 1
run tb2048_c "" --steps 20 --warmup 3 || exit 1
