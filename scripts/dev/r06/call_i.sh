# round-6 call I: the new ragged-chunk test of the LDS-DMA pass-B kernels, then the split-K
# block targets of those kernels (DION_TB_PBRGL 512 / 1024 / 2048, DION_TB_PBCGL 512 / 1024)
set -o pipefail
mkdir -p gpurun_out/r06i
export TMPDIR=/tmp
O=gpurun_out/r06i
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_tail.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
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
pb = {n[:12]: round(v["avg_launch_ms"], 4) for n, v in k.items() if "proj_h3" in n}
print(f"{sys.argv[1]:>10s} {d['value']:8.2f} GiB/s {d['ms_per_step']:8.3f} ms  pass B {pb}")
PY
}
run def_a "" --steps 20 --warmup 3 || exit 1
run tbr512 libdion_codec_tbr512.so --steps 20 --warmup 3 || exit 1
run tbr2048 libdion_codec_tbr2048.so --steps 20 --warmup 3 || exit 1
run mx_def "" --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
run mx_tbr512 libdion_codec_tbr512.so --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
run mx_tbc512 libdion_codec_tbc512.so --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
run mx_tbr2048 libdion_codec_tbr2048.so --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
run def_b "" --steps 20 --warmup 3 || exit 1
