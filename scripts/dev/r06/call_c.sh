# round-6 call C: transposed pass B on LDS-DMA staging (rowproj_h3gl_kernel): parity subset,
# then same-box A/B of the staging depth / block width against the round-5 register kernel
set -o pipefail
mkdir -p gpurun_out/r06c
export TMPDIR=/tmp
O=gpurun_out/r06c
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused_tail.py tests/test_gpu_fullsize.py tests/test_gpu_fs.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "pass_b or fused_tail or project_r_fixup or config3 or config5 or f6 or f7 or twelve" > $O/pytest.log 2>&1
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
pb = [v for n, v in k.items() if n.startswith("rowproj_h3")]
print(f"{sys.argv[1]:>10s} {d['value']:8.2f} GiB/s {d['ms_per_step']:8.3f} ms  pass-B-T {pb[0]['avg_launch_ms'] if pb else 0:.4f} ms {pb[0]['GB/s'] if pb else 0:.0f} GB/s")
PY
}
run gl0_a libdion_codec_gl0.so --steps 20 --warmup 3 || exit 1
run d3_a "" --steps 20 --warmup 3 || exit 1
run d2 libdion_codec_d2.so --steps 20 --warmup 3 || exit 1
run d4 libdion_codec_d4.so --steps 20 --warmup 3 || exit 1
run nw4 libdion_codec_nw4.so --steps 20 --warmup 3 || exit 1
run gl0_b libdion_codec_gl0.so --steps 20 --warmup 3 || exit 1
run d3_b "" --steps 20 --warmup 3 || exit 1
run mx_gl0 libdion_codec_gl0.so --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
run mx_d3 "" --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
