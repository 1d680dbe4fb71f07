# round-6 call E: pass B not transposed on LDS-DMA staging (colproj_h3gl_kernel): parity subset,
# same-box A/B against the register column kernel (pbc0) and its staging variants, rocprof of the
# default Llama / Mixtral steps (single stream); the replicated pipeline (W > 1 on the N = 1 stream
# schedule) simulated at W = 8 beside this box's N = 1 line
set -o pipefail
mkdir -p gpurun_out/r06e
export TMPDIR=/tmp
O=gpurun_out/r06e
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused_tail.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "pass_b or fused_tail or project_r_fixup or config3 or config4 or config5 or twelve or explicit_sketch or replicated_pipeline" > $O/pytest.log 2>&1
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
pb = [v for n, v in k.items() if n.startswith("colproj_h3")]
print(f"{sys.argv[1]:>10s} {d['value']:8.2f} GiB/s {d['ms_per_step']:8.3f} ms  pass-B {pb[0]['avg_launch_ms'] if pb else 0:.4f} ms {pb[0]['GB/s'] if pb else 0:.0f} GB/s")
PY
}
run pbc0_a libdion_codec_pbc0.so --steps 20 --warmup 3 || exit 1
run def_a "" --steps 20 --warmup 3 || exit 1
run pbcd2 libdion_codec_pbcd2.so --steps 20 --warmup 3 || exit 1
run pbcd4 libdion_codec_pbcd4.so --steps 20 --warmup 3 || exit 1
run pbcct4 libdion_codec_pbcct4.so --steps 20 --warmup 3 || exit 1
run pbc0_b libdion_codec_pbc0.so --steps 20 --warmup 3 || exit 1
run def_b "" --steps 20 --warmup 3 || exit 1
run mx_pbc0 libdion_codec_pbc0.so --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
run mx_def "" --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
unset DION_DEV_ALLOW_LIB_PATH
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_llama -o run -- python bench.py --streams 1 --no-cpu-baseline --steps 3 --warmup 2 > $O/prof_llama.log 2>&1 || exit 1
echo "prof llama ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mx -o run -- python bench.py --workload mixtral-8x7b-experts-r128 --streams 1 --no-cpu-baseline --steps 3 --warmup 2 > $O/prof_mx.log 2>&1 || exit 1
echo "prof mixtral ok"
line() { grep '^{"metric' "$1" > "$2" && python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['step']['frac'] if 'step' in r else '')" "$2"; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/n1_llama.log 2>&1 || exit 1
line $O/n1_llama.log $O/n1_llama.json || exit 1
timeout -k 10 300 python bench.py --simulate-world 8 --steps 20 --warmup 3 --no-cpu-baseline > $O/sim8_llama.log 2>&1 || exit 1
line $O/sim8_llama.log $O/sim8_llama.json || exit 1
