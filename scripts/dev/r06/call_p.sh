# round-6 call P: the update kernel (rank_stream_kernel) with its tile offsets' q part in the
# scalar offset (DION_RS_SOFF=1, this tree: r = 128 135 -> 120 VGPRs, two 8-wave blocks per CU;
# r = 64 158 -> 154) against the previous kernel (variant rs0): parity subset, then a same-box
# bench A/B on both workloads
set -o pipefail
mkdir -p gpurun_out/r06p
export TMPDIR=/tmp
O=gpurun_out/r06p
export DION_DEV_ALLOW_LIB_PATH=1
V=$PWD/megatron-dion_amd/csrc/variants
MX="--workload mixtral-8x7b-experts-r128"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_update_precision.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
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
up = {n[:16]: round(v["avg_launch_ms"], 4) for n, v in k.items() if "rank_stream" in n}
print(f"{sys.argv[1]:>10s} {d['value']:8.2f} GiB/s {d['ms_per_step']:8.3f} ms  update {up}")
PY
}
run mx "" $MX --steps 10 --warmup 2 || exit 1
run mx_rs0 libdion_codec_rs0.so $MX --steps 10 --warmup 2 || exit 1
run mx_b "" $MX --steps 10 --warmup 2 || exit 1
run mx_rs0_b libdion_codec_rs0.so $MX --steps 10 --warmup 2 || exit 1
run llama "" --steps 20 --warmup 3 || exit 1
run llama_rs0 libdion_codec_rs0.so --steps 20 --warmup 3 || exit 1
run llama_b "" --steps 20 --warmup 3 || exit 1
run llama_rs0_b libdion_codec_rs0.so --steps 20 --warmup 3 || exit 1
