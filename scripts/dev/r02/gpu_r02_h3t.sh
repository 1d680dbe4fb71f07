# one GPU box call: the transposed-h3 change -- the parity tests that touch it, the gpu
export DION_DEV_ALLOW_LIB_PATH=1
# suite, then the Llama bench A/B against the bf16x6 transposed kernels (variant x6t)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -a -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
for v in default x6t; do
  lib=""; [ "$v" != default ] && lib="DION_LIB_PATH=$PWD/megatron-dion_amd/csrc/variants/libdion_codec_$v.so"
  timeout -k 10 300 env $lib python bench.py --steps 8 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_${v}_$rep.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "[$v] rc=$rc"; tail -5 gpurun_out/ab_${v}_$rep.log; exit $rc; fi
  python - "$v" gpurun_out/ab_${v}_$rep.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(f"{sys.argv[1]:10s} {d['value']:8.2f} GiB/s  {d['ms_per_step']:8.3f} ms")
for k, v in d["roofline"]["kernels"].items():
    print(f"    {k:40s} {v['avg_launch_ms']:7.4f} ms {v['GB/s']:8.1f} GB/s")
PY
done
done
