# the bf16 three-step test with the batched-reduction sketch QR (default) and the previous
export DION_DEV_ALLOW_LIB_PATH=1
# library (qrold), twice each
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in default qrold default qrold; do
  if [ $lib = default ]; then export DION_LIB_PATH=; else export DION_LIB_PATH=$PWD/megatron-dion_amd/csrc/variants/libdion_codec_$lib.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/bf16_$lib.log 2>&1
  echo "$lib rc=$? $(tail -n 1 gpurun_out/bf16_$lib.log)"; grep -o "AssertionError: .*" gpurun_out/bf16_$lib.log | head -3
done
