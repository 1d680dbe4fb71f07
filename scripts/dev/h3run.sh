# dev: accuracy (vs fp64) and speed of pass-B variants
export DION_DEV_ALLOW_LIB_PATH=1
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-default pbh3}; do
  if [ "$v" = default ]; then lib=""; else lib="$PWD/megatron-dion_amd/csrc/variants/libdion_codec_$v.so"; fi
  echo "== $v"
  DION_LIB_PATH=$lib timeout -k 10 120 python scripts/dev/proj_check.py ${CHECK_OP:-pb} 28672 4096 64 2 2>&1 | tail -1
  for op in ${OPS:-pb}; do DION_LIB_PATH=$lib timeout -k 10 120 python scripts/dev/kbench.py $op 5 2>&1 | tail -1; done
done
