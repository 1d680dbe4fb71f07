# A/B of codec kernel variants on Llama-size batches: bash scripts/dev/ab_kernels.sh variant1 [variant2 ...]
export DION_DEV_ALLOW_LIB_PATH=1
# ("default" = the in-tree library); ops: pa_ef pa_ef_T pb pb_T w w_T
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = default ]; then lib=""; else lib="$PWD/megatron-dion_amd/csrc/variants/libdion_codec_$v.so"; fi
  for op in ${OPS:-pa_ef pa_ef_T pb pb_T w w_T}; do
    DION_LIB_PATH=$lib timeout -k 10 120 python scripts/dev/kbench.py $op 5 > gpurun_out/ab_${v}_$op.log 2>&1
    rc=$?
    echo "$v $op rc=$rc $(tail -1 gpurun_out/ab_${v}_$op.log)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
