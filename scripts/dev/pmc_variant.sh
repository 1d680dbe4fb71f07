# dev: SQ counter groups of one kbench op for a library variant: VARIANT=name OPS="pb pb_T" bash scripts/dev/pmc_variant.sh
export DION_DEV_ALLOW_LIB_PATH=1
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$VARIANT" ] && [ "$VARIANT" != default ]; then export DION_LIB_PATH=$PWD/megatron-dion_amd/csrc/variants/libdion_codec_$VARIANT.so; fi
for OP in ${OPS:-pb}; do
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
             "SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
             "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    timeout -s KILL 120 rocprofv3 --pmc $grp -d "$PWD/gpurun_out/pmcsq_${OP}_$i" -o run --output-format csv -- python scripts/dev/kbench.py $OP 2 > gpurun_out/pmcsq_${OP}_$i.log 2>&1
    rc=$?; echo "pmc $OP group $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmcsq_${OP}_$i.log; exit $rc; fi
    i=$((i+1))
  done
done
python scripts/pmc_sq_summary.py gpurun_out > gpurun_out/pmc_sq_variant.json
