# PMC counter groups for one kbench op:  bash scripts/dev/pmc_kernel.sh <op>
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
OP=$1
timeout -k 10 120 python scripts/dev/kbench.py $OP 5 > gpurun_out/kb_$OP.log 2>&1 || exit $?
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM" \
           "GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"; do
  timeout -k 10 300 rocprofv3 --pmc $grp -d "$PWD/gpurun_out/pmc_${OP}_$i" -o run --output-format csv -- python scripts/dev/kbench.py $OP 2 > gpurun_out/pmc_${OP}_$i.log 2>&1
  rc=$?; echo "pmc $OP group $i rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  i=$((i+1))
done
