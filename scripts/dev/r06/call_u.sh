# round-6 call U: the final tree's single-stream rocprofv3 kernel trace of the Mixtral step, and
# the SQ counters of the r = 128 LDS-DMA pass A (G in step pairs) on kbench's Mixtral fc1 batch
set -o pipefail
mkdir -p gpurun_out/r06u
export TMPDIR=/tmp
O=gpurun_out/r06u
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mx1 -o run -- python bench.py --workload mixtral-8x7b-experts-r128 --streams 1 --no-cpu-baseline --steps 3 --warmup 2 > $O/prof_mx1.log 2>&1 || exit 1
echo "prof mixtral ok"
R=128; OP=pa_ef
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  KB_R=$R timeout -s KILL 120 rocprofv3 --pmc $grp -d "$PWD/$O/pmcsq_${OP}_r${R}_$i" -o run --output-format csv -- python scripts/dev/kbench.py $OP 2 > $O/pmcsq_${OP}_r${R}_$i.log 2>&1
  rc=$?; echo "sq $OP r$R group $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/pmcsq_${OP}_r${R}_$i.log; exit $rc; fi
  i=$((i+1))
done
python scripts/pmc_sq_summary.py $O > $O/pmc_sq.json
echo "summary rc=$?"
