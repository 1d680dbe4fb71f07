# round-6 call F: PMC HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the final kernels
# on the Llama and Mixtral steps, and SQ counters of the LDS-DMA pass-B kernels
set -o pipefail
mkdir -p gpurun_out/r06f
export TMPDIR=/tmp
O=gpurun_out/r06f
for wl in llama3-8b-2d-grad-set-r64 mixtral-8x7b-experts-r128; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c -d "$PWD/$O/pmc_${wl}_$c" -o run --output-format csv -- python bench.py --workload $wl --steps 1 --warmup 1 --probe-steps 0 --no-cpu-baseline --streams 1 > $O/pmc_${wl}_$c.log 2>&1
    rc=$?; echo "pmc $wl $c rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/pmc_${wl}_$c.log; exit $rc; fi
  done
  python scripts/pmc_traffic.py $O/pmc_${wl}_FETCH_SIZE $O/pmc_${wl}_WRITE_SIZE > $O/pmc_traffic_$wl.json || exit 1
done
for spec in "64 pbf_T" "128 pbf" "128 pbf_T" "64 pbf" "64 pa_ef"; do
  set -- $spec; R=$1; OP=$2
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
             "SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES" \
             "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    KB_R=$R timeout -s KILL 120 rocprofv3 --pmc $grp -d "$PWD/$O/pmcsq_${OP}_r${R}_$i" -o run --output-format csv -- python scripts/dev/kbench.py $OP 2 > $O/pmcsq_${OP}_r${R}_$i.log 2>&1
    rc=$?; echo "sq $OP r$R group $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/pmcsq_${OP}_r${R}_$i.log; exit $rc; fi
    i=$((i+1))
  done
done
python scripts/pmc_sq_summary.py $O > $O/pmc_sq.json
echo "summary rc=$?"
# the round-5 call-L tree (2163ed7, where test_bf16_matches_oracle_three_steps[wide_T_bf16G] met a
# flipped Q column): the pivot record of that flip
(cd r05L_tree && timeout -k 10 120 python scripts/dev/r06/diag_bf16_flip.py ../$O/bf16_flip_r05L.json > ../$O/bf16_flip_r05L.log 2>&1)
echo "flip diag rc=$?"; tail -6 $O/bf16_flip_r05L.log
