# rocprofv3 kernel stats + PMC HBM traffic + SQ counters of one bench workload (one GPU box call)
# usage: TAG=mixtral ARGS="--workload mixtral-8x7b-experts-r128" bash scripts/gpu_r03_prof_wl.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-llama}
CMD="python bench.py --no-cpu-baseline --streams 1 ${ARGS:-}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_$TAG" -o run --output-format csv -- $CMD --steps 3 --warmup 1 > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "stats $TAG rc=$rc"; tail -1 gpurun_out/prof_$TAG.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c -d "$PWD/gpurun_out/pmc_${TAG}_$c" -o run --output-format csv -- $CMD --steps 1 --warmup 1 --probe-steps 0 > gpurun_out/pmc_${TAG}_$c.log 2>&1
  rc=$?; echo "pmc $TAG $c rc=$rc"; if [ $rc -ne 0 ]; then tail -3 gpurun_out/pmc_${TAG}_$c.log; exit $rc; fi
done
python scripts/pmc_traffic.py gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE > gpurun_out/pmc_traffic_$TAG.json
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  timeout -s KILL 300 rocprofv3 --pmc $grp -d "$PWD/gpurun_out/sq/pmcsq_${TAG}_$i" -o run --output-format csv -- $CMD --steps 1 --warmup 1 --probe-steps 0 > gpurun_out/pmcsq_${TAG}_$i.log 2>&1
  rc=$?; echo "sq $TAG group $i rc=$rc"; if [ $rc -ne 0 ]; then tail -3 gpurun_out/pmcsq_${TAG}_$i.log; exit $rc; fi
  i=$((i+1))
done
python scripts/pmc_sq_summary.py gpurun_out/sq > gpurun_out/pmc_sq_$TAG.json
echo "summary rc=$?"
