# one GPU box call: N = 2 gloo bench rehearsal, pass-A variant A/B, counter list
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc_counters.txt 2>&1 || true
timeout -k 10 600 python bench.py --gpus 2 --backend gloo --layers ${GLOO_LAYERS:-4} --steps 3 --warmup 1 > gpurun_out/bench_gloo2.log 2>&1
rc=$?; echo "gloo bench rc=$rc"; grep -a '"metric"' gpurun_out/bench_gloo2.log | tail -1 | cut -c1-400
if [ $rc -ne 0 ]; then tail -20 gpurun_out/bench_gloo2.log; exit $rc; fi
OPS="${OPS:-pa_ef pa_ef_T}" bash scripts/dev/ab_kernels.sh ${VARIANTS:-default}
