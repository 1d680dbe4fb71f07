# parity of the ring-free + rank-depth-1 build, then bench A/B of the in-tree build against
export DION_DEV_ALLOW_LIB_PATH=1
# the two variants on the Llama and Mixtral sets
set -o pipefail
mkdir -p gpurun_out
DION_LIB_PATH=$PWD/megatron-dion_amd/csrc/variants/libnoring_rd1.so timeout -k 10 400 python -u -m pytest \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1
rc=$?; tail -2 gpurun_out/par.log; [ $rc = 0 ] || exit 1
for v in libnoring_rd1.so libnoring.so; do
  echo "== $v (old = variant)"
  OLD_LIB=$v bash scripts/gpu_r03_llab.sh || exit 1
  OLD_LIB=$v BENCH_ARGS="--workload mixtral-8x7b-experts-r128" bash scripts/gpu_r03_llab.sh || exit 1
done
