# r = 128 fused pass A row kernel with 16-row waves and a prefetch stage (kr1) vs 32-row
export DION_DEV_ALLOW_LIB_PATH=1
# waves without (default): parity (full-size Mixtral shapes and the r = 128 seeded cases
# through kr1), kbench, Mixtral bench lines with each, stream counts
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
KR1=$PWD/megatron-dion_amd/csrc/variants/libdion_codec_kr1.so
DION_LIB_PATH=$KR1 timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_kr1.log 2>&1
rc=$?; echo "pytest kr1 rc=$rc"; tail -n 2 gpurun_out/pytest_kr1.log; if [ $rc -ne 0 ]; then exit $rc; fi
KB_R=128 OPS="pa_ef" bash scripts/dev/ab_kernels.sh default kr1 default kr1 || exit $?
for v in default kr1; do
  for st in 2 3; do
    if [ $v = default ]; then export DION_LIB_PATH=; else export DION_LIB_PATH=$KR1; fi
    timeout -k 10 400 python bench.py --workload mixtral-8x7b-experts-r128 --steps 4 --warmup 2 --no-cpu-baseline --streams $st > gpurun_out/mx_${v}_$st.log 2>&1
    rc=$?; echo "mixtral $v streams=$st rc=$rc $(tail -n 1 gpurun_out/mx_${v}_$st.log | grep -o '"value": [0-9.]*')  $(tail -n 1 gpurun_out/mx_${v}_$st.log | grep -o '"ms_per_step": [0-9.]*')"; if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
