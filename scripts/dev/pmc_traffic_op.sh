# HBM bytes per kernel of one kbench op: bash scripts/dev/pmc_traffic_op.sh <op> [lib variant]
export DION_DEV_ALLOW_LIB_PATH=1
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
OP=$1
if [ -n "$2" ]; then export DION_LIB_PATH=$PWD/megatron-dion_amd/csrc/variants/libdion_codec_$2.so; fi
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d "$PWD/gpurun_out/pmct_${OP}$2_$c" -o run --output-format csv -- python scripts/dev/kbench.py $OP 2 > gpurun_out/pmct_${OP}$2_$c.log 2>&1
  rc=$?; echo "pmc $OP$2 $c rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
python scripts/pmc_traffic.py gpurun_out/pmct_${OP}$2_FETCH_SIZE gpurun_out/pmct_${OP}$2_WRITE_SIZE > gpurun_out/pmct_${OP}$2.json
