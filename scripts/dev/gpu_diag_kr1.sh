set -o pipefail
export DION_DEV_ALLOW_LIB_PATH=1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python scripts/dev/diag_kr1.py default || exit $?
DION_LIB_PATH=$PWD/megatron-dion_amd/csrc/variants/libdion_codec_kr1.so timeout -k 10 120 python scripts/dev/diag_kr1.py kr1 || exit $?
python scripts/dev/diag_kr1_cmp.py
