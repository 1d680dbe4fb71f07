set -o pipefail
export DION_DEV_ALLOW_LIB_PATH=1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python scripts/dev/diag_h3t2.py > gpurun_out/diag_h3t.log 2>&1 && \
DION_LIB_PATH=$PWD/megatron-dion_amd/csrc/variants/libdion_codec_x6t.so timeout -k 10 120 python scripts/dev/diag_h3t2.py > gpurun_out/diag_x6t.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/diag_h3t.log; echo ---x6t; grep -v amdgpu.ids gpurun_out/diag_x6t.log | head -8; exit $rc
