set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/dev/r05/diag_dense2.py > gpurun_out/r05h.log 2>&1; echo "rc=$?"
grep -E "^call|^   col" gpurun_out/r05h.log | head -80
