set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/dev/r05/diag_ortho.py 2>&1 | grep -v Warn | tail -8
