set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/dev/r05/diag_dense.py > gpurun_out/r05f_dense.log 2>&1; echo "dense rc=$?"
grep -v Gloo gpurun_out/r05f_dense.log | grep rank | head -60
