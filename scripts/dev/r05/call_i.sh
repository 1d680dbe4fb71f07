# round-5 call I: triangular-solve variants; Mixtral phase costs; end-to-end with host copies
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 scripts/ubench/trsm_ab > gpurun_out/r05i_trsm.log 2>&1; echo "trsm rc=$?"; cat gpurun_out/r05i_trsm.log
timeout -k 10 400 python scripts/dev/r05/diag_phases.py --workload mixtral-8x7b-experts-r128 --streams 2 --steps 6 --modes base,no_ortho,no_fixup,only_streaming > gpurun_out/r05i_diag_mx.log 2>&1
echo "diag rc=$?"; grep '^{"streams' gpurun_out/r05i_diag_mx.log
timeout -k 10 400 python scripts/e2e_pcie.py > gpurun_out/r05i_e2e.log 2>&1; echo "e2e rc=$?"; tail -3 gpurun_out/r05i_e2e.log
