# round-6 call G1: the final tree's GPU suite and smoke, and the pivot record of round 5's bf16
# column flip on the round-5 call-L tree (r05L_tree, dev-only, not part of the product)
set -o pipefail
mkdir -p gpurun_out/r06g
export TMPDIR=/tmp
O=gpurun_out/r06g
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider --durations=15 > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
(cd r05L_tree && timeout -k 10 120 python scripts/dev/r06/diag_bf16_flip.py ../$O/bf16_flip_r05L.json > ../$O/bf16_flip_r05L.log 2>&1)
echo "flip diag rc=$?"; grep -v amdgpu.ids $O/bf16_flip_r05L.log | tail -6
