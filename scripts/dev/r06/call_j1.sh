# round-6 call J1: the final tree's GPU suite and smoke
set -o pipefail
mkdir -p gpurun_out/r06j
export TMPDIR=/tmp
O=gpurun_out/r06j
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider --durations=15 > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
