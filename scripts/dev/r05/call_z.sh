# round-5 call Z: the final tree's library (rebuilt for the header comment) on the box: smoke,
# the ABI / fused-path tests, one short bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05z_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r05z_smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "fixup or gram or pipelined or explicit" > gpurun_out/r05z_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/r05z_parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r05z_bench.log 2>&1
echo "bench rc=$?"; grep '^{"metric' gpurun_out/r05z_bench.log | cut -c1-200
