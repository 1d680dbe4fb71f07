# wide pass A: parity tests of the deferred-EF pass A, then A/B against the round-3 kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "deferred_ef or project_kernels or schedule" > gpurun_out/r04_w1_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r04_w1_pytest.log; [ $rc = 0 ] || exit 1
AB_ROUNDS=3 bash scripts/dev/r04/ab.sh pa o,qkv,fc1 x0 w1 > gpurun_out/r04_ab_w1.txt 2>&1 || exit 1
cat gpurun_out/r04_ab_w1.txt
timeout -k 10 250 ./scripts/ubench/passa_geom3 > gpurun_out/r04_geom3b.txt 2>&1
