# r = 128 LDS-DMA weight update: update precision + deferred-EF parity tests, then the Mixtral probe A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_update_precision.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_glw_pytest.log 2>&1 || { tail -30 gpurun_out/r04_glw_pytest.log; exit 1; }
tail -2 gpurun_out/r04_glw_pytest.log
bash scripts/dev/r04/probe_ab.sh "--workload mixtral-8x7b-experts-r128 --steps 4 --warmup 2" "$@"
