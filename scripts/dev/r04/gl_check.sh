# r = 128 LDS-DMA pass A: parity tests (in-tree build), then the per-kernel probe of xlib/ builds on Mixtral
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "deferred_ef" > gpurun_out/r04_gl_pytest.log 2>&1 || { tail -30 gpurun_out/r04_gl_pytest.log; exit 1; }
tail -3 gpurun_out/r04_gl_pytest.log
bash scripts/dev/r04/probe_ab.sh "--workload mixtral-8x7b-experts-r128 --steps 4 --warmup 2" "$@"
