# LDS-DMA pass A at r = 64: parity tests (in-tree build), then the Llama probe A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "deferred_ef" > gpurun_out/r04_gl64_pytest.log 2>&1 || { tail -30 gpurun_out/r04_gl64_pytest.log; exit 1; }
tail -2 gpurun_out/r04_gl64_pytest.log
bash scripts/dev/r04/probe_ab.sh "--steps 10 --warmup 3" "$@"
