#!/bin/bash
# round 3: weight-update precision isolation (default h3 rank_stream vs bf16x6 rank_update)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_update_precision.py -v --timeout 120 --timeout-method thread > gpurun_out/upd_h3.log 2>&1
rc=$?; echo "h3 rc=$rc"; tail -15 gpurun_out/upd_h3.log
[ $rc -le 1 ] || exit $rc
cp gpurun_out/update_precision.json gpurun_out/update_precision_h3.json
DION_RANK_VARIANT=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_update_precision.py -v --timeout 120 --timeout-method thread > gpurun_out/upd_x6.log 2>&1
rc=$?; echo "x6 rc=$rc"; tail -5 gpurun_out/upd_x6.log
cp gpurun_out/update_precision.json gpurun_out/update_precision_x6.json
exit 0
