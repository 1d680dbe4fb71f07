#!/bin/bash
timeout -k 10 300 python -u -m pytest tests/test_gpu_update_precision.py -v --timeout 120 --timeout-method thread > gpurun_out/upd_h3c.log 2>&1
tail -12 gpurun_out/upd_h3c.log; cat gpurun_out/update_precision.json
