# stream count / launch-group size A/B on the Mixtral r=128 and Llama sets (bench lines)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for args in "--streams 2" "--streams 3" "--streams 4" "--streams 3 --coalesce 8" "--streams 2"; do
  timeout -k 10 400 python bench.py --workload mixtral-8x7b-experts-r128 --steps 4 --warmup 2 --no-cpu-baseline --probe-steps 0 $args > gpurun_out/mx.log 2>&1
  rc=$?; echo "mixtral $args rc=$rc $(tail -n 1 gpurun_out/mx.log | cut -c1-200 | grep -o '"value": [0-9.]*, .*ms_per_step": [0-9.]*')"; if [ $rc -ne 0 ]; then exit $rc; fi
done
for args in "--streams 2" "--streams 3" "--streams 2"; do
  timeout -k 10 400 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --probe-steps 0 $args > gpurun_out/ll.log 2>&1
  rc=$?; echo "llama $args rc=$rc $(tail -n 1 gpurun_out/ll.log | cut -c1-200 | grep -o '"value": [0-9.]*, .*ms_per_step": [0-9.]*')"; if [ $rc -ne 0 ]; then exit $rc; fi
done
