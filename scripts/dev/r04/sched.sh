set -o pipefail
mkdir -p gpurun_out
for v in "a:" "b:--lookahead 1" "c:--lookahead 2" "d:--streams 3 --lookahead 1" "e:--streams 3" "f:--lookahead 3"; do
  tag=${v%%:*}; args=${v#*:}
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --probe-steps 0 --no-cpu-baseline $args > gpurun_out/r04_sched_$tag.log 2>&1 || exit 1
  echo "$tag [$args] $(tail -1 gpurun_out/r04_sched_$tag.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --probe-steps 0 --no-cpu-baseline > gpurun_out/r04_sched_a2.log 2>&1 || exit 1
echo "a2 [] $(tail -1 gpurun_out/r04_sched_a2.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
