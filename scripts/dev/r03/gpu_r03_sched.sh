# dev: stream schedules on the Llama set, one box (A/B inside one call)
mkdir -p gpurun_out
for cfg in "--streams 2" "--streams 3 --lookahead 1" "--streams 3 --lookahead 2" "--streams 2" "--streams 4 --lookahead 1"; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $cfg > gpurun_out/sched.log 2>&1 || { tail -5 gpurun_out/sched.log; exit 1; }
  echo "$cfg: $(tail -1 gpurun_out/sched.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
