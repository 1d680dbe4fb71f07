# round-5 call Y: pipeline depth and stream count around the new default (streams 3, lookahead 2),
# one box, 20 steps each (Mixtral 10)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # label, extra bench args
  local label=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/r05y_$label.log 2>&1 || return 1
  python - "$label" gpurun_out/r05y_$label.log <<'PY'
import json, sys
line = next(l for l in open(sys.argv[2]) if l.startswith('{"metric'))
d = json.loads(line)
print(f"{sys.argv[1]:>12s} {d['value']:8.2f} {d['unit']} {d['ms_per_step']:8.3f} ms")
PY
}
for i in 1 2; do
  run la2s3_$i || exit 1
  run la3s3_$i --lookahead 3 || exit 1
  run la2s4_$i --streams 4 || exit 1
  run la4s3_$i --lookahead 4 || exit 1
done
run mx_la2s3 --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
run mx_la3s3 --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 --lookahead 3 || exit 1
run mx_la0s2 --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 --lookahead 0 --streams 2 || exit 1
run bf16_la2s3 --state-dtype bf16 || exit 1
run bf16_la0s2 --state-dtype bf16 --lookahead 0 --streams 2 || exit 1
