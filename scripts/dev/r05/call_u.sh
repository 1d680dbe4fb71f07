# round-5 call U: schedule knobs of the N = 1 step on one box with the round's tree (matrices per
# launch group, streams, pipelined lookahead), 20 steps each, the default first and last
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # label, extra bench args
  local label=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/r05u_$label.log 2>&1 || return 1
  python - "$label" gpurun_out/r05u_$label.log <<'PY'
import json, sys
line = next(l for l in open(sys.argv[2]) if l.startswith('{"metric'))
d = json.loads(line)
print(f"{sys.argv[1]:>12s} {d['value']:8.2f} {d['unit']} {d['ms_per_step']:8.3f} ms")
PY
}
run default_a || exit 1
run coalesce8 --coalesce 8 || exit 1
run coalesce24 --coalesce 24 || exit 1
run coalesce32 --coalesce 32 || exit 1
run streams3 --streams 3 || exit 1
run lookahead1 --lookahead 1 --streams 3 || exit 1
run default_b || exit 1
run mx_default --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
run mx_coalesce32 --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 --coalesce 32 || exit 1
run mx_coalesce8 --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 --coalesce 8 || exit 1
