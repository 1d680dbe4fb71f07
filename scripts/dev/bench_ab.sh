# dev: bench A/B of schedule options in one box call: ARGS_LIST="--lookahead 0|--lookahead 1" (| separated;
# a case may carry environment assignments before a ';': "DION_LOCAL_ORDER=stagger;--streams 2")
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS='|' read -ra CASES <<< "${ARGS_LIST:---lookahead 0}"
i=0
for rep in 1 2; do
for a in "${CASES[@]}"; do
  envs=""; args="$a"; if [[ "$a" == *";"* ]]; then envs="${a%%;*}"; args="${a#*;}"; fi
  timeout -k 10 240 env $envs python bench.py --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline --probe-steps 0 $args > gpurun_out/ab_$i.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "[$a] rc=$rc"; tail -5 gpurun_out/ab_$i.log; exit $rc; fi
  python - "$a" gpurun_out/ab_$i.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(f"{sys.argv[1]:40s} {d['value']:8.2f} GiB/s  {d['ms_per_step']:8.3f} ms")
PY
  i=$((i+1))
done
done
