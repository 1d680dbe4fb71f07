# round-5 call W: the pipelined schedule (latency stream + streaming streams, lookahead) against
# the default two-stream stagger, several samples on one box; the reductions change against
# call U's tree (variants/lib_u.so, default schedule)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export DION_DEV_ALLOW_LIB_PATH=1
run() {  # label, lib ("" = this tree), extra bench args
  local label=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then
    DION_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/r05w_$label.log 2>&1 || return 1
  else
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/r05w_$label.log 2>&1 || return 1
  fi
  python - "$label" gpurun_out/r05w_$label.log <<'PY'
import json, sys
line = next(l for l in open(sys.argv[2]) if l.startswith('{"metric'))
d = json.loads(line)
print(f"{sys.argv[1]:>12s} {d['value']:8.2f} {d['unit']} {d['ms_per_step']:8.3f} ms")
PY
}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "fixup or golden or explicit" > gpurun_out/r05w_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/r05w_parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  run u_$i variants/lib_u.so || exit 1
  run new_$i "" || exit 1
  run la1s3_$i "" --lookahead 1 --streams 3 || exit 1
  run la2s3_$i "" --lookahead 2 --streams 3 || exit 1
  run la1s2_$i "" --lookahead 1 --streams 2 || exit 1
done
run mx_new "" --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
run mx_la1s3 "" --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 --lookahead 1 --streams 3 || exit 1
