# round-5 call AA: grid-size tuning constants (DION_TB_* split-K block targets, DION_RSL update
# row-block length) re-measured under the pipelined schedule: variant libraries against this
# tree, two samples each on one box (Llama), Mixtral for the best candidates
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export DION_DEV_ALLOW_LIB_PATH=1
run() {  # label, lib ("" = this tree), extra bench args
  local label=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then
    DION_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/r05aa_$label.log 2>&1 || return 1
  else
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/r05aa_$label.log 2>&1 || return 1
  fi
  python - "$label" gpurun_out/r05aa_$label.log <<'PY'
import json, sys
line = next(l for l in open(sys.argv[2]) if l.startswith('{"metric'))
d = json.loads(line)
print(f"{sys.argv[1]:>12s} {d['value']:8.2f} {d['unit']} {d['ms_per_step']:8.3f} ms")
PY
}
for i in 1 2; do
  run base_$i "" || exit 1
  for v in pa1024 pa4096 pbc1024 pbr2048 pat2048 rsl512; do
    run ${v}_$i variants/lib_$v.so || exit 1
  done
done
run mx_base "" --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
for v in pa1024 pa4096 pbc1024 pbr2048 pat2048 rsl512; do
  run mx_$v variants/lib_$v.so --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 || exit 1
done
