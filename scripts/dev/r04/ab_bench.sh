# bench A/B of xlib/ builds in one box call: bash scripts/dev/r04/ab_bench.sh "ARGS" name1 name2 ...
# (each library through DION_LIB_PATH, two rounds in alternating order)
set -o pipefail
mkdir -p gpurun_out
args=$1; shift
for rnd in 1 2; do
  for v in "$@"; do
    DION_DEV_ALLOW_LIB_PATH=1 DION_LIB_PATH=$PWD/xlib/lib$v.so timeout -k 10 300 python bench.py $args --no-cpu-baseline --probe-steps 0 > gpurun_out/r04_abb_$v.log 2>&1 || exit 1
    echo "$rnd $v $(grep '^{"metric' gpurun_out/r04_abb_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
