# per-kernel probe table of xlib/ builds: bash scripts/dev/r04/probe_ab.sh "ARGS" name1 name2 ...
set -o pipefail
mkdir -p gpurun_out
args=$1; shift
for v in "$@"; do
  DION_DEV_ALLOW_LIB_PATH=1 DION_LIB_PATH=$PWD/xlib/lib$v.so timeout -k 10 300 python bench.py $args --no-cpu-baseline --probe-steps 2 > gpurun_out/r04_pab_$v.log 2>&1 || exit 1
  grep '^{"metric' gpurun_out/r04_pab_$v.log | python -c '
import json,sys
d=json.loads(sys.stdin.read()); print("'$v'", d["value"], d["ms_per_step"])
for k,x in d["roofline"]["kernels"].items(): print("   ", k, x["avg_launch_ms"], x["GB/s"])'
done
