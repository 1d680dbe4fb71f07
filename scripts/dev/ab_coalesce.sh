# launch-group size sweep on the Llama set (bench lines, 2 streams)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in 16 8 12 24 32 16; do
  timeout -k 10 400 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --probe-steps 0 --coalesce $c > gpurun_out/ll.log 2>&1
  rc=$?; echo "llama coalesce=$c rc=$rc $(tail -n 1 gpurun_out/ll.log | grep -o '"value": [0-9.]*') $(tail -n 1 gpurun_out/ll.log | grep -o '"ms_per_step": [0-9.]*')"; if [ $rc -ne 0 ]; then exit $rc; fi
done
