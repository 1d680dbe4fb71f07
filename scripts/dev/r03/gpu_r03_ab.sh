# dev: same-box A/B of two codec builds on the Llama bench (default lib vs $AB_LIB)
export DION_DEV_ALLOW_LIB_PATH=1
mkdir -p gpurun_out
for i in 1 2; do
  for lib in default "$AB_LIB"; do
    if [ "$lib" = default ]; then unset DION_LIB_PATH; else export DION_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    echo "$lib: $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
