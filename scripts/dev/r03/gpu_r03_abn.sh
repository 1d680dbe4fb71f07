# same-box A/B of the default library against the variant libraries named in $LIBS (Llama bench)
export DION_DEV_ALLOW_LIB_PATH=1
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for lib in default $LIBS; do
    if [ "$lib" = default ]; then unset DION_LIB_PATH; else export DION_LIB_PATH=$PWD/megatron-dion_amd/csrc/variants/$lib; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/abn.log 2>&1 || { tail -5 gpurun_out/abn.log; exit 1; }
    tail -1 gpurun_out/abn.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print('$lib', d['value'], d['ms_per_step'], ' '.join(f'{n.split(\"<\")[0]}={v[\"avg_launch_ms\"]}' for n, v in k.items()))"
  done
done
