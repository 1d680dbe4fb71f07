# round-6 call D: single-stream rocprofv3 kernel stats (Llama: the register pass B and the LDS-DMA
# staging depths; Mixtral: register vs D = 3), the W = 8 schedule simulated on one GPU for both
# workloads (the W > 1 path now on the fused tail), the bf16 column-flip pivot record, and the
# --gpus 2 gloo rehearsal of the child launcher
set -o pipefail
mkdir -p gpurun_out/r06d
export TMPDIR=/tmp
O=gpurun_out/r06d
export DION_DEV_ALLOW_LIB_PATH=1
prof() {  # label, lib ("" = this tree), bench args
  local label=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then
    DION_LIB_PATH=$PWD/megatron-dion_amd/csrc/variants/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$label -o run -- python bench.py --streams 1 --no-cpu-baseline "$@" > $O/prof_$label.log 2>&1 || return 1
  else
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$label -o run -- python bench.py --streams 1 --no-cpu-baseline "$@" > $O/prof_$label.log 2>&1 || return 1
  fi
  echo "prof $label ok"
}
prof llama_d3 "" --steps 3 --warmup 2 || exit 1
prof llama_gl0 libdion_codec_gl0.so --steps 3 --warmup 2 || exit 1
prof llama_d2 libdion_codec_d2.so --steps 3 --warmup 2 || exit 1
prof llama_d4 libdion_codec_d4.so --steps 3 --warmup 2 || exit 1
prof mx_d3 "" --workload mixtral-8x7b-experts-r128 --steps 3 --warmup 2 || exit 1
prof mx_gl0 libdion_codec_gl0.so --workload mixtral-8x7b-experts-r128 --steps 3 --warmup 2 || exit 1
unset DION_DEV_ALLOW_LIB_PATH
line() { grep '^{"metric' "$1" > "$2" && python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['step']['frac'] if 'step' in r else '')" "$2"; }
timeout -k 10 300 python bench.py --simulate-world 8 --steps 20 --warmup 3 --no-cpu-baseline > $O/sim8_llama.log 2>&1 || exit 1
line $O/sim8_llama.log $O/sim8_llama.json || exit 1
timeout -k 10 300 python bench.py --simulate-world 8 --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 --no-cpu-baseline > $O/sim8_mixtral.log 2>&1 || exit 1
line $O/sim8_mixtral.log $O/sim8_mixtral.json || exit 1
timeout -k 10 120 python scripts/dev/r06/diag_bf16_flip.py $O/bf16_flip.json > $O/bf16_flip.log 2>&1 || exit 1
tail -6 $O/bf16_flip.log
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --layers 4 --steps 3 --warmup 1 > $O/gloo2.log 2>&1 || exit 1
line $O/gloo2.log $O/gloo2.json
