# round-4 measurement set, call A: the driver's default bench line, then single-stream kernel
# traces (rocprofv3 --kernel-trace --stats) reconciled with the bench's probe for the Llama set
# (f32 and bf16 state) and the Mixtral set, and the Mixtral / bf16 default bench lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/r04_bench_llama.log 2>&1 || exit 1
grep '^{"metric' gpurun_out/r04_bench_llama.log | tail -1 | cut -c1-200
WL=llama3-8b-2d-grad-set-r64 TAG=llama bash scripts/dev/r04/recon.sh || exit 1
WL=llama3-8b-2d-grad-set-r64 TAG=bf16 EXTRA="--state-dtype bf16" bash scripts/dev/r04/recon.sh || exit 1
WL=mixtral-8x7b-experts-r128 TAG=mixtral bash scripts/dev/r04/recon.sh || exit 1
timeout -k 10 300 python bench.py --workload mixtral-8x7b-experts-r128 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r04_bench_mixtral.log 2>&1 || exit 1
grep '^{"metric' gpurun_out/r04_bench_mixtral.log | tail -1 | cut -c1-200
timeout -k 10 300 python bench.py --state-dtype bf16 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04_bench_bf16.log 2>&1 || exit 1
grep '^{"metric' gpurun_out/r04_bench_bf16.log | tail -1 | cut -c1-200
