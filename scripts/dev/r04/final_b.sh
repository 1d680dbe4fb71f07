# round-4 closing call B: rocprofv3 kernel stats reconciled with the probe (Llama, bf16 state),
# PMC traffic of the bf16 and Mixtral steps, SQ counters of the Llama streaming kernels
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
WL=llama3-8b-2d-grad-set-r64 TAG=llama_f bash scripts/dev/r04/recon.sh || exit 1
WL=llama3-8b-2d-grad-set-r64 TAG=bf16_f EXTRA="--state-dtype bf16" bash scripts/dev/r04/recon.sh || exit 1
TAG=bf16 EXTRA="--state-dtype bf16" bash scripts/dev/r04/pmc_wl.sh || exit 1
WL=mixtral-8x7b-experts-r128 TAG=mixtral bash scripts/dev/r04/pmc_wl.sh || exit 1
bash scripts/gpu_pmc_sq.sh
