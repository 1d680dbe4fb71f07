# round-5 call AB: PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of the Llama step's kernels and
# the SQ counters of the streaming kernels, on the final tree
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_pmc.sh || exit 1
cp gpurun_out/pmc_traffic.json gpurun_out/r05ab_llama_pmc_traffic.json
bash scripts/gpu_pmc_sq.sh || exit 1
cp gpurun_out/pmc_sq.json gpurun_out/r05ab_llama_pmc_sq.json
echo done
