# one call: r = 128 16-row pass A (kr1 variant) parity + A/B; then the default build's GPU
export DION_DEV_ALLOW_LIB_PATH=1
# suite, smoke, bench line and the round's committed profiles (rocprof stats, PMC traffic,
# SQ counters)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/dev/ab_r02h.sh || echo "kr1 A/B rc=$? (continuing with the default build)"
export DION_LIB_PATH=
bash scripts/gpu_r02_tests.sh || exit $?
bash scripts/gpu_r02_profiles.sh || exit $?
