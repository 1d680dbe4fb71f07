# round-5 call D: stream schedules, one process each (priority / CU mask / pipelined)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in base base_hi pipe1 pipe1_hi pipe2 pipe2_hi base; do
  timeout -k 10 120 python scripts/dev/r05/diag_sched.py --config $c 2>&1 | grep '^{' || exit 1
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python scripts/dev/r05/diag_sched.py --config pipe2_mask 2>&1 | grep '^{'
GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python scripts/dev/r05/diag_sched.py --config base 2>&1 | grep '^{'
