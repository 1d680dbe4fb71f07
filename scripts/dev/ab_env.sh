# A/B of an env knob on kbench ops: VAR=DION_RANK_VARIANT VALUES="0 1 2" OPS="w w_T" bash scripts/dev/ab_env.sh
set -o pipefail
mkdir -p gpurun_out
for v in $VALUES; do
  for op in $OPS; do
    env $VAR=$v timeout -k 10 120 python scripts/dev/kbench.py $op 5 > gpurun_out/abenv_${v}_$op.log 2>&1
    rc=$?
    echo "$VAR=$v $op rc=$rc $(tail -1 gpurun_out/abenv_${v}_$op.log)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
