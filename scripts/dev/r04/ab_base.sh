# baseline of the codec A/B harness + TA/TD counters of pass A (fc1 group)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/megatron-dion_amd/csrc/libdion_codec.so
timeout -k 10 240 ./scripts/ubench/codec_ab pa,pb,upd o,qkv,fc1,fc2 $L > gpurun_out/r04_ab_base.txt 2>&1 || exit 1
cat gpurun_out/r04_ab_base.txt
i=0
for c in "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE" "TD_TD_BUSY_sum TA_FLAT_WRITE_WAVEFRONTS_sum" "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"; do
  i=$((i+1))
  AB_ROUNDS=1 AB_REPS=2 timeout -s KILL 90 rocprofv3 --pmc $c -d $PWD/gpurun_out/r04_pmc_ta$i -o run --output-format csv -- ./scripts/ubench/codec_ab pa,pb,upd fc1 $L > gpurun_out/r04_pmc_ta$i.log 2>&1
  echo "pmc pass $i rc=$?"
done
