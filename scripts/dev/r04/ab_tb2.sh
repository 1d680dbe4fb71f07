set -o pipefail
AB_ROUNDS=3 bash scripts/dev/r04/ab.sh upd o,qkv,fc1,fc2 t1 rsl256 rsl1024 > gpurun_out/r04_ab_tb2_upd.txt 2>&1 || exit 1
AB_ROUNDS=3 bash scripts/dev/r04/ab.sh pa fc2 t1 pat1024 pat4096 > gpurun_out/r04_ab_tb2_pat.txt 2>&1 || exit 1
