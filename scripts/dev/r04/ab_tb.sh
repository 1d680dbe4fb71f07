set -o pipefail
AB_ROUNDS=3 bash scripts/dev/r04/ab.sh pb o,qkv,fc1,fc2 t0 pbc512 pbc1024 pbr1024 pbr4096 > gpurun_out/r04_ab_tb_pb.txt 2>&1 || exit 1
AB_ROUNDS=3 bash scripts/dev/r04/ab.sh pa o,qkv t0 pa1024 pa768 > gpurun_out/r04_ab_tb_pa.txt 2>&1 || exit 1
