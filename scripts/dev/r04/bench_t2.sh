set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04_bench_t2.log 2>&1 || exit 1
tail -1 gpurun_out/r04_bench_t2.log | cut -c1-400
AB_ROUNDS=3 bash scripts/dev/r04/ab.sh upd qkv,fc1 t2 rsl128 > gpurun_out/r04_ab_t2.txt 2>&1 || exit 1
AB_ROUNDS=3 bash scripts/dev/r04/ab.sh pa fc2 t2 pat512 >> gpurun_out/r04_ab_t2.txt 2>&1 || exit 1
AB_ROUNDS=3 bash scripts/dev/r04/ab.sh pb fc2 t2 pbr768 x0 >> gpurun_out/r04_ab_t2.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04_bench_t2b.log 2>&1 || exit 1
tail -1 gpurun_out/r04_bench_t2b.log | cut -c1-400
