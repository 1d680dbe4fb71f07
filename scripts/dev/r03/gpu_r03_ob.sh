# dev: ortho kernel variants (build/libdion_*.so) under rocprofv3 --stats
export DION_DEV_ALLOW_LIB_PATH=1
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in inv0 inv1 inv2 fact0; do
  DION_LIB_PATH=$PWD/build/libdion_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/ob_$v" -o run --output-format csv -- python scripts/dev/ortho_bench.py > gpurun_out/ob_$v.log 2>&1 || exit $?
  tail -1 gpurun_out/ob_$v.log
  f=$(find gpurun_out/ob_$v -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | grep -v "at::native\|Name" | sed 's/(.*)"/"/' 
done
