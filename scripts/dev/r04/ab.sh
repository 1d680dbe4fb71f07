# A/B of xlib/ variants through the C ABI: bash scripts/dev/r04/ab.sh OPS SHAPES name1 name2 ...
set -o pipefail
mkdir -p gpurun_out
ops=$1; shapes=$2; shift 2
libs=""
for v in "$@"; do libs="$libs $PWD/xlib/lib$v.so"; done
AB_PB_FIXED=1 timeout -k 10 ${AB_TIMEOUT:-300} ./scripts/ubench/codec_ab $ops $shapes $libs
