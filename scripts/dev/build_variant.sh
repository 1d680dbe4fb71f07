# build a kernel variant of the codec library: bash scripts/dev/build_variant.sh <name> [-DFOO=1 ...]
set -e
name=$1; shift
mkdir -p megatron-dion_amd/csrc/variants
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" -o megatron-dion_amd/csrc/variants/libdion_codec_$name.so megatron-dion_amd/csrc/dion_codec.hip
echo built $name
