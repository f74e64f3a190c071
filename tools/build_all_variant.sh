#!/bin/bash
# Build an A/B variant of libsbz with extra hipcc defines applied to every translation unit:
#   tools/build_all_variant.sh NAME -DFOO=1 ...
# Output: contact_zones_amd/libsbz_NAME.so (git-ignored; travels to the GPU box with gpurun).
set -e
cd "$(dirname "$0")/../contact_zones_amd/csrc"
name=$1; shift
TORCH_LIB=$(python -c 'import os,torch;print(os.path.join(os.path.dirname(torch.__file__),"lib"))')
mkdir -p build_$name
for f in sbz_api sbz_lik sbz_mh sbz_mh_src; do
  extra=""; [ $f = sbz_mh ] || [ $f = sbz_lik ] && extra="-mllvm -disable-machine-licm"  # as the Makefile
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off $extra "$@" -c $f.hip -o build_$name/$f.o &
done
wait
g++ -shared -o ../libsbz_$name.so build_$name/sbz_api.o build_$name/sbz_lik.o build_$name/sbz_mh.o build_$name/sbz_mh_src.o \
    -L$TORCH_LIB -lamdhip64 -Wl,--disable-new-dtags,-rpath,$TORCH_LIB -Wl,--no-undefined
