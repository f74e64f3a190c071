#!/bin/bash
# Build an A/B variant of libsbz with extra hipcc defines: tools/build_variant.sh NAME -DFOO=1 ...
# Output: contact_zones_amd/libsbz_NAME.so (git-ignored; travels to the GPU box with gpurun).
set -e
cd "$(dirname "$0")/../contact_zones_amd/csrc"
name=$1; shift
TORCH_LIB=$(python -c 'import os,torch;print(os.path.join(os.path.dirname(torch.__file__),"lib"))')
mkdir -p build_$name
make -s build/sbz_api.o build/sbz_mh.o build/sbz_mh_src.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=${FPC:-off} -mllvm -disable-machine-licm "$@" -c sbz_lik.hip -o build_$name/sbz_lik.o 2>&1 | grep -E "error" -A3 || true
g++ -shared -o ../libsbz_$name.so build/sbz_api.o build/sbz_mh.o build/sbz_mh_src.o build_$name/sbz_lik.o -L$TORCH_LIB -lamdhip64 \
    -Wl,--disable-new-dtags,-rpath,$TORCH_LIB -Wl,--no-undefined
