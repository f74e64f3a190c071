#!/bin/bash
# Build a diagnostic variant of libsbz with extra hipcc defines for the SAMPLE_SOURCE = true
# sampler kernel: tools/build_src_variant.sh NAME -DSBZ_SRC_STAMP=1 ...
# Output: contact_zones_amd/libsbz_NAME.so (git-ignored; travels to the GPU box with gpurun).
# OPT=-O2 etc. overrides the optimisation level.
set -e
cd "$(dirname "$0")/../contact_zones_amd/csrc"
name=$1; shift
TORCH_LIB=$(python -c 'import os,torch;print(os.path.join(os.path.dirname(torch.__file__),"lib"))')
mkdir -p build_$name
make -s build/sbz_api.o build/sbz_lik.o build/sbz_mh.o
/opt/rocm/bin/hipcc ${OPT:--O3} -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -mllvm -disable-machine-licm "$@" -c sbz_mh_src.hip -o build_$name/sbz_mh_src.o
g++ -shared -o ../libsbz_$name.so build/sbz_api.o build/sbz_lik.o build/sbz_mh.o build_$name/sbz_mh_src.o \
    -L$TORCH_LIB -lamdhip64 -Wl,--disable-new-dtags,-rpath,$TORCH_LIB -Wl,--no-undefined
