#!/bin/bash
# A/B variant with the source-mode sampler translation unit of a git revision and everything else
# from the working tree: tools/build_src_rev.sh REV NAME [hipcc defines...]
# Output: contact_zones_amd/libsbz_NAME.so (git-ignored; travels with gpurun).
set -e
root="$(cd "$(dirname "$0")/.." && pwd)"
rev=$1; name=$2; shift 2
tmp=$(mktemp -d /tmp/sbzsrc.XXXX)
mkdir -p $tmp/include $tmp/contact_zones_amd/csrc
cp "$root"/include/sbz.h $tmp/include/
cp "$root"/contact_zones_amd/csrc/*.h $tmp/contact_zones_amd/csrc/
git -C "$root" show $rev:contact_zones_amd/csrc/sbz_mh_src.hip > $tmp/contact_zones_amd/csrc/sbz_mh_src.hip
TORCH_LIB=$(python -c 'import os,torch;print(os.path.join(os.path.dirname(torch.__file__),"lib"))')
make -s -C "$root/contact_zones_amd/csrc" build/sbz_api.o build/sbz_lik.o build/sbz_mh.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -mllvm -disable-machine-licm "$@" \
    -c $tmp/contact_zones_amd/csrc/sbz_mh_src.hip -o $tmp/sbz_mh_src.o
b="$root/contact_zones_amd/csrc/build"
g++ -shared -o "$root/contact_zones_amd/libsbz_$name.so" $b/sbz_api.o $b/sbz_lik.o $b/sbz_mh.o $tmp/sbz_mh_src.o \
    -L$TORCH_LIB -lamdhip64 -Wl,--disable-new-dtags,-rpath,$TORCH_LIB -Wl,--no-undefined
rm -rf $tmp
echo "built contact_zones_amd/libsbz_$name.so (sbz_mh_src.hip from $rev)"
