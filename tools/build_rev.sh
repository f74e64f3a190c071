#!/bin/bash
# Build libsbz from a git revision as an A/B variant: tools/build_rev.sh REV NAME [hipcc defines...]
# Output: contact_zones_amd/libsbz_NAME.so (git-ignored; travels with gpurun).
set -e
root="$(cd "$(dirname "$0")/.." && pwd)"
rev=$1; name=$2; shift 2
tmp=$(mktemp -d /tmp/sbzrev.XXXX)
mkdir -p $tmp/include $tmp/contact_zones_amd/csrc
git -C "$root" show $rev:include/sbz.h > $tmp/include/sbz.h
for f in $(git -C "$root" ls-tree --name-only $rev contact_zones_amd/csrc/); do
    git -C "$root" show $rev:$f > $tmp/$f
done
TORCH_LIB=$(python -c 'import os,torch;print(os.path.join(os.path.dirname(torch.__file__),"lib"))')
cd $tmp/contact_zones_amd/csrc
for src in *.hip; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off "$@" -c $src -o ${src%.hip}.o 2>&1 | grep -E "error" -A3 || true
done
g++ -shared -o "$root/contact_zones_amd/libsbz_$name.so" *.o -L$TORCH_LIB -lamdhip64 \
    -Wl,--disable-new-dtags,-rpath,$TORCH_LIB -Wl,--no-undefined
rm -rf $tmp
echo "built contact_zones_amd/libsbz_$name.so from $rev"
