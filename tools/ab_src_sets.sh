#!/bin/bash
# Per-operator µs/step of source-sampler library variants at cfg5 (256 chains, GPU-drawn initial
# sources): VARIANTS="default nolicm ..." SETS=default,p_zones bash tools/ab_src_sets.sh
for v in ${VARIANTS:-default}; do
  lib=$PWD/contact_zones_amd/libsbz.so; [ $v != default ] && lib=$PWD/contact_zones_amd/libsbz_$v.so
  echo "## $v"
  SBZ_LIB_PATH=$lib timeout -k 10 300 python -u tools/src_optime.py --sites 2000 --features 500 --states 10 --zones 8 --families 4 --chains 256 --steps ${STEPS:-200} --burnin 20 --gpu-init --sets ${SETS:-default} 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done
