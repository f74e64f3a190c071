#!/bin/bash
# Mixture sampler, 4 vs 8 waves per chain (libsbz_w8: tools/build_mh_variant.sh w8 -DSBZ_MH_WAVES=8)
# with move groups of 4 / 8: sampler tests on the variant, then tools/mh_optime.py per setting.
set -u
SBZ_LIB_PATH=$PWD/contact_zones_amd/libsbz_w8.so timeout -k 10 400 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_mcmc.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_w8.log 2>&1 || { tail -30 gpurun_out/pt_w8.log; exit 1; }
tail -1 gpurun_out/pt_w8.log
for r in 1 2; do
for v in default w8; do
  lib=$PWD/contact_zones_amd/libsbz.so; [ $v != default ] && lib=$PWD/contact_zones_amd/libsbz_$v.so
  for g in 4 8; do
    [ $v = default ] && [ $g = 8 ] && continue
    echo "$v group $g"; SBZ_LIB_PATH=$lib timeout -k 10 200 python -u tools/mh_optime.py --steps 3000 --sets ${SETS:-default,weights,zone_moves} --options "{\"mh_group\": $g}" 2>&1 | grep -v '^{' | grep -v amdgpu.ids || exit 1
  done
done
done
