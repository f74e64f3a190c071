#!/bin/bash
# Mixture-sampler group A/B on one GPU box: sampler parity tests, then tools/mh_optime.py per
# SBZ_OPT_MH_GROUP value (GROUPS, default "1 4") and the phase-stamp builds when present
# (tools/build_mh_variant.sh stK -DSBZ_MH_STAMP=K).  Stops at the first failure.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_mcmc.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_grp.log 2>&1 || { tail -30 gpurun_out/pt_grp.log; exit 1; }
tail -1 gpurun_out/pt_grp.log
for g in ${MHGROUPS:-1 4}; do
  echo "group $g"; timeout -k 10 200 python -u tools/mh_optime.py --steps 3000 --sets ${SETS:-default,weights,p_global,p_zones,p_families,zone_moves} --options "{\"mh_group\": $g}" 2>&1 | grep -v '^{' | grep -v amdgpu.ids || exit 1
done
for k in 1 2 3 4 5 6; do
  [ -f contact_zones_amd/libsbz_st$k.so ] || continue
  echo "stamps K=$k"; SBZ_LIB_PATH=$PWD/contact_zones_amd/libsbz_st$k.so timeout -k 10 200 python -u tools/mh_optime.py --steps 3000 --sets ${STAMP_SETS:-default} --stamps 2>&1 | grep -v '^{' | grep -v amdgpu.ids || exit 1
done
