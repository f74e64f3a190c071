#!/bin/bash
# Round 6: mixture-sampler zone moves with the compaction-free neighbour marking (libsbz.so) against
# the build before it (libsbz_mhbase.so): the sampler parity tests on the new build, then
# tools/mh_optime.py (zone moves alone and the default mix), alternated ROUNDS times (SKIP_TESTS=1:
# no tests).
set -u
mkdir -p gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_mcmc.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_mark.log 2>&1 || { tail -30 gpurun_out/pt_mark.log; exit 1; }
  tail -1 gpurun_out/pt_mark.log
fi
for r in $(seq ${ROUNDS:-2}); do
for v in mhbase default; do
  lib=$PWD/contact_zones_amd/libsbz.so; [ $v != default ] && lib=$PWD/contact_zones_amd/libsbz_$v.so
  echo "$v"; SBZ_LIB_PATH=$lib timeout -k 10 200 python -u tools/mh_optime.py --steps 3000 --sets zone_moves,default 2>&1 | grep -v '^{' | grep -v amdgpu.ids || exit 1
done
done
