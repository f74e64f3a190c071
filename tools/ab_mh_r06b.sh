#!/bin/bash
# Late round 6: mixture-sampler delta_param variants against the shipped build (libsbz_base.so):
# the sampler parity tests on the first variant, then tools/mh_optime.py alternated ROUNDS times.
set -u
mkdir -p gpurun_out
set -- ${VARIANTS:-base spa}
first=${TEST_VARIANT:-$2}
SBZ_LIB_PATH=$PWD/contact_zones_amd/libsbz_$first.so timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_mcmc.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_mhb.log 2>&1 || { tail -30 gpurun_out/pt_mhb.log; exit 1; }
tail -1 gpurun_out/pt_mhb.log
for r in $(seq ${ROUNDS:-2}); do
for v in "$@"; do
  echo "$v"; SBZ_LIB_PATH=$PWD/contact_zones_amd/libsbz_$v.so timeout -k 10 200 python -u tools/mh_optime.py --steps 3000 --sets ${SETS:-default,weights,p_zones,p_global} 2>&1 | grep -v '^{' | grep -v amdgpu.ids || exit 1
done
done
