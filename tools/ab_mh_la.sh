#!/bin/bash
# Late round 6: the mixture sampler with plan batches of 32 (libsbz.so) against batches of 24
# (libsbz_base.so): sampler parity tests on the new build, then tools/mh_optime.py alternated.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_mcmc.py tests/test_gpu_likelihood.py -k "not cfg5 or planned" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_la.log 2>&1 || { tail -30 gpurun_out/pt_la.log; exit 1; }
tail -1 gpurun_out/pt_la.log
for r in 1 2; do
for v in base default; do
  lib=$PWD/contact_zones_amd/libsbz.so; [ $v != default ] && lib=$PWD/contact_zones_amd/libsbz_$v.so
  echo "$v"; SBZ_LIB_PATH=$lib timeout -k 10 200 python -u tools/mh_optime.py --steps 3000 --sets default,weights,p_zones 2>&1 | grep -v '^{' | grep -v amdgpu.ids || exit 1
done
done
