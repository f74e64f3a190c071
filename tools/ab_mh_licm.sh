#!/bin/bash
# mh_kernel built without MachineLICM (-mllvm -disable-machine-licm: loop invariants are not
# hoisted into registers held across the step loop; 276 instead of 440 registers per lane), at 4
# and 8 waves per chain, against production: sampler parity tests of each variant, then
# alternated step-time rounds (tools/mh_optime.py).
mkdir -p gpurun_out
for v in nolicm nolicm8; do
  SBZ_LIB_PATH=$PWD/contact_zones_amd/libsbz_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_mcmc.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${v}_pytest.log 2>&1
  echo "$v sampler tests rc=$?"; tail -1 gpurun_out/${v}_pytest.log
done
for r in 1 2; do VARIANTS="default nolicm nolicm8" bash tools/ab_mh_variants.sh || exit 1; done
# the source-mode sampler kernel without MachineLICM (180 VGPRs, no scratch, against 256 + 48 B)
SBZ_LIB_PATH=$PWD/contact_zones_amd/libsbz_srcnolicm.so timeout -k 10 300 python -u -m pytest tests/test_gpu_source.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/srcnolicm_pytest.log 2>&1
echo "srcnolicm source tests rc=$?"; tail -1 gpurun_out/srcnolicm_pytest.log
MH_VARIANTS="default" SRC_VARIANTS="default srcnolicm" bash tools/ab_flog.sh || exit 1
