#!/bin/bash
# The max-ILP machine scheduler (-mllvm -amdgpu-sched-strategy=gcn-max-ilp) on the sampler
# (mhilp) and the likelihood kernels (likilp), against production: parity, then alternated rounds.
SBZ_LIB_PATH=$PWD/contact_zones_amd/libsbz_mhilp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_sampler.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mhilp_pytest.log 2>&1
echo "mhilp sampler tests rc=$?"; tail -1 gpurun_out/mhilp_pytest.log
SBZ_LIB_PATH=$PWD/contact_zones_amd/libsbz_likilp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_likelihood.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/likilp_pytest.log 2>&1
echo "likilp likelihood tests rc=$?"; tail -1 gpurun_out/likilp_pytest.log
for r in 1 2; do VARIANTS="default mhilp" bash tools/ab_mh_variants.sh || exit 1; done
for r in 1 2 3; do VARIANTS="default likilp" bash tools/ab_lik_variants.sh 2>&1 | grep -v amdgpu.ids || exit 1; done
