#!/bin/bash
# mh_kernel at 8 waves per chain (2 per SIMD; the 256-register cap spills
# ~190 VGPRs to scratch) against the production 4.  Parity of the variant on the sampler tests,
# then alternated step-time rounds (tools/mh_optime.py).
set -o pipefail
mkdir -p gpurun_out
SBZ_LIB_PATH=$PWD/contact_zones_amd/libsbz_mw8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mw8_pytest.log 2>&1
echo "mw8 sampler tests rc=$?"; tail -3 gpurun_out/mw8_pytest.log
for r in 1 2; do VARIANTS="default mw8" bash tools/ab_mh_variants.sh || exit 1; done
