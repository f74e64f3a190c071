#!/bin/bash
# The likelihood kernels without MachineLICM (tools/build_variant.sh liknolicm -mllvm
# -disable-machine-licm) against production: parity of the variant, then alternated launch times.
SBZ_LIB_PATH=$PWD/contact_zones_amd/libsbz_liknolicm.so timeout -k 10 300 python -u -m pytest tests/test_gpu_likelihood.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/liknolicm_pytest.log 2>&1
echo "liknolicm likelihood tests rc=$?"; tail -1 gpurun_out/liknolicm_pytest.log
for r in 1 2 3; do VARIANTS="default liknolicm" bash tools/ab_lik_variants.sh || exit 1; done
