#!/bin/bash
# Source-sampler A/B at the real-data shapes (Balkan 28x47x3 Z3 Fam5, 256 chains; South America
# 100x36x5 Z6 Fam6, 128 chains): the source GPU tests, then libsbz_base.so (a copy of the library
# before the change, made by hand) against libsbz.so, alternated twice (tools/src_optime.py).
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_source.py tests/test_gpu_mcmc.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_src_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05_src_tests.log; [ $rc -eq 0 ] || exit $rc
for lib in libsbz_base.so libsbz.so libsbz_base.so libsbz.so; do echo "## $lib"
  SBZ_LIB_PATH=$PWD/contact_zones_amd/$lib timeout -k 10 300 python -u tools/src_optime.py --sites 28 --features 47 --states 3 --zones 3 --families 5 --chains 256 --steps 2000 --burnin 200 --sets default,weights,p_global 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  SBZ_LIB_PATH=$PWD/contact_zones_amd/$lib timeout -k 10 300 python -u tools/src_optime.py --sites 100 --features 36 --states 5 --zones 6 --families 6 --chains 128 --steps 2000 --burnin 200 --sets default 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done
