set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_source.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_src_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05_src_tests.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="default" bash tools/ab_tb.sh || exit 1
VARIANTS="default rot stag2 stag4 default rot" bash tools/ab_lik_variants.sh || exit 1
SBZ_LIB_PATH=$PWD/contact_zones_amd/libsbz_stamp.so timeout -k 10 300 python -u tools/tb_stamps.py 40 > gpurun_out/r05_tb_stamps4.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r05_tb_stamps4.txt | tail -30
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharding.py -x -q --timeout 300 --timeout-method thread -k independent > gpurun_out/r05_indep.log 2>&1; rc=$?; tail -3 gpurun_out/r05_indep.log; exit $rc
