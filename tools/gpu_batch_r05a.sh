set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_source.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_src_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05_src_tests.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="default nolicm rb1 default nolicm" SETS=default,zone_moves,weights,p_global,p_zones,p_families bash tools/ab_src_sets.sh > gpurun_out/r05_ab_src_sets.txt 2>&1 || exit 1
cat gpurun_out/r05_ab_src_sets.txt
VARIANTS="default rot stag2 stag4 default rot" bash tools/ab_lik_variants.sh || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_likelihood.py -x -q --timeout 200 --timeout-method thread -k "hpm or pm" > gpurun_out/r05_lik_pm.log 2>&1; rc=$?; tail -2 gpurun_out/r05_lik_pm.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r05_tb_stamps4.txt
for set in zone_moves p_zones p_global weights; do SBZ_LIB_PATH=$PWD/contact_zones_amd/libsbz_stamp.so timeout -k 10 300 python -u tools/tb_stamps.py 100 $set 2>&1 | grep -v amdgpu.ids >> gpurun_out/r05_tb_stamps4.txt || exit 1; done
cat gpurun_out/r05_tb_stamps4.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharding.py -x -q --timeout 300 --timeout-method thread -k independent > gpurun_out/r05_indep.log 2>&1; rc=$?; tail -3 gpurun_out/r05_indep.log; exit $rc
