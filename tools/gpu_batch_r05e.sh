set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_source.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_src_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05_src_tests.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="default" SETS=default,zone_moves,weights,p_zones bash tools/ab_src_sets.sh 2>&1
SBZ_LIB_PATH=$PWD/contact_zones_amd/libsbz_stamp.so timeout -k 10 300 python -u tools/tb_stamps.py 100 zone_moves 2>&1 | grep -v amdgpu.ids
