set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_source.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_src_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05_src_tests.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="default" SETS=default,weights bash tools/ab_src_sets.sh 2>&1
