#!/bin/bash
# GPU-box routine: parity tests, smoke, bench, kernel-trace profile.  Every GPU step is
# time-limited and the script stops at the first failure.
set -u
mkdir -p gpurun_out
STEPS=${STEPS:-200}
run() { echo "== $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
run timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
run timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
run timeout -k 10 400 python bench.py --steps $STEPS --warmup 20 ${BENCH_ARGS:-} > gpurun_out/bench.json
cat gpurun_out/bench.json
if [ "${PROFILE:-1}" = "1" ]; then
  export TMPDIR=/tmp
  run timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps $STEPS --warmup 20 --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
  find gpurun_out/prof -name "*kernel_stats.csv" -exec cat {} \;
fi
