#!/bin/bash
# Round-end evidence on one GPU box: parity tests, smoke, the default bench line, a rocprofv3
# kernel-trace profile of the same bench, the PMC traffic passes, and a 2-rank rehearsal of the
# N > 1 bench path (both ranks on the one GPU, collectives over gloo).  Stops at the first failure.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "== $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
run timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
run timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
run timeout -k 10 500 python bench.py --steps 200 --warmup 20 > gpurun_out/bench.json
tail -c 400 gpurun_out/bench.json
run timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/prof.log 2>&1
find gpurun_out/prof -name "*kernel_stats.csv" -exec head -5 {} \;
run timeout -k 10 900 bash tools/pmc.sh --mh-steps 0 --src-steps 0 --source-lik-steps 0 > gpurun_out/pmc.log 2>&1
tail -3 gpurun_out/pmc.log
SBZ_DIST_BACKEND=gloo run timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 2 --steps 50 --warmup 5 --cpu-seconds 0 --mh-steps 2000 --mh-burnin 2000 --src-steps 200 --src-burnin 200 > gpurun_out/bench_2rank.json 2> gpurun_out/bench_2rank.err
tail -c 300 gpurun_out/bench_2rank.json
echo EVIDENCE_OK
