#!/bin/bash
# Round-6 evidence on one GPU box: parity tests, smoke, the default bench line, a rocprofv3
# kernel-trace profile of the same bench, the PMC passes of the likelihood kernels, the mixture
# sampler and the source-mode sampler, and a 2-rank rehearsal of the N > 1 bench path (both ranks
# on the one GPU, collectives over gloo; the line marks itself "rehearsal").  Stops at the first
# failure.  Usage: bash tools/evidence_r06.sh [--no-tests]
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "== $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
if [ "${1:-}" != "--no-tests" ]; then
  run timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
  run timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
run timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
tail -c 400 gpurun_out/bench_default.json
rm -rf gpurun_out/prof6
run timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof6 -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 --cpu-sampler-seconds 0 --cpu-src-sampler-seconds 0 > gpurun_out/prof6.log 2>&1
find gpurun_out/prof6 -name "*kernel_stats.csv" -exec head -14 {} \; | cut -c1-160
rm -rf gpurun_out/pmc6
PMC_OUT=gpurun_out/pmc6 run timeout -k 10 900 bash tools/pmc.sh --mh-steps 0 --src-steps 0 --other-steps 0 --cpu-sampler-seconds 0 --cpu-src-sampler-seconds 0 --src-sampler-steps 0 > gpurun_out/pmc6.log 2>&1
tail -4 gpurun_out/pmc6.log
rm -rf gpurun_out/pmc6_mh
PMC_OUT=gpurun_out/pmc6_mh run timeout -k 10 900 bash tools/pmc.sh --steps 2 --warmup 1 --mh-steps 3000 --mh-burnin 0 --src-steps 0 --source-lik-steps 0 --other-steps 0 --cpu-sampler-seconds 0 --cpu-src-sampler-seconds 0 --src-sampler-steps 0 > gpurun_out/pmc6_mh.log 2>&1
tail -4 gpurun_out/pmc6_mh.log
rm -rf gpurun_out/pmc6_src
PMC_OUT=gpurun_out/pmc6_src run timeout -k 10 900 bash tools/pmc_src.sh default 2000 > gpurun_out/pmc6_src.log 2>&1
tail -4 gpurun_out/pmc6_src.log
SBZ_DIST_BACKEND=gloo run timeout -k 10 500 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 2 --steps 50 --warmup 5 --cpu-seconds 0 --cpu-sampler-seconds 0 --cpu-src-sampler-seconds 0 --src-sampler-steps 200 --src-sampler-burnin 50 --mh-steps 2000 --mh-burnin 2000 --src-steps 200 --src-burnin 200 > gpurun_out/bench_2rank.json 2> gpurun_out/bench_2rank.err
tail -c 300 gpurun_out/bench_2rank.json
echo EV_OK
