#!/bin/bash
# Round 6: the by-site likelihood entry with 2-bit source planes -- the likelihood parity tests,
# the bench source leg (by-position, by-site planes, by-site bytes) and a rocprofv3 kernel trace.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_likelihood.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pk_pytest.log 2>&1; rc=$?; tail -5 gpurun_out/pk_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --mh-steps 0 --src-steps 0 --other-steps 0 --cpu-seconds 0 --cpu-sampler-seconds 0 --cpu-src-sampler-seconds 0 --src-sampler-steps 0 > gpurun_out/pk_bench.json 2> gpurun_out/pk_bench.err || { tail -20 gpurun_out/pk_bench.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/pk_bench.json').read().strip().splitlines()[-1]);l=d['likelihood_source_branch'];print(l['launch_us'], json.dumps(l['by_site']))"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pk -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --mh-steps 0 --src-steps 0 --other-steps 0 --cpu-seconds 0 --cpu-sampler-seconds 0 --cpu-src-sampler-seconds 0 --src-sampler-steps 0 > gpurun_out/prof_pk.log 2>&1 || exit 1
head -8 gpurun_out/prof_pk/run_kernel_stats.csv | cut -c1-200
