set -u
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_likelihood.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pt_lik.log 2>&1 || { tail -30 gpurun_out/pt_lik.log; exit 1; }
tail -1 gpurun_out/pt_lik.log
Q="--steps 20 --warmup 5 --cpu-seconds 0 --cpu-sampler-seconds 0 --cpu-src-sampler-seconds 0 --mh-steps 0 --src-steps 0 --src-sampler-steps 0 --other-steps 0"
timeout -k 10 300 python bench.py $Q > gpurun_out/bench_tr.json 2> gpurun_out/bench_tr.err || { tail -20 gpurun_out/bench_tr.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/bench_tr.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], json.dumps(d['likelihood_source_branch']['by_site']), d['likelihood_source_branch']['launch_us'], d.get('processes_at_exit'))"
rm -rf gpurun_out/prof_tr
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tr -o run --output-format csv -- python3 bench.py $Q > gpurun_out/prof_tr.log 2>&1 || { tail -5 gpurun_out/prof_tr.log; exit 1; }
find gpurun_out/prof_tr -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200 | head -12
