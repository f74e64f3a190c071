set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --cpu-seconds 0 --mh-steps 0 --src-steps 0 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { tail -20 gpurun_out/bench_quick.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/bench_quick.json').read().strip().splitlines()[-1])
print(d['value'], json.dumps(d['roofline']))
print(json.dumps(d['likelihood_source_branch']))
print({k:(v['launch_us'] if isinstance(v,dict) else v) for k,v in d['likelihood_other_configs'].items()})"
# A/B of likelihood variants (VARIANTS) and tasks per CU
if [ -n "${VARIANTS:-}" ]; then
  for r in 1 2; do VARIANTS="$VARIANTS" bash tools/ab_lik_variants.sh || exit 1; done
fi
if [ "${TASKS_AB:-0}" = 1 ]; then bash tools/ab_lik_tasks.sh || exit 1; fi
