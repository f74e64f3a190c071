#!/bin/bash
# By-site source-branch launch (source_to_pm_kernel + lik_source_rc_kernel) of libsbz variants,
# cfg5, 256 chains: bench.py's likelihood_source_branch.by_site, VARIANTS="default tr128 ..."
set -u
Q="--steps 5 --warmup 2 --cpu-seconds 0 --cpu-sampler-seconds 0 --cpu-src-sampler-seconds 0 --mh-steps 0 --src-steps 0 --src-sampler-steps 0 --other-steps 0 --source-lik-steps 40"
for v in ${VARIANTS:-default}; do
  lib=$PWD/contact_zones_amd/libsbz.so; [ $v != default ] && lib=$PWD/contact_zones_amd/libsbz_$v.so
  SBZ_LIB_PATH=$lib timeout -k 10 300 python bench.py $Q > gpurun_out/ab_tr_$v.json 2> gpurun_out/ab_tr_$v.err || { tail -5 gpurun_out/ab_tr_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/ab_tr_$v.json').read().strip().splitlines()[-1])['likelihood_source_branch']
print('$v', 'by-position %.1f us' % d['launch_us'], 'by-site %.1f us' % d['by_site']['launch_us'], 'transpose est %.1f us' % d['by_site']['reorder_us_est'])"
done
