#!/bin/bash
# By-site source-branch launch with 2-bit source planes (source_to_pk_kernel + lik_source_rc_kernel
# <planes>) and with the byte reorder (src_pack = 0), for libsbz variants built by
# tools/build_lik_variant.sh (e.g. -DSBZ_PK_P=128): cfg5, 256 chains, bench.py's
# likelihood_source_branch.by_site.  VARIANTS="default p128 ..." ROUNDS=2
set -u
mkdir -p gpurun_out
Q="--steps 5 --warmup 2 --cpu-seconds 0 --cpu-sampler-seconds 0 --cpu-src-sampler-seconds 0 --mh-steps 0 --src-steps 0 --src-sampler-steps 0 --other-steps 0 --source-lik-steps 40"
for r in $(seq ${ROUNDS:-2}); do
for v in ${VARIANTS:-default}; do
  lib=$PWD/contact_zones_amd/libsbz.so; [ $v != default ] && lib=$PWD/contact_zones_amd/libsbz_$v.so
  SBZ_LIB_PATH=$lib timeout -k 10 300 python bench.py $Q > gpurun_out/ab_pk_$v.json 2> gpurun_out/ab_pk_$v.err || { tail -5 gpurun_out/ab_pk_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/ab_pk_$v.json').read().strip().splitlines()[-1])['likelihood_source_branch']
s=d['by_site']
print('$v', 'by-position %.1f us' % d['launch_us'], 'by-site planes %.1f us' % s['launch_us'], 'bytes %.1f us' % s['byte_reorder']['launch_us'])"
done
done
