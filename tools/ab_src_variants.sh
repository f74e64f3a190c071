#!/bin/bash
# Source-branch leg (repack + lik_source_rc_kernel) of libsbz variants: VARIANTS="default rc2 ..."
mkdir -p gpurun_out/abs
for v in ${VARIANTS:-default}; do
  lib=$PWD/contact_zones_amd/libsbz.so; [ $v != default ] && lib=$PWD/contact_zones_amd/libsbz_$v.so
  SBZ_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 4 --cpu-seconds 0 --mh-steps 0 --src-steps 0 --source-lik-steps 40 > gpurun_out/abs/$v.json || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1]))['likelihood_source_branch']; print(sys.argv[1], round(d['launch_us'],1), d.get('frac'), d.get('kernel_us'))" gpurun_out/abs/$v.json
done
