#!/bin/bash
# Source-branch likelihood launch time (likelihood_source_branch leg) of libsbz variants
# (tools/build_lik_variant.sh): VARIANTS="default ab1 ..."
mkdir -p gpurun_out/abs
for v in ${VARIANTS:-default}; do
  lib=$PWD/contact_zones_amd/libsbz.so; [ $v != default ] && lib=$PWD/contact_zones_amd/libsbz_$v.so
  SBZ_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --mh-steps 0 --src-steps 0 --other-steps 0 --source-lik-steps 100 > gpurun_out/abs/$v.json || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['likelihood_source_branch']; print(sys.argv[1], round(s['launch_us'],2), round(s['frac'],3))" gpurun_out/abs/$v.json
done
