#!/bin/bash
# Mixture-leg launch time of libsbz variants (tools/build_lik_variant.sh): VARIANTS="default ab1 ..."
mkdir -p gpurun_out/abv
for v in ${VARIANTS:-default}; do
  lib=$PWD/contact_zones_amd/libsbz.so; [ $v != default ] && lib=$PWD/contact_zones_amd/libsbz_$v.so
  SBZ_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 300 --warmup 30 --cpu-seconds 0 --cpu-sampler-seconds 0 --src-sampler-steps 0 --mh-steps 0 --src-steps 0 --source-lik-steps 0 --other-steps 100 > gpurun_out/abv/$v.json || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['roofline']['launch_us_event'],2), round(d['likelihood_other_configs']['cfg5_Fam0_2000x500x10_Z8']['launch_us'],2) if 'likelihood_other_configs' in d else '')" gpurun_out/abv/$v.json
done
