#!/bin/bash
# Sampler step time of libsbz variants (tools/build_mh_variant.sh): VARIANTS="default nst ..."
for v in ${VARIANTS:-default}; do
  lib=$PWD/contact_zones_amd/libsbz.so; [ $v != default ] && lib=$PWD/contact_zones_amd/libsbz_$v.so
  echo -n "$v "; SBZ_LIB_PATH=$lib timeout -k 10 200 python tools/mh_optime.py --steps 2000 --sets default,weights 2>&1 | tail -1 || exit 1
done
