#!/bin/bash
# A/B bench of library variants on the GPU box.
#   tools/ab.sh SPEC...   SPEC = variant[:ENV=VAL[,ENV=VAL]]  ("default" = contact_zones_amd/libsbz.so)
# Writes gpurun_out/ab_<spec>.json; stops at the first failing run.
set -o pipefail
for spec in "$@"; do
    v=${spec%%:*}
    envs=""
    [[ $spec == *:* ]] && envs=${spec#*:}
    lib=$PWD/contact_zones_amd/libsbz.so
    [ "$v" != "default" ] && lib=$PWD/contact_zones_amd/libsbz_$v.so
    tag=$(echo "$spec" | tr ':=,' '___')
    env ${envs//,/ } SBZ_LIB_PATH=$lib SBZ_ALLOW_NONFINITE=1 timeout -k 10 300 python bench.py \
        --steps ${STEPS:-200} --warmup 20 --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/ab_$tag.json || exit $?
done
