#!/bin/bash
# A/B bench of built library variants on the GPU box: tools/ab.sh VARIANT... ("" = default lib)
# Writes gpurun_out/ab_<variant>.json; stops at the first failing run.
set -o pipefail
for v in "$@"; do
    lib=$PWD/contact_zones_amd/libsbz${v:+_$v}.so
    SBZ_LIB_PATH=$lib SBZ_ALLOW_NONFINITE=1 timeout -k 10 300 python bench.py --steps ${STEPS:-200} --warmup 20 \
        --cpu-seconds 0 ${BENCH_ARGS} > gpurun_out/ab_${v:-default}.json || exit $?
done
