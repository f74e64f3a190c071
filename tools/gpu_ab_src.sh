#!/bin/bash
# Per-operator A/B of source-sampler library variants at cfg5 (tools/ab_src_sets.sh), output in gpurun_out/ab_src.txt
set -u
mkdir -p gpurun_out
VARIANTS="${VARIANTS:-base default base default}" STEPS=${STEPS:-400} SETS=${SETS:-default,weights,p_global,p_zones,p_families} bash tools/ab_src_sets.sh > gpurun_out/ab_src.txt 2>&1; cat gpurun_out/ab_src.txt
