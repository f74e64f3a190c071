#!/bin/bash
# Source-sampler stage stamps at cfg5 (an SBZ_TB_STAMP=1 build: tools/build_src_variant.sh tbst
# -DSBZ_TB_STAMP=1), per operator set.  Usage: bash tools/src_stamps_r06.sh [LIB_NAME] [SETS]
set -u
lib=${1:-tbst}
for s in ${2:-p_zones weights p_families zone_moves}; do
  SBZ_LIB_PATH=$PWD/contact_zones_amd/libsbz_$lib.so timeout -k 10 300 python -u tools/tb_stamps.py 100 $s 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done
