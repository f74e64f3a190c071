#!/bin/bash
# Round-6 sampler timing on one GPU box: mixture sampler per operator family (tools/mh_optime.py)
# and the source-mode sampler at cfg5 / Balkan shapes (tools/src_optime.py).  Stops at the first
# failure.  Usage: bash tools/optime_r06.sh TAG [MH_SETS] [SRC_SETS]
set -u
tag=${1:-base}; mh_sets=${2:-default,weights,p_global,p_zones,p_families,zone_moves}; src_sets=${3:-default}
mkdir -p gpurun_out
run() { echo "== $*" >&2; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
if [ "$mh_sets" != none ]; then
  run timeout -k 10 300 python -u tools/mh_optime.py --steps 3000 --sets $mh_sets > gpurun_out/mh_optime_$tag.txt 2>&1
  cat gpurun_out/mh_optime_$tag.txt | grep -v '^{'
fi
if [ "$src_sets" != none ]; then
  run timeout -k 10 300 python -u tools/src_optime.py --sites 2000 --features 500 --states 10 --zones 8 --families 4 --chains 256 --steps 1000 --gpu-init --sets $src_sets > gpurun_out/src_optime_$tag.txt 2>&1
  cat gpurun_out/src_optime_$tag.txt | grep -v '^{'
fi
