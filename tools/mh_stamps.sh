#!/bin/bash
# Sampler phase stamps (SBZ_MH_STAMP builds of revision d12ba3a, the last with the instrumentation:
# tools/build_rev.sh d12ba3a stK -DSBZ_MH_STAMP=K): mean
# shader cycles per step of each phase / sub-phase, by operator, at the bench's cfg5 shape.
mkdir -p gpurun_out
for k in ${KS:-1 2 3 4 5 6 7 8 9 10 11 12}; do
  echo "# SBZ_MH_STAMP=$k" >> gpurun_out/mh_stamps.txt
  SBZ_LIB_PATH=$PWD/contact_zones_amd/libsbz_st$k.so timeout -k 10 120 python tools/mh_optime.py --stamps --steps 1000 --sets default >> gpurun_out/mh_stamps.txt 2>&1 || exit 1
done
cat gpurun_out/mh_stamps.txt | grep -v "^default"
