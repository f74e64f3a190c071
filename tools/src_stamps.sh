#!/bin/bash
# Source-mode sampler phase stamps (SBZ_SRC_STAMP builds of revision d12ba3a, the last with the
# instrumentation: tools/build_rev.sh d12ba3a sst<k> -DSBZ_SRC_STAMP=<k>; KS selects which were built): the production library first, then each k,
# on the Balkan- and South-America-shaped synthetic legs.
mkdir -p gpurun_out
: > gpurun_out/src_stamps.txt
for shp in "--sites 28 --features 47 --states 3 --zones 3 --families 5 --chains 256" "--sites 100 --features 36 --states 5 --zones 6 --families 6 --chains 128"; do
  echo "## $shp" >> gpurun_out/src_stamps.txt
  echo "# production" >> gpurun_out/src_stamps.txt
  timeout -k 10 120 python tools/src_stamps.py $shp >> gpurun_out/src_stamps.txt 2>/dev/null || exit 1
  for k in ${KS:-1 2 9 10 11}; do
    echo "# SBZ_SRC_STAMP=$k" >> gpurun_out/src_stamps.txt
    SBZ_LIB_PATH=$PWD/contact_zones_amd/libsbz_sst$k.so timeout -k 10 120 python tools/src_stamps.py $shp >> gpurun_out/src_stamps.txt 2>/dev/null || exit 1
  done
done
cat gpurun_out/src_stamps.txt
