set -u
mkdir -p gpurun_out
for k in ${KS:-1 2 3}; do
  SBZ_LIB_PATH=$PWD/contact_zones_amd/libsbz_st$k.so timeout -k 10 300 python -u tools/mh_optime.py --steps 3000 --stamps --sets default,weights > gpurun_out/mhst$k.log 2>&1 || { tail -5 gpurun_out/mhst$k.log; exit 1; }
  echo "## stamp $k"; tail -1 gpurun_out/mhst$k.log
done
