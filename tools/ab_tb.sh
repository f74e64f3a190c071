for v in ${VARIANTS:-default}; do
  lib=$PWD/contact_zones_amd/libsbz.so; [ $v != default ] && lib=$PWD/contact_zones_amd/libsbz_$v.so
  SBZ_LIB_PATH=$lib timeout -k 10 200 python -u tools/src_optime.py --sites 2000 --features 500 --states 10 --zones 8 --families 4 --chains 256 --steps 60 --burnin 0 --sets zone_moves 2>&1 | grep -v amdgpu.ids | head -1 | sed "s/^/$v /" || exit 1
done
