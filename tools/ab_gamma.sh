for r in 1 2; do VARIANTS="default g1" bash tools/ab_mh_variants.sh; done
for r in 1 2; do for v in default sg1; do lib=$PWD/contact_zones_amd/libsbz.so; [ $v != default ] && lib=$PWD/contact_zones_amd/libsbz_$v.so
 echo -n "$v "; SBZ_LIB_PATH=$lib timeout -k 10 200 python tools/src_optime.py --sets default 2>/dev/null | tail -1 | cut -c1-200
 echo -n "$v SA "; SBZ_LIB_PATH=$lib timeout -k 10 200 python tools/src_optime.py --sets default --sites 100 --features 36 --states 5 --zones 6 --families 6 --chains 128 2>/dev/null | tail -1 | cut -c1-200; done; done
