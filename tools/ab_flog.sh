#!/bin/bash
# flog() / fdiv_pos() on the samplers' critical paths against the library log and division:
# MH_VARIANTS for the cfg5 mixture sampler step time (e.g. dlog0: the delta as the library's
# log(mn / mo), tools/build_mh_variant.sh dlog0 -DSBZ_MH_DLOG=0), SRC_VARIANTS for the
# source-mode sampler on the Balkan / South America shapes (e.g. noflog:
# tools/build_all_variant.sh noflog -DSBZ_FLOG=0); two alternated rounds.
libof() { if [ $1 = default ]; then echo $PWD/contact_zones_amd/libsbz.so; else echo $PWD/contact_zones_amd/libsbz_$1.so; fi; }
for r in 1 2; do
  for v in ${MH_VARIANTS:-default dlog0}; do
    echo -n "$v mh "; SBZ_LIB_PATH=$(libof $v) timeout -k 10 200 python tools/mh_optime.py --steps 2000 --sets default,weights 2>&1 | tail -1 || exit 1
  done
  for v in ${SRC_VARIANTS:-default noflog}; do
    echo -n "$v src_balkan "; SBZ_LIB_PATH=$(libof $v) timeout -k 10 200 python tools/bench_source_sampler.py --sites 28 --features 47 --states 3 --zones 3 --families 5 --chains 256 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['us_per_step'],3), round(d['ess_per_sec']))" || exit 1
    echo -n "$v src_sa "; SBZ_LIB_PATH=$(libof $v) timeout -k 10 200 python tools/bench_source_sampler.py 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['us_per_step'],3), round(d['ess_per_sec']))" || exit 1
  done
done
