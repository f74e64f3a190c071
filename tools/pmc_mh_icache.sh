#!/bin/bash
# Instruction-fetch PMC of the mixture sampler (mh_kernel, cfg5, 256 chains, default operators,
# tools/mh_optime.py): I-cache requests / misses and wave-cycle buckets, one rocprofv3 pass each.
# Usage: bash tools/pmc_mh_icache.sh [TAG]   (library: SBZ_LIB_PATH or the in-tree libsbz.so)
set -u
export TMPDIR=/tmp
tag=${1:-base}
OUT=gpurun_out/pmc_ic_$tag
mkdir -p $OUT
i=0
for pass in \
  "SQC_ICACHE_REQ SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-trace -d $OUT/p$i -o run --output-format csv -- python3 tools/mh_optime.py --steps 3000 --sets default > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(int)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if "mh_kernel" not in k:
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    print(k[:60])
    for c, v in sorted(d.items()):
        print(f"  {c:32s} {v:.4g}")
    if d.get("SQC_ICACHE_REQ"):
        print(f"  icache miss rate {d.get('SQC_ICACHE_MISSES', 0) / d['SQC_ICACHE_REQ']:.3f}")
PY
