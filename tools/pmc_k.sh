#!/bin/bash
# Two SQ PMC passes of the mixture bench for each SBZ_LIK_KERNEL value given:
#   bash tools/pmc_k.sh count dense ...   -> gpurun_out/pmck/<kernel>/p{1,2} + summary
set -u
export TMPDIR=/tmp
OUT=gpurun_out/pmck
mkdir -p $OUT
for k in "$@"; do
  i=0
  for pass in \
    "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
    "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU"; do
    i=$((i+1))
    SBZ_LIK_KERNEL=$k timeout -k 10 120 rocprofv3 --pmc $pass --kernel-trace -d $OUT/$k/p$i -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --cpu-seconds 0 --mh-steps 0 --src-steps 0 > $OUT/$k.p$i.log 2>&1 || { echo "pmc $k pass $i failed"; tail -5 $OUT/$k.p$i.log; exit 1; }
  done
  echo "== $k"; python3 tools/pmc_summary.py $OUT/$k | grep -v "^HBM"
done
