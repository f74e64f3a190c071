#!/bin/bash
# PMC passes of the SAMPLE_SOURCE = true sampler at the cfg5 shape (2000x500x10, Z8, Fam4, 256
# chains, sources in HBM, the table passes) under one operator set of tools/src_optime.py (default:
# the reference's STEPS): one launch of STEPS steps after the one-step GPU source draw, each counter
# pass its own rocprofv3 run (--pmc never combined with sys/runtime traces).
# Usage: bash tools/pmc_src.sh [SET] [STEPS]; summary in $PMC_OUT/pmc.json (default gpurun_out/pmc_src),
# whose _meta.src_steps_total (STEPS + 1) turns the per-dispatch means into per-step figures.
set -u
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc_src}
SET=${1:-default}
STEPS=${2:-2000}
mkdir -p $OUT
i=0
for pass in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU" \
  "FETCH_SIZE GRBM_GUI_ACTIVE" \
  "WRITE_SIZE TCC_HIT TCC_MISS" ; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $pass --kernel-trace -d $OUT/p$i -o run --output-format csv -- python3 tools/src_optime.py --sites 2000 --features 500 --states 10 --zones 8 --families 4 --chains 256 --steps $STEPS --burnin 0 --sets $SET --gpu-init > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
PMC_META="{\"workload\": \"cfg5 source sampler 2000x500x10 Z8 Fam4, 256 chains, set $SET\", \"src_set\": \"$SET\", \"src_steps_total\": $((STEPS + 1)), \"src_chains\": 256}" python3 tools/pmc_summary.py $OUT
