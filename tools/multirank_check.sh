#!/bin/bash
# The experiment CLI (python -m contact_zones_amd) as one process and as 2 torchrun ranks on the
# same seed: the chains shard over the ranks (Philox keyed by global chain id, initial samples from
# the agreed seed), so the results files must be byte-identical.  On a one-GPU box both ranks share
# the GPU, which RCCL refuses, so the rehearsal runs the collectives over gloo (SBZ_DIST_BACKEND);
# on a multi-GPU node leave it unset (nccl = RCCL).
set -u
OUT=${OUT:-$PWD/gpurun_out/multirank}
rm -rf "$OUT"; mkdir -p "$OUT"
CFG=tests/golden/io/data/experiments/balkan/config.json
SRC=${SRC:-false}
SET="{\"model\":{\"N_AREAS\":2,\"SAMPLE_SOURCE\":$SRC},\"mcmc\":{\"N_STEPS\":4000,\"N_SAMPLES\":40,\"WARM_UP\":{\"N_WARM_UP_STEPS\":1000,\"N_WARM_UP_CHAINS\":7}},\"results\":{\"RESULTS_PATH\":\"$OUT\"}}"
timeout -k 10 300 python -m contact_zones_amd "$CFG" --name single --seed 7 --set "$SET" > "$OUT/single.log" 2>&1 || { echo "single run failed"; tail -20 "$OUT/single.log"; exit 1; }
SBZ_DIST_BACKEND=${SBZ_DIST_BACKEND:-gloo} timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node ${NPROC:-2} \
    --master-addr 127.0.0.1 --master-port ${PORT:-29611} -m contact_zones_amd "$CFG" --name ranks --seed 7 --set "$SET" \
    > "$OUT/ranks.log" 2>&1 || { echo "torchrun failed"; tail -30 "$OUT/ranks.log"; exit 1; }
n=0
for f in $(cd "$OUT/single" && find . -type f | sort); do
  cmp "$OUT/single/$f" "$OUT/ranks/$f" || { echo "DIFFER: $f"; exit 1; }
  n=$((n + 1))
done
[ "$n" -gt 0 ] || { echo "no results files"; exit 1; }
echo "multirank ok: $n results files byte-identical (1 process vs ${NPROC:-2} ranks)"
