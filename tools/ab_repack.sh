#!/bin/bash
# Per-kernel A/B of libsbz variants on the source-branch bench (rocprofv3 kernel stats).
#   tools/ab_repack.sh SPEC...   SPEC = variant[:ENV=VAL[,ENV=VAL]]  ("default" = contact_zones_amd/libsbz.so)
set -o pipefail
for spec in "$@"; do
    v=${spec%%:*}
    envs=""
    [[ $spec == *:* ]] && envs=${spec#*:}
    for kv in ${envs//,/ }; do export "$kv"; done
    lib=$PWD/contact_zones_amd/libsbz.so
    [ "$v" != "default" ] && lib=$PWD/contact_zones_amd/libsbz_$v.so
    tag=$(echo "$spec" | tr ':=,' '___')
    export SBZ_LIB_PATH=$lib SBZ_ALLOW_NONFINITE=1
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/abr_$tag -o rp --output-format csv -- \
        python3 bench.py --mode source --steps 50 --warmup 5 --cpu-seconds 1 --mh-steps 0 --src-steps 0 \
        --source-lik-steps 0 > gpurun_out/abr_$tag.log 2>&1 || { echo "$spec failed"; tail -5 gpurun_out/abr_$tag.log; exit 1; }
    python3 - "$tag" <<'PY'
import csv, glob, re, sys
f = glob.glob(f"gpurun_out/abr_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "sbz" in r["Name"]:
        print(sys.argv[1], re.search(r"\w+_kernel(<[^>]*>)?", r["Name"]).group(0), r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
    for kv in ${envs//,/ }; do unset "${kv%%=*}"; done
done
