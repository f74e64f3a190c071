#!/bin/bash
# Per-kernel A/B of libsbz variants on the source-branch bench (rocprofv3 kernel stats).
#   tools/ab_repack.sh VARIANT...   ("default" = contact_zones_amd/libsbz.so)
set -o pipefail
for v in "$@"; do
    lib=$PWD/contact_zones_amd/libsbz.so
    [ "$v" != "default" ] && lib=$PWD/contact_zones_amd/libsbz_$v.so
    export SBZ_LIB_PATH=$lib SBZ_ALLOW_NONFINITE=1
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/abr_$v -o rp --output-format csv -- \
        python3 bench.py --mode source --steps 50 --warmup 5 --cpu-seconds 1 --mh-steps 0 --src-steps 0 \
        --source-lik-steps 0 > gpurun_out/abr_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/abr_$v.log; exit 1; }
    python3 - "$v" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/abr_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "sbz" in r["Name"]:
        print(sys.argv[1], r["Name"].split("(")[0].split("::")[-1][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
