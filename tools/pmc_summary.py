"""Average rocprofv3 PMC counters per dispatch for each sbz kernel (tools/pmc.sh output).

Prints a table and writes <out>/pmc.json:
  {kernel: {counter: mean_per_dispatch, ...}, "_hbm": {...}} where "_hbm" holds the dominant
mixture kernel's HBM traffic per launch, corrected as MI355X_MICROARCH.md (HBM section)
prescribes: FETCH_SIZE (KB) is doubled on gfx950 (calibrated for 16-B/lane streaming reads;
this kernel's 4-8-B/lane loads are outside the calibrated case, so the absolute is approximate),
WRITE_SIZE (KB) taken as is.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = defaultdict(lambda: defaultdict(list))
for fn in sorted(glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True)):
    with open(fn) as f:
        for row in csv.DictReader(f):
            k = row.get("Kernel_Name", "?")
            if "sbz" not in k:
                continue
            short = k.replace("void ", "").replace("sbz::(anonymous namespace)::", "").split("(")[0]
            vals[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
summary = {}
for k, d in vals.items():
    print(k)
    summary[k] = {}
    for c, v in sorted(d.items()):
        m = sum(v) / len(v)
        summary[k][c] = m
        summary[k]["_dispatches"] = len(v)
        print(f"  {c:28s} mean {m:.6g}  (n={len(v)})")
mix = [k for k in summary if "mixture_kernel" in k or "zoned_kernel" in k]
if mix:
    k = max(mix, key=lambda n: summary[n].get("GRBM_GUI_ACTIVE", 0))
    s = summary[k]
    fetch = s.get("FETCH_SIZE", 0.0) * 1024 * 2
    write = s.get("WRITE_SIZE", 0.0) * 1024
    hit, miss = s.get("TCC_HIT", 0.0), s.get("TCC_MISS", 0.0)
    summary["_hbm"] = {"kernel": k, "fetch_bytes": fetch, "write_bytes": write,
                       "traffic_bytes": fetch + write,
                       "l2_hit_rate": hit / (hit + miss) if hit + miss else None,
                       "lds_bank_conflict_frac": (s.get("SQ_LDS_BANK_CONFLICT", 0) /
                                                  s["SQ_LDS_IDX_ACTIVE"]) if s.get("SQ_LDS_IDX_ACTIVE") else None,
                       "valu_insts_per_wave": (s.get("SQ_INSTS_VALU", 0) / s["SQ_WAVES"]) if s.get("SQ_WAVES") else None,
                       "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM); WRITE_SIZE x1"}
    print("HBM per launch:", json.dumps(summary["_hbm"]))
# every kernel's HBM traffic per dispatch (same correction), LDS conflicts, VALU per wave, waits
summary["_per_kernel"] = {}
for k, s in summary.items():
    if k.startswith("_") or not isinstance(s, dict):
        continue
    e = {"dispatches": s.get("_dispatches")}
    if "FETCH_SIZE" in s or "WRITE_SIZE" in s:
        e["fetch_bytes"] = s.get("FETCH_SIZE", 0.0) * 1024 * 2
        e["write_bytes"] = s.get("WRITE_SIZE", 0.0) * 1024
        e["traffic_bytes"] = e["fetch_bytes"] + e["write_bytes"]
    if s.get("SQ_LDS_IDX_ACTIVE"):
        e["lds_bank_conflict_frac"] = s.get("SQ_LDS_BANK_CONFLICT", 0) / s["SQ_LDS_IDX_ACTIVE"]
    if s.get("SQ_WAVES"):
        e["valu_insts_per_wave"] = s.get("SQ_INSTS_VALU", 0) / s["SQ_WAVES"]
        e["lds_insts_per_wave"] = s.get("SQ_INSTS_LDS", 0) / s["SQ_WAVES"]
    if s.get("SQ_WAVE_CYCLES"):
        e["wait_any_frac"] = s.get("SQ_WAIT_ANY", 0) / s["SQ_WAVE_CYCLES"]
        e["active_inst_any_frac"] = s.get("SQ_ACTIVE_INST_ANY", 0) / s["SQ_WAVE_CYCLES"]
        e["wait_inst_lds_frac"] = s.get("SQ_WAIT_INST_LDS", 0) / s["SQ_WAVE_CYCLES"]
    if s.get("TCC_HIT", 0) + s.get("TCC_MISS", 0):
        e["l2_hit_rate"] = s["TCC_HIT"] / (s["TCC_HIT"] + s["TCC_MISS"])
    summary["_per_kernel"][k] = e
    print(k, json.dumps(e))
# the profiled bench run's workload (its JSON line in the pass logs), so bench.py can match it
meta = {"command": "bash tools/pmc.sh (rocprofv3 --pmc <pass> --kernel-trace -- python3 bench.py ...)"}
# the kernel sources the counters were measured on (bench.py uses the counters only for the same sources)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
try:
    import bench
    meta["source_hash"] = bench.kernel_source_hash()
except Exception as e:  # pragma: no cover
    meta["source_hash_error"] = repr(e)
for log in sorted(glob.glob(os.path.join(out, "p*.log"))):
    for line in open(log):
        if line.startswith("{"):
            try:
                cfg = json.loads(line)["config"]
                meta["workload_key"] = cfg.get("workload_key")
                meta["workload"] = cfg.get("workload")
            except (ValueError, KeyError):
                pass
if os.environ.get("PMC_META"):  # extra _meta fields of the caller (tools/pmc_src.sh)
    meta.update(json.loads(os.environ["PMC_META"]))
summary["_meta"] = meta
json.dump(summary, open(os.path.join(out, "pmc.json"), "w"), indent=1)
