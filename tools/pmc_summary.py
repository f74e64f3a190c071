"""Average rocprofv3 PMC counters per dispatch for each kernel (tools/pmc.sh output)."""
import csv
import glob
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
for k, d in vals.items():
    print(k)
    for c, v in sorted(d.items()):
        # several rows per dispatch (one per XCD / instance) are summed by rocprofv3 already
        print(f"  {c:28s} mean {sum(v)/len(v):.6g}  (n={len(v)})")
