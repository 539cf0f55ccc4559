"""Summarise tools/r4_state_pmc.sh: per counter, the mean over the last 20 step_kernel dispatches, S = 5 vs 40."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r4sp"
for S in (5, 40):
    vals = defaultdict(dict)
    for f in glob.glob(f"{root}/*{S}/**/*counter_collection.csv", recursive=True):
        if not any(f"/{p}{S}/" in f for p in ("sq", "f", "w", "wr")):
            continue
        for r in csv.DictReader(open(f)):
            if "step_kernel" not in r["Kernel_Name"]:
                continue
            d = int(r["Dispatch_Id"])
            vals[r["Counter_Name"]][d] = vals[r["Counter_Name"]].get(d, 0.0) + float(r["Counter_Value"])
    out = {}
    for c, dv in sorted(vals.items()):
        last = [dv[k] for k in sorted(dv)[-20:]]
        out[c] = sum(last) / len(last)
    print(S, {k: f"{v:.4g}" for k, v in out.items()})
