"""TOOL: summarise tools/step_window_pmc.sh -- per counter, the mean over the last 20 step_kernel dispatches after
S = 5 and S = 40 untimed steps, their ratio, and the S = 5 series (launch by launch) to show the trend."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/swp/swp"
res = {}
for S in (5, 40):
    vals = defaultdict(dict)
    for f in glob.glob(os.path.join(root, f"*{S}", "**", "*counter_collection.csv"), recursive=True):
        if not os.path.basename(os.path.dirname(f)).endswith(str(S)) and f"{S}/" not in f:
            continue
        for r in csv.DictReader(open(f)):
            if "step_kernel" not in r["Kernel_Name"]:
                continue
            d = int(r["Dispatch_Id"])
            vals[r["Counter_Name"]][d] = vals[r["Counter_Name"]].get(d, 0.0) + float(r["Counter_Value"])
    res[S] = vals
for c in sorted(set(res[5]) | set(res[40])):
    out = {"counter": c}
    for S in (5, 40):
        dv = res[S].get(c, {})
        last = [dv[k] for k in sorted(dv)[-20:]]
        out[f"S{S}"] = round(sum(last) / len(last), 1) if last else None
        if S == 5 and dv:
            out["S5_series"] = [round(dv[k], 1) for k in sorted(dv)][-20:]
    if out.get("S5") and out.get("S40"):
        out["ratio_5_40"] = round(out["S5"] / out["S40"], 3)
    print(json.dumps(out))
