"""TOOL: summarise tools/pmc_grad.sh's passes for the update kernels -- per kernel: dispatches, time, MFMA busy
cycles against the MFMA-cycle capacity of the dispatch (duration x 2.4 GHz x 1,024 SIMDs, and x the clock the
chip held: GRBM_GUI_ACTIVE / 8 XCDs), HBM bytes
(FETCH_SIZE x 2 KiB units -- gfx950 reports half of streaming reads -- + WRITE_SIZE KiB).

    python tools/pmc_grad_summary.py [gpurun_out/pmc_grad]
"""
import collections
import csv
import json
import os
import sys

D = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_grad"
CLOCK_GHZ, SIMDS = 2.4, 1024


def kname(n):
    for k in ("grad_coop_kernel", "grad_kernel", "dw2_kernel", "fold_kernel", "policy_kernel", "rollout_kernel", "Cijk"):
        if k in n:
            return k
    return None


def per_kernel(path):
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        k = kname(r["Kernel_Name"])
        if k:
            out[k][r["Counter_Name"]] += float(r["Counter_Value"])
    return out


sq = per_kernel(os.path.join(D, "sq", "run_counter_collection.csv"))
fe = per_kernel(os.path.join(D, "fetch", "run_counter_collection.csv"))
wr = per_kernel(os.path.join(D, "write", "run_counter_collection.csv"))
dur = collections.defaultdict(float)
calls = collections.Counter()
for r in csv.DictReader(open(os.path.join(D, "trace", "run_kernel_trace.csv"))):
    k = kname(r["Kernel_Name"])
    if k:
        dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        calls[k] += 1
for k in sorted(dur):
    cap = dur[k] * CLOCK_GHZ * 1e9 * SIMDS
    fetch = fe[k].get("FETCH_SIZE", 0.0) * 1024 * 2
    write = wr[k].get("WRITE_SIZE", 0.0) * 1024
    print(json.dumps({"kernel": k, "dispatches": calls[k], "seconds": round(dur[k], 4),
                      "mfma_busy_cycles": sq[k].get("SQ_VALU_MFMA_BUSY_CYCLES"),
                      "mfma_busy_frac": round(sq[k].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / cap, 3) if cap else None,
                      # the same busy cycles against the clock the chip held (GRBM_GUI_ACTIVE / 8 XCDs per dispatch)
                      "clock_GHz": round(sq[k].get("GRBM_GUI_ACTIVE", 0.0) / 8 / dur[k] / 1e9, 3) if dur[k] else None,
                      "mfma_busy_frac_at_clock": round(sq[k].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
                                                       / (sq[k].get("GRBM_GUI_ACTIVE", 0.0) / 8 * SIMDS), 3)
                      if sq[k].get("GRBM_GUI_ACTIVE") else None,
                      "valu_insts": sq[k].get("SQ_INSTS_VALU"), "waves": sq[k].get("SQ_WAVES"),
                      "hbm_fetch_GB": round(fetch / 1e9, 2), "hbm_write_GB": round(write / 1e9, 2),
                      "hbm_GBps": round((fetch + write) / dur[k] / 1e9, 1) if dur[k] else None}))
