"""TOOL: summarise the PMC passes of tools/gpu.sh (pmc_refconf / pmc_configs2; also round 3/4's tools/pmc_grad.sh
layout) for the update / rollout kernels -- per kernel: dispatches, time, MFMA busy cycles against the MFMA-cycle
capacity of the dispatch (duration x 2.4 GHz x 1,024 SIMDs, and x the clock the chip held: GRBM_GUI_ACTIVE / 8 XCDs),
HBM bytes (FETCH_SIZE x 2 KiB units -- gfx950 reports half of streaming reads -- + WRITE_SIZE KiB), and every other
counter of the passes that ran (SQ waits per wave-cycle, LDS bank conflicts per LDS-array cycle, TCC hit rate).

    python tools/pmc_grad_summary.py [gpurun_out/pmc_grad]
"""
import collections
import csv
import json
import os
import sys

D = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_grad"
CLOCK_GHZ, SIMDS = 2.4, 1024
KERNELS = ("grad_coop_kernel", "deep_grad_kernel", "deep_rollout_kernel", "deep_policy_kernel", "onehot_dw1_mfma_kernel", "onehot_dw1_ring_kernel", "onehot_dw1_kernel",
           "onehot_l0_mfma_kernel",
           "onehot_l1_kernel", "dw2_kernel", "fold_kernel", "grad_kernel", "policy_kernel", "rollout_kernel", "Cijk")


def kname(n):
    for k in KERNELS:
        if k in n:
            return k
    return None


def per_kernel(path):
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    if not os.path.exists(path):
        return out
    for r in csv.DictReader(open(path)):
        k = kname(r["Kernel_Name"])
        if k:
            out[k][r["Counter_Name"]] += float(r["Counter_Value"])
    return out


passes = {p: per_kernel(os.path.join(D, p, "run_counter_collection.csv")) for p in ("sq", "sqw", "fetch", "write", "tcc")}
dur = collections.defaultdict(float)
calls = collections.Counter()
for r in csv.DictReader(open(os.path.join(D, "trace", "run_kernel_trace.csv"))):
    k = kname(r["Kernel_Name"])
    if k:
        dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        calls[k] += 1
for k in sorted(dur, key=lambda k: -dur[k]):
    sq, sqw, tcc = passes["sq"][k], passes["sqw"][k], passes["tcc"][k]
    cap = dur[k] * CLOCK_GHZ * 1e9 * SIMDS
    fetch = passes["fetch"][k].get("FETCH_SIZE", 0.0) * 1024 * 2
    write = passes["write"][k].get("WRITE_SIZE", 0.0) * 1024
    mfma = sq.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    grbm = sq.get("GRBM_GUI_ACTIVE", 0.0)
    rec = {"kernel": k, "dispatches": calls[k], "seconds": round(dur[k], 4),
           "mfma_busy_frac": round(mfma / cap, 3) if cap else None,
           # the same busy cycles against the clock the chip held (GRBM_GUI_ACTIVE / 8 XCDs per dispatch)
           "clock_GHz": round(grbm / 8 / dur[k] / 1e9, 3) if dur[k] and grbm else None,
           "mfma_busy_frac_at_clock": round(mfma / (grbm / 8 * SIMDS), 3) if grbm else None,
           "hbm_fetch_GB": round(fetch / 1e9, 2), "hbm_write_GB": round(write / 1e9, 2),
           "hbm_GBps": round((fetch + write) / dur[k] / 1e9, 1) if dur[k] else None}
    wc = sqw.get("SQ_WAVE_CYCLES")
    if wc:   # quad-cycle buckets per wave-cycle (disjoint: wait + issue-stall + active ~= 1)
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if c in sqw:
                rec[c.lower() + "_frac"] = round(sqw[c] / wc, 3)
        if "SQ_VALU_MFMA_COEXEC_CYCLES" in sqw and mfma:
            rec["mfma_coexec_frac_of_busy"] = round(sqw["SQ_VALU_MFMA_COEXEC_CYCLES"] / mfma, 3)
    if sq.get("SQ_LDS_IDX_ACTIVE"):
        rec["lds_bank_conflict_frac"] = round(sq.get("SQ_LDS_BANK_CONFLICT", 0.0) / sq["SQ_LDS_IDX_ACTIVE"], 3)
    if tcc.get("TCC_HIT_sum", 0) + tcc.get("TCC_MISS_sum", 0):
        rec["tcc_hit_rate"] = round(tcc["TCC_HIT_sum"] / (tcc["TCC_HIT_sum"] + tcc["TCC_MISS_sum"]), 3)
        rec["tcc_requests"] = tcc["TCC_HIT_sum"] + tcc["TCC_MISS_sum"]
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_WAVES", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
        v = sq.get(c, sqw.get(c))
        if v is not None:
            rec[c.lower()] = v
    rec["mfma_busy_cycles"] = mfma
    print(json.dumps(rec))
