"""TOOL: the bench line's timed launches read back from a rocprofv3 kernel trace of the same command.

    rocprofv3 --kernel-trace --output-format csv -d D -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > b.log
    python tools/trace_window.py D b.log [--keep OUT.csv]
    python tools/trace_window.py OUT.csv b.log          (the same figures from a kept file)

bench.py's headline leg is the run's LAST K step_kernel dispatches (W warm-up launches before them); the configs[4]
Philox + one-hot leg's K timed launches come before the headline's chip warm-up.  For each leg this prints the
mean dispatch duration of those K launches and their span / K (first start to last end -- what the line's HIP-event
kernel_ms measures: back-to-back launches, gaps included), beside the line's kernel_ms, and writes the step_kernel
rows (name, start, end) to --keep so the figure is reproducible from a committed file.
"""
import csv
import glob
import json
import os
import sys


def load_rows(d):
    rows = []
    if d.endswith(".csv"):   # a --keep file (committed under profiles/): start_ns,end_ns,kernel
        with open(d) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["start_ns"]), int(r["end_ns"]), r["kernel"]))
        rows.sort()
        return rows
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name", "")
                if "step_kernel" in name:
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    return rows


def window(rows, k):
    """The last k dispatches: their mean duration, their span / k, and the span of dispatches 2..k / (k - 1) -- the
    window bench.py's HIP events bracket (an event before launch 1 would time its host enqueue latency too)."""
    dur = [e - s for s, e, _ in rows[-k:]]
    return {"launches": len(dur), "mean_dispatch_us": sum(dur) / len(dur) / 1e3,
            "span_over_k_us": (rows[-1][1] - rows[-k][0]) / k / 1e3,
            "span_2_to_k_us": (rows[-1][1] - rows[-k][1]) / max(k - 1, 1) / 1e3, "kernel": rows[-1][2][:120]}


def main():
    d, log = sys.argv[1], sys.argv[2]
    keep = sys.argv[sys.argv.index("--keep") + 1] if "--keep" in sys.argv else None
    line = None
    for ln in open(log):
        if ln.startswith("{"):
            line = json.loads(ln)
    rows = load_rows(d)
    if keep:   # the last 100 dispatches of every step_kernel instantiation (the timed windows are among them)
        last = {}
        for r in rows:
            last.setdefault(r[2], []).append(r)
        kept = sorted(r for v in last.values() for r in v[-100:])
        with open(keep, "w") as fh:
            fh.write("start_ns,end_ns,kernel\n")
            for s, e, n in kept:
                fh.write(f"{s},{e},\"{n}\"\n")
    K = line["steps"] if line else 20
    out = {"headline": window(rows, K)}
    if line:
        out["headline"]["line_kernel_us"] = line["roofline"]["kernel_ms"] * 1e3
        out["headline"]["span_vs_line"] = out["headline"]["span_2_to_k_us"] / out["headline"]["line_kernel_us"]
        alg = line["roofline"]["algorithmic_bytes_per_launch"]
        out["headline"]["frac_from_span"] = alg / (out["headline"]["span_2_to_k_us"] * 1e-6) / 8e12
        out["headline"]["frac_from_mean_dispatch"] = alg / (out["headline"]["mean_dispatch_us"] * 1e-6) / 8e12
        c4 = line.get("configs4_onehot_philox")
        if c4 and "roofline" in c4:
            # the configs[4] leg: the K launches of the other step_kernel instantiation (Philox + one-hot) that
            # come last among its dispatches
            name4 = None
            for s, e, n in rows:
                if n != rows[-1][2]:
                    name4 = n
            sub = [r for r in rows if r[2] == name4] if name4 else []
            if len(sub) >= K:
                w4 = window(sub, K)
                w4["line_kernel_us"] = c4["roofline"]["kernel_ms"] * 1e3
                w4["span_vs_line"] = w4["span_2_to_k_us"] / w4["line_kernel_us"]
                a4 = c4["roofline"]["algorithmic_bytes_per_launch"]
                w4["frac_from_span"] = a4 / (w4["span_2_to_k_us"] * 1e-6) / 8e12
                w4["frac_from_mean_dispatch"] = a4 / (w4["mean_dispatch_us"] * 1e-6) / 8e12
                out["configs4"] = w4
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
