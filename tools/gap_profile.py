"""TOOL: where the GPU sits idle inside a window of a rocprofv3 kernel trace (host-bound gaps between launches).

    rocprofv3 --kernel-trace --output-format csv -d D -o run -- python3 tools/bench_refconfig.py --episodes 1048576
    python tools/gap_profile.py D [--after KERNEL_SUBSTR] [--before KERNEL_SUBSTR] [--durations KERNEL_SUBSTR]

The window: from the LAST dispatch whose name contains --after (default: the last update's first gradient kernel,
'onehot_l0_mfma_kernel') to the end of the trace.  Prints the window's span, the summed dispatch time (union of
intervals), the idle time, and the idle gaps grouped by the kernel that ends them (the host work in front of it).
--durations: also the launches of that kernel in the window by duration bucket (count, summed time) -- how much of
its time is in launches too short to fill the chip.
"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    after = sys.argv[sys.argv.index("--after") + 1] if "--after" in sys.argv else "onehot_l0_mfma_kernel"
    before = sys.argv[sys.argv.index("--before") + 1] if "--before" in sys.argv else None
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # the window starts at the first dispatch of the last run of `after` kernels: walk back from the last one while
    # the gap to the previous `after` dispatch is short (same update)
    idx = [i for i, r in enumerate(rows) if after in r[2]]
    if not idx:
        print("no dispatch named", after)
        return
    start_i = idx[-1]
    for a, b in zip(reversed(idx[:-1]), reversed(idx[1:])):
        if rows[b][0] - rows[a][1] > 50_000_000:   # 50 ms: a previous update
            break
        start_i = a
    win = rows[start_i:]
    if before:
        end = [i for i, r in enumerate(win) if before in r[2]]
        if end:
            win = win[:end[-1] + 1]
    t0, t_end = win[0][0], max(r[1] for r in win)
    busy, cur_s, cur_e = 0, win[0][0], win[0][1]
    gaps = collections.Counter()
    ngaps = collections.Counter()
    per_kernel = collections.Counter()
    for s, e, n in win:
        per_kernel[n[:90]] += e - s
    for s, e, n in win[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps[n[:90]] += s - cur_e
            ngaps[n[:90]] += 1
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = t_end - t0
    print(f"window: {len(win)} dispatches, span {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms, "
          f"idle {(span - busy) / 1e6:.2f} ms ({(span - busy) / span:.1%})")
    print("kernel time in the window:")
    for n, t in per_kernel.most_common(12):
        print(f"  {t / 1e6:9.2f} ms  {n}")
    print("idle gaps by the kernel that ends them:")
    for n, t in gaps.most_common(15):
        print(f"  {t / 1e6:9.2f} ms in {ngaps[n]:6d} gaps  before {n}")
    if "--durations" in sys.argv:
        k = sys.argv[sys.argv.index("--durations") + 1]
        edges = [0, 20, 50, 100, 200, 500, 1000, 2000, 5000, float("inf")]
        cnt, tot = collections.Counter(), collections.Counter()
        for s, e, n in win:
            if k in n:
                us = (e - s) / 1e3
                b = next(i for i in range(len(edges) - 1) if us < edges[i + 1])
                cnt[b] += 1
                tot[b] += us
        print(f"launches of {k} by duration:")
        for b in range(len(edges) - 1):
            if cnt[b]:
                print(f"  {edges[b]:6.0f} - {edges[b + 1]:6.0f} us: {cnt[b]:6d} launches, {tot[b] / 1e3:9.2f} ms")


if __name__ == "__main__":
    main()
