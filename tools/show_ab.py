"""TOOL: summarise an A/B log of bench.py runs (tools/ab_libs.sh): kernel us and frac per library and mode."""
import collections
import json
import sys

cur = None
res = collections.defaultdict(list)
for line in open(sys.argv[1]):
    if line.startswith("== "):
        cur = line[3:].strip()
    elif line.startswith("{") and cur:
        d = json.loads(line)
        res[cur].append((d["roofline"]["kernel_ms"] * 1e3, d["roofline"]["frac"], d["value"]))
for k, v in res.items():
    us = [round(x[0], 2) for x in v]
    print(f"{k}: kernel_us {us} frac {[round(x[1], 3) for x in v]} steps/s {[f'{x[2]:.3g}' for x in v]}")
