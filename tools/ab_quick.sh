#!/bin/bash
# Interleaved A/B of step-kernel builds on one box: bash tools/ab_quick.sh <out_dir> <lib> <lib> ...
# Bench workload (headline mode), 200-step and 20-step runs per library, 3 rounds.
set -o pipefail
O=$1; shift
mkdir -p $O
B="--no-cpu-baseline --no-policy --no-train --traffic off"
for rep in 1 2 3; do
  for lib in "$@"; do
    for st in 200 20; do
      echo "== $lib steps=$st" >> $O/ab.log
      timeout -k 10 120 python -u bench.py $B --steps $st --warmup $((st / 10 + 5)) --lib $lib >> $O/ab.log 2>&1 || exit 1
    done
  done
done
python3 - "$O/ab.log" <<'PY'
import json, sys, collections
res = collections.defaultdict(list)
cur = None
for line in open(sys.argv[1]):
    if line.startswith("=="):
        cur = line.strip()[3:]
    elif line.startswith("{"):
        d = json.loads(line)
        res[cur].append((round(d["ms_per_step"] * 1e3, 2), round(d["roofline"]["kernel_ms"] * 1e3, 2)))
for k, v in res.items():
    print(k, "wall_us/step, event_us/launch:", v)
PY
