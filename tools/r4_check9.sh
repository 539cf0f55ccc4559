#!/bin/bash
# Round 4: (1) does the runner-config leg slow the headline? the driver's bench command with and without it;
# (2) VERDICT r3 item 4b: the XCD-aware static partition of the step kernel (-DG2048_STEP_XCD=1 / 2 builds)
# against the shipped strided partition, interleaved, 200 launches each, HIP-event kernel time.
# Outputs under gpurun_out/r4c9/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c9
mkdir -p $O
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --traffic off > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
grep '^{' $O/bench_default.log | cut -c1-200
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --traffic off --no-refconfig > $O/bench_norefconf.log 2>&1 || { tail -20 $O/bench_norefconf.log; exit 1; }
grep '^{' $O/bench_norefconf.log | cut -c1-200
B="--no-cpu-baseline --no-policy --no-train --no-refconfig --traffic off --steps 200 --warmup 20"
SHIP=rl-2048-with-reinforce-and-actor-critic_amd/libg2048.so
for rep in 1 2 3; do
  for lib in $SHIP tools/libg2048_xcd1.so tools/libg2048_xcd2.so; do
    echo "== $lib" >> $O/ab_xcd.log
    timeout -k 10 120 python -u bench.py $B --lib $lib >> $O/ab_xcd.log 2>&1 || exit 1
  done
done
python3 - <<'PY'
import json
cur = None
for line in open("gpurun_out/r4c9/ab_xcd.log"):
    if line.startswith("== "):
        cur = line[3:].strip()
    elif line.startswith("{"):
        d = json.loads(line)
        print(cur, "kernel_us", round(d["roofline"]["kernel_ms"] * 1e3, 2), "ms_per_step", round(d["ms_per_step"] * 1e3, 2))
PY
echo DONE > $O/done.log
