#!/bin/bash
# Round 4: the 8-wave g2048_dw2 for 256-wide layers (shipped) against the column-split 4-wave form
# (tools/libg2048_dw2split.so): gradient tests, dw2 alone, the configs[2] update; then the headline with / without
# the runner-config leg and the XCD-partition step A/B.  Outputs under gpurun_out/r4c10/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c10
mkdir -p $O
SHIP=rl-2048-with-reinforce-and-actor-critic_amd/libg2048.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_grad.py -m gpu -v -s -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $O/tests_grad.log 2>&1 || { tail -60 $O/tests_grad.log; exit 1; }
tail -1 $O/tests_grad.log
timeout -k 10 200 python -u tools/bench_dw2.py --lib $SHIP tools/libg2048_dw2split.so $SHIP tools/libg2048_dw2split.so --parts 256 > $O/dw2_ab.log 2>&1 || { tail -20 $O/dw2_ab.log; exit 1; }
grep '^{' $O/dw2_ab.log
U="tools/bench_update.py --episodes 1048576 --critic --repeats 2"
timeout -k 10 200 python3 -u $U > $O/upd_wide.log 2>&1 || exit 1
grep '^{' $O/upd_wide.log
timeout -k 10 200 python3 -u $U --lib tools/libg2048_dw2split.so > $O/upd_split.log 2>&1 || exit 1
grep '^{' $O/upd_split.log
timeout -k 10 200 python3 -u $U > $O/upd_wide2.log 2>&1 || exit 1
grep '^{' $O/upd_wide2.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --traffic off > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
grep '^{' $O/bench_default.log | cut -c1-200
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --traffic off --no-refconfig > $O/bench_norefconf.log 2>&1 || { tail -20 $O/bench_norefconf.log; exit 1; }
grep '^{' $O/bench_norefconf.log | cut -c1-200
B="--no-cpu-baseline --no-policy --no-train --no-refconfig --traffic off --steps 200 --warmup 20"
for rep in 1 2 3; do
  for lib in $SHIP tools/libg2048_xcd1.so tools/libg2048_xcd2.so; do
    echo "== $lib" >> $O/ab_xcd.log
    timeout -k 10 120 python -u bench.py $B --lib $lib >> $O/ab_xcd.log 2>&1 || exit 1
  done
done
python3 - <<'PY'
import json
cur = None
for line in open("gpurun_out/r4c10/ab_xcd.log"):
    if line.startswith("== "):
        cur = line[3:].strip()
    elif line.startswith("{"):
        d = json.loads(line)
        print(cur, "kernel_us", round(d["roofline"]["kernel_ms"] * 1e3, 2), "ms_per_step_us", round(d["ms_per_step"] * 1e3, 2))
PY
echo DONE > $O/done.log
