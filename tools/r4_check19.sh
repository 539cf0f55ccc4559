#!/bin/bash
# obs stores plain vs non-temporal on the driver's start window (steps 5-25) and later (40-60)
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4c19
mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python3 -u tools/step_launch_probe.py --reps 3 --modes fresh,fresh40 > $O/nt1_$r.log 2>&1
  G2048_LIB=tools/libg2048_nt0.so timeout -k 10 200 python3 -u tools/step_launch_probe.py --reps 3 --modes fresh,fresh40 > $O/nt0_$r.log 2>&1
done
echo done
