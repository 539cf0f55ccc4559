#!/bin/bash
# A/B of internal step-kernel knobs: one JSON line per (knob, mode) in gpurun_out/ab.log
set -o pipefail
mkdir -p gpurun_out
B="--no-cpu-baseline --no-policy --traffic off --steps 100 --warmup 10"
for knob in "G2048_STEP_U=1" "G2048_STEP_U=2"; do
 for mode in "--rng pcg64 --obs log2" "--rng philox --obs none" "--rng pcg64 --obs none"; do
  echo "== $knob $mode" >> gpurun_out/ab.log
  env $knob timeout -k 10 120 python -u bench.py $B $mode >> gpurun_out/ab.log 2>&1 || { echo "FAIL $?" >> gpurun_out/ab.log; exit 1; }
 done
done
echo AB DONE >> gpurun_out/ab.log
