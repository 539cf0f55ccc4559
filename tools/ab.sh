#!/bin/bash
# diagnostic A/B runs: one JSON line per configuration in gpurun_out/ab.log
set -o pipefail
mkdir -p gpurun_out
B="--no-cpu-baseline --no-policy --traffic off --steps 100 --warmup 10"
for extra in "" "--no-auto-reset"; do
 for mode in "--rng pcg64 --obs log2" "--rng philox --obs none"; do
  echo "== $extra $mode" >> gpurun_out/ab.log
  timeout -k 10 120 python -u bench.py $B $mode $extra >> gpurun_out/ab.log 2>&1 || { echo "FAIL $?" >> gpurun_out/ab.log; exit 1; }
  python3 - >> gpurun_out/ab.log <<'PY'
PY
 done
done
echo AB DONE >> gpurun_out/ab.log
