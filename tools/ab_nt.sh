#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
B="--no-cpu-baseline --no-policy --traffic off --steps 100 --warmup 10"
for rep in 1 2; do
for lib in tools/libg2048_diag.so tools/libg2048_diag_nt.so; do   # build the _nt variant with -DG2048_OBS_NT=1, the other with 0
  for mode in "--rng pcg64 --obs log2" "--rng philox --obs onehot" "--rng philox --obs onehot --boards 4194304"; do
    echo "== $lib $mode" >> gpurun_out/ab_nt.log
    timeout -k 10 120 python -u bench.py $B $mode --lib $lib >> gpurun_out/ab_nt.log 2>&1 || exit 1
  done
done
done
