#!/bin/bash
# Step-kernel timing attribution on the GPU box: bench.py (pcg64 + log2 obs, 1M boards) under the diag build
# with each G2048_DIAG_FLAGS value; one JSON line per value in gpurun_out/diag.log.
set -o pipefail
mkdir -p gpurun_out
B="--no-cpu-baseline --no-policy --no-train --traffic off --steps 100 --warmup 10 ${DIAG_MODE:---rng pcg64 --obs log2}"
for f in ${DIAG_FLAGS:-0 1 2 4 16 3 23 8 9}; do
  echo "== flags=$f" >> gpurun_out/diag.log
  G2048_DIAG_FLAGS=$f timeout -k 10 120 python -u bench.py $B --lib ${DIAG_LIB:-tools/libg2048_dg.so} >> gpurun_out/diag.log 2>&1 || { echo "FAIL $?" >> gpurun_out/diag.log; exit 1; }
done
echo DIAG DONE >> gpurun_out/diag.log
