#!/bin/bash
# one-hot gather: 16 vs 32 W1-row loads in flight (G2048_DEEP_GATHER_UNROLL 4 vs 8), runner config, interleaved
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4c21
mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python3 tools/bench_refconfig.py --label u4 > $O/u4_$r.log 2>&1
  G2048_LIB=tools/libg2048_gu8.so timeout -k 10 200 python3 tools/bench_refconfig.py --label u8 > $O/u8_$r.log 2>&1
done
grep -h '^{' $O/*.log | cut -c1-200
