#!/bin/bash
# A/B of step-kernel builds on one box, interleaved: bash tools/ab_libs.sh <lib> <lib> ...
# MODES (env): bench mode arguments separated by ';' (default: the headline mode).  TEST_LIB (env): a build to run
# the env parity tests on first (through tests/conftest.py's G2048_TOOLS_LIB).
set -o pipefail
O=${O:-gpurun_out/ab_libs}
mkdir -p $O
if [ -n "$TEST_LIB" ]; then
  G2048_TOOLS_LIB=$TEST_LIB timeout -k 10 400 python -u -m pytest tests/test_gpu_env.py tests/test_gpu_ref_fixtures.py -m gpu -x -q \
      -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
B="--no-cpu-baseline --no-policy --no-train --traffic off --steps 200 --warmup 20"
IFS=';' read -ra MS <<< "${MODES:---rng pcg64 --obs log2}"
for rep in 1 2 3; do
  for m in "${MS[@]}"; do
    for lib in "$@"; do
      echo "== $lib $m" >> $O/ab.log
      timeout -k 10 120 python -u bench.py $B $m --lib $lib >> $O/ab.log 2>&1 || exit 1
    done
  done
done
