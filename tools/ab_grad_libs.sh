#!/bin/bash
# A/B of gradient-kernel builds on one box: the gradient parity tests on the shipped library, then the configs[1]
# and configs[2]-size actor-critic update timed per library, interleaved: bash tools/ab_grad_libs.sh <lib> <lib> ...
set -o pipefail
O=${O:-gpurun_out/ab_grad_libs}
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest ${GT:-tests/test_gpu_grad.py} -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for lib in "$@"; do
    echo "== $lib" >> $O/ab.log
    timeout -k 10 300 python3 -u tools/bench_update.py --episodes ${EPS:-65536 1048576} --repeats 2 --critic --lib $lib >> $O/ab.log 2>&1 || exit 1
  done
done
