#!/bin/bash
# GPU env parity tests, then the step kernel in three modes (one JSON line each in gpurun_out/sweep.log).
set -o pipefail
mkdir -p gpurun_out
B="--no-cpu-baseline --no-policy --traffic off --steps 100 --warmup 10"
timeout -k 10 300 python -u -m pytest tests/test_gpu_env.py -m gpu -q -p no:cacheprovider --timeout 200 -x > gpurun_out/sweep_tests.log 2>&1; echo "TESTS EXIT $?" >> gpurun_out/sweep_tests.log
for mode in "--rng pcg64 --obs log2" "--rng philox --obs onehot" "--rng philox --obs none" "--rng pcg64 --obs none"; do
  echo "== $mode" >> gpurun_out/sweep.log
  timeout -k 10 120 python -u bench.py $B $mode >> gpurun_out/sweep.log 2>&1 || { echo "FAIL $?" >> gpurun_out/sweep.log; exit 1; }
done
echo SWEEP DONE >> gpurun_out/sweep.log
