#!/bin/bash
# A/B of the step kernel on one box: the previous build (tools/libg2048_prev.so) against the shipped library,
# interleaved, bench workload, kernel time from bench's HIP events.  Then the env parity tests on the new build.
set -o pipefail
O=${O:-gpurun_out/ab_step}
mkdir -p $O
B="--no-cpu-baseline --no-policy --no-train --traffic off --steps 200 --warmup 20"
SHIP=rl-2048-with-reinforce-and-actor-critic_amd/libg2048.so
for rep in 1 2 3; do
  for lib in tools/libg2048_prev.so $SHIP; do
    echo "== $lib" >> $O/ab.log
    timeout -k 10 120 python -u bench.py $B --lib $lib >> $O/ab.log 2>&1 || exit 1
  done
done
timeout -k 10 600 python -u -m pytest ${ABT:-tests/test_gpu_env.py tests/test_gpu_ref_fixtures.py} -m gpu -x -q -p no:cacheprovider \
    --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
exit $rc
