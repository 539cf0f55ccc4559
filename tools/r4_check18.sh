#!/bin/bash
# step kernel: resetting lanes store their step outputs in the sweep (whole lines) -- A/B against the hole-leaving
# build, then the env / lean / fixture suites on the new build
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4c18
mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python3 -u tools/step_launch_probe.py --reps 3 --modes fresh,fresh40,eager > $O/new_$r.log 2>&1
  G2048_LIB=tools/libg2048_rs0.so timeout -k 10 200 python3 -u tools/step_launch_probe.py --reps 3 --modes fresh,fresh40,eager > $O/old_$r.log 2>&1
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_env.py tests/test_gpu_lean_rare.py tests/test_gpu_ref_fixtures.py tests/test_gpu_env_large.py > $O/tests.log 2>&1
timeout -k 10 200 python3 bench.py > $O/bench.log 2>&1
echo done
