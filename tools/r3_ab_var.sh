#!/bin/bash
# Round 3 step-kernel variant A/B: env parity on the variant (through G2048_TOOLS_LIB), then interleaved bench runs
# of the variant against the shipped build.   bash tools/r3_ab_var.sh OUT variant.so
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
G2048_TOOLS_LIB=$2 timeout -k 10 500 python -u -m pytest "tests/test_gpu_env.py::test_env_step_vs_oracle" tests/test_gpu_env_large.py tests/test_gpu_ref_fixtures.py \
    -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
O=$O bash tools/ab_libs.sh rl-2048-with-reinforce-and-actor-critic_amd/libg2048.so $2 || exit 1
echo DONE >> $O/ab.log
