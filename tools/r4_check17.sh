#!/bin/bash
# Round 4: the k-split dense layers of g2048_deep_grad (and its probe): deep + reference-fixture tests, runner config.
# Outputs under gpurun_out/r4c17/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c17
mkdir -p $O
SHIP=rl-2048-with-reinforce-and-actor-critic_amd/libg2048.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_deep.py tests/test_gpu_ref_fixtures.py -m gpu -v -s -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_refconf -o rc -- python3 tools/bench_refconfig.py --label round4 > $O/refconf.log 2>&1 || { tail -30 $O/refconf.log; exit 1; }
grep '^{' $O/refconf.log | cut -c1-330
echo DONE > $O/done.log
