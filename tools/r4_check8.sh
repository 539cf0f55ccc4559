#!/bin/bash
# Round 4: the 8-wave g2048_deep_grad -- deep-kernel tests, then the reference runner config (timing + kernel stats).
# Outputs under gpurun_out/r4c8/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c8
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_deep.py -m gpu -v -s -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $O/tests_deep.log 2>&1 || { tail -60 $O/tests_deep.log; exit 1; }
tail -1 $O/tests_deep.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_refconf -o rc -- python3 tools/bench_refconfig.py --label round4 > $O/refconf_after.log 2>&1 || { tail -30 $O/refconf_after.log; exit 1; }
grep '^{' $O/refconf_after.log
echo DONE > $O/done.log
