#!/bin/bash
# Round 4: the any-depth / one-hot kernels (g2048_deep.hip) -- unit tests, the reference-fixture rollouts and
# updates of every case (one-hot / 3- and 4-layer nets and the runner's documented config included), then the
# runner-config training iteration timed on the round-3 checkout (before) and on this tree (after).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_deep.py tests/test_capi.py -m gpu -v -s -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $O/tests_deep.log 2>&1 || { tail -40 $O/tests_deep.log; exit 1; }
tail -1 $O/tests_deep.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_ref_fixtures.py -m gpu -v -s -p no:cacheprovider -k "rollout or update" \
    --timeout 200 --timeout-method thread > $O/tests_fixtures.log 2>&1 || { tail -60 $O/tests_fixtures.log; exit 1; }
tail -1 $O/tests_fixtures.log
timeout -k 10 300 python -u tools/bench_refconfig.py --label round4 > $O/refconf_after.log 2>&1 || { tail -30 $O/refconf_after.log; exit 1; }
cat $O/refconf_after.log | grep '^{'
timeout -k 10 700 python -u tools/bench_refconfig.py --repo tools/_r3tree --label round3 > $O/refconf_before.log 2>&1 || { tail -30 $O/refconf_before.log; exit 1; }
cat $O/refconf_before.log | grep '^{'
echo DONE > $O/done.log
