#!/bin/bash
# Round 4: deep / one-hot kernels, actor d2 records and the column-split g2048_dw2 -- unit + reference-fixture
# tests, then A/B timings: g2048_dw2 alone (previous build vs this), the configs[2] update (round-3 checkout vs this
# tree) and the reference runner config (round-3 checkout = before, this tree = after).  Outputs under gpurun_out/r4c3/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_deep.py tests/test_gpu_grad.py tests/test_capi.py tests/test_gpu_ref_fixtures.py \
    -m gpu -v -s -p no:cacheprovider -k "not runner_matches" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/bench_dw2.py --lib tools/libg2048_r4a.so "" --parts 256 128 > $O/dw2_ab.log 2>&1 || { tail -20 $O/dw2_ab.log; exit 1; }
grep '^{' $O/dw2_ab.log
timeout -k 10 300 python -u tools/bench_update.py --episodes 1048576 --critic --repeats 1 > $O/update_c2_after.log 2>&1 || { tail -20 $O/update_c2_after.log; exit 1; }
grep '^{' $O/update_c2_after.log
timeout -k 10 300 python -u tools/bench_update.py --repo tools/_r3tree --episodes 1048576 --critic --repeats 1 > $O/update_c2_r3.log 2>&1 || { tail -20 $O/update_c2_r3.log; exit 1; }
grep '^{' $O/update_c2_r3.log
timeout -k 10 300 python -u tools/bench_refconfig.py --label round4 > $O/refconf_after.log 2>&1 || { tail -30 $O/refconf_after.log; exit 1; }
grep '^{' $O/refconf_after.log
timeout -k 10 700 python -u tools/bench_refconfig.py --repo tools/_r3tree --label round3 > $O/refconf_before.log 2>&1 || { tail -30 $O/refconf_before.log; exit 1; }
grep '^{' $O/refconf_before.log
echo DONE > $O/done.log
