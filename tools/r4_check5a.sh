#!/bin/bash
# Round 4: unit + reference-fixture GPU tests of the deep / one-hot kernels, actor d2 records, column-split g2048_dw2
# and the cooperative gradient kernel; then the configs[2] update A/B: cooperative (default) / grad_kernel
# (G2048_GRAD_COOP=0) / the round-3 checkout.  Outputs under gpurun_out/r4c5/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c5
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_gpu_grad.py tests/test_gpu_deep.py tests/test_capi.py tests/test_gpu_ref_fixtures.py \
    -m gpu -v -s -p no:cacheprovider -k "not runner_matches" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/bench_update.py --episodes 1048576 --critic --repeats 2 > $O/update_c2_coop.log 2>&1 || { tail -20 $O/update_c2_coop.log; exit 1; }
grep '^{' $O/update_c2_coop.log
G2048_GRAD_COOP=0 timeout -k 10 200 python -u tools/bench_update.py --episodes 1048576 --critic --repeats 2 > $O/update_c2_nocoop.log 2>&1 || { tail -20 $O/update_c2_nocoop.log; exit 1; }
grep '^{' $O/update_c2_nocoop.log
timeout -k 10 200 python -u tools/bench_update.py --repo tools/_r3tree --episodes 1048576 --critic --repeats 2 > $O/update_c2_r3.log 2>&1 || { tail -20 $O/update_c2_r3.log; exit 1; }
grep '^{' $O/update_c2_r3.log
timeout -k 10 200 python -u tools/bench_update.py --episodes 1048576 --critic --repeats 2 > $O/update_c2_coop2.log 2>&1 || { tail -20 $O/update_c2_coop2.log; exit 1; }
grep '^{' $O/update_c2_coop2.log
echo DONE > $O/done.log
