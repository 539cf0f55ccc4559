#!/bin/bash
# Round 4: configs[2] update A/B -- cooperative gradient kernel (default) / grad_kernel (G2048_GRAD_COOP=0) / the
# round-3 checkout -- then the deep-kernel tests and the at-size fp64 tests on this build.  Outputs under
# gpurun_out/r4c5/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c5
mkdir -p $O
timeout -k 10 200 python -u tools/bench_update.py --episodes 1048576 --critic --repeats 2 > $O/update_c2_coop.log 2>&1 || { tail -20 $O/update_c2_coop.log; exit 1; }
grep '^{' $O/update_c2_coop.log
G2048_GRAD_COOP=0 timeout -k 10 200 python -u tools/bench_update.py --episodes 1048576 --critic --repeats 2 > $O/update_c2_nocoop.log 2>&1 || { tail -20 $O/update_c2_nocoop.log; exit 1; }
grep '^{' $O/update_c2_nocoop.log
timeout -k 10 200 python -u tools/bench_update.py --repo tools/_r3tree --episodes 1048576 --critic --repeats 2 > $O/update_c2_r3.log 2>&1 || { tail -20 $O/update_c2_r3.log; exit 1; }
grep '^{' $O/update_c2_r3.log
timeout -k 10 200 python -u tools/bench_update.py --episodes 1048576 --critic --repeats 2 > $O/update_c2_coop2.log 2>&1 || { tail -20 $O/update_c2_coop2.log; exit 1; }
grep '^{' $O/update_c2_coop2.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_deep.py -m gpu -v -s -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $O/tests_deep.log 2>&1 || { tail -60 $O/tests_deep.log; exit 1; }
tail -1 $O/tests_deep.log
timeout -k 10 420 python -u -m pytest tests/test_gpu_configs_at_size.py -m gpu -v -s -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $O/at_size.log 2>&1 || { tail -60 $O/at_size.log; exit 1; }
tail -1 $O/at_size.log
echo DONE > $O/done.log
