#!/bin/bash
# Round 4: where the configs[2] update time goes -- rocprofv3 kernel stats of the update with the cooperative gradient
# kernel and actor records (default) and without records; update_s of each (coop x records) combination; the
# one-hot dW1 scatter test and the reference runner config (timing + kernel stats).  Outputs under gpurun_out/r4c6/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c6
mkdir -p $O
U="tools/bench_update.py --episodes 1048576 --critic --repeats 1"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_rec -o upd -- python3 $U > $O/prof_rec.log 2>&1 || { tail -20 $O/prof_rec.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_norec -o upd -- python3 $U --no-actor-records > $O/prof_norec.log 2>&1 || { tail -20 $O/prof_norec.log; exit 1; }
timeout -k 10 200 python3 -u $U --repeats 2 --no-actor-records > $O/upd_coop_norec.log 2>&1 || exit 1
grep '^{' $O/upd_coop_norec.log
G2048_GRAD_COOP=0 timeout -k 10 200 python3 -u $U --repeats 2 --no-actor-records > $O/upd_nocoop_norec.log 2>&1 || exit 1
grep '^{' $O/upd_nocoop_norec.log
timeout -k 10 200 python3 -u $U --repeats 2 > $O/upd_coop_rec.log 2>&1 || exit 1
grep '^{' $O/upd_coop_rec.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_deep.py -m gpu -v -s -p no:cacheprovider -k "onehot" --timeout 120 \
    --timeout-method thread > $O/tests_onehot.log 2>&1 || { tail -40 $O/tests_onehot.log; exit 1; }
tail -1 $O/tests_onehot.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_refconf -o rc -- python3 tools/bench_refconfig.py --label round4 > $O/refconf_after.log 2>&1 || { tail -30 $O/refconf_after.log; exit 1; }
grep '^{' $O/refconf_after.log
echo DONE > $O/done.log
