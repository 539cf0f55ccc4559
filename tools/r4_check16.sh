#!/bin/bash
# Round 4: tile-pipelined wide g2048_dw2 vs stage-by-stage (tools/libg2048_dw2stage.so), the critic-row glue trim,
# the spread deep output layer: gradient + deep tests, dw2 alone, configs[2] update, runner config.
# Outputs under gpurun_out/r4c16/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c16
mkdir -p $O
SHIP=rl-2048-with-reinforce-and-actor-critic_amd/libg2048.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_grad.py tests/test_gpu_deep.py -m gpu -v -s -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/bench_dw2.py --lib $SHIP tools/libg2048_dw2stage.so $SHIP tools/libg2048_dw2stage.so --parts 256 > $O/dw2_ab.log 2>&1 || { tail -20 $O/dw2_ab.log; exit 1; }
grep '^{' $O/dw2_ab.log
U="tools/bench_update.py --episodes 1048576 --critic --repeats 2"
timeout -k 10 200 python3 -u $U > $O/upd_pipe.log 2>&1 || exit 1
grep '^{' $O/upd_pipe.log
timeout -k 10 200 python3 -u $U --lib tools/libg2048_dw2stage.so > $O/upd_stage.log 2>&1 || exit 1
grep '^{' $O/upd_stage.log
timeout -k 10 200 python3 -u $U > $O/upd_pipe2.log 2>&1 || exit 1
grep '^{' $O/upd_pipe2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_refconf -o rc -- python3 tools/bench_refconfig.py --label round4 > $O/refconf.log 2>&1 || { tail -30 $O/refconf.log; exit 1; }
grep '^{' $O/refconf.log | cut -c1-330
echo DONE > $O/done.log
