#!/bin/bash
# Round 4: the tile-pipelined loop of the 8-wave g2048_dw2 (shipped) against the stage-by-stage loop
# (tools/libg2048_dw2stage.so): gradient tests, dw2 alone, the configs[2] update.  Outputs under gpurun_out/r4c15/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c15
mkdir -p $O
SHIP=rl-2048-with-reinforce-and-actor-critic_amd/libg2048.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_grad.py -m gpu -v -s -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $O/tests_grad.log 2>&1 || { tail -60 $O/tests_grad.log; exit 1; }
tail -1 $O/tests_grad.log
timeout -k 10 200 python -u tools/bench_dw2.py --lib $SHIP tools/libg2048_dw2stage.so $SHIP tools/libg2048_dw2stage.so --parts 256 > $O/dw2_ab.log 2>&1 || { tail -20 $O/dw2_ab.log; exit 1; }
grep '^{' $O/dw2_ab.log
U="tools/bench_update.py --episodes 1048576 --critic --repeats 2"
timeout -k 10 200 python3 -u $U > $O/upd_pipe.log 2>&1 || exit 1
grep '^{' $O/upd_pipe.log
timeout -k 10 200 python3 -u $U --lib tools/libg2048_dw2stage.so > $O/upd_stage.log 2>&1 || exit 1
grep '^{' $O/upd_stage.log
timeout -k 10 200 python3 -u $U > $O/upd_pipe2.log 2>&1 || exit 1
grep '^{' $O/upd_pipe2.log
echo DONE > $O/done.log
