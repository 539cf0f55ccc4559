#!/bin/bash
# Round 4: g2048_dw2 with the 256-wide output split over two workgroups (shipped) vs one workgroup
# (-DG2048_DW2_SPLIT=0 build), alone and in the configs[2] update; then the reference runner config after / before
# (round-3 checkout).  Outputs under gpurun_out/r4c7/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c7
mkdir -p $O
timeout -k 10 200 python -u tools/bench_dw2.py --lib rl-2048-with-reinforce-and-actor-critic_amd/libg2048.so tools/libg2048_dw2nosplit.so rl-2048-with-reinforce-and-actor-critic_amd/libg2048.so tools/libg2048_dw2nosplit.so --parts 256 128 > $O/dw2_split_ab.log 2>&1 || { tail -20 $O/dw2_split_ab.log; exit 1; }
grep '^{' $O/dw2_split_ab.log
U="tools/bench_update.py --episodes 1048576 --critic --repeats 2"
timeout -k 10 200 python3 -u $U --lib tools/libg2048_dw2nosplit.so > $O/upd_nosplit.log 2>&1 || exit 1
grep '^{' $O/upd_nosplit.log
timeout -k 10 200 python3 -u $U > $O/upd_split.log 2>&1 || exit 1
grep '^{' $O/upd_split.log
timeout -k 10 300 python -u tools/bench_refconfig.py --label round4 > $O/refconf_after.log 2>&1 || { tail -30 $O/refconf_after.log; exit 1; }
grep '^{' $O/refconf_after.log
timeout -k 10 600 python -u tools/bench_refconfig.py --repo tools/_r3tree --label round3 > $O/refconf_before.log 2>&1 || { tail -30 $O/refconf_before.log; exit 1; }
grep '^{' $O/refconf_before.log
echo DONE > $O/done.log
