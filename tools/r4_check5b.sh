#!/bin/bash
# Round 4: g2048_dw2 A/B against the round-4 start build, and the reference runner config before (round-3
# checkout) / after.  Outputs under gpurun_out/r4c5b/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c5b
mkdir -p $O
timeout -k 10 200 python -u tools/bench_dw2.py --lib tools/libg2048_r4a.so "" --parts 256 128 > $O/dw2_ab.log 2>&1 || { tail -20 $O/dw2_ab.log; exit 1; }
grep '^{' $O/dw2_ab.log
timeout -k 10 300 python -u tools/bench_refconfig.py --label round4 > $O/refconf_after.log 2>&1 || { tail -30 $O/refconf_after.log; exit 1; }
grep '^{' $O/refconf_after.log
timeout -k 10 600 python -u tools/bench_refconfig.py --repo tools/_r3tree --label round3 > $O/refconf_before.log 2>&1 || { tail -30 $O/refconf_before.log; exit 1; }
grep '^{' $O/refconf_before.log
echo DONE > $O/done.log
