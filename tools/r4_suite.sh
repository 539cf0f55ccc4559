#!/bin/bash
# Round 4: the whole GPU suite and smoke() on the shipped build.  Outputs under gpurun_out/r4suite/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4suite2
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/gpu_tests_all.log 2>&1 || { tail -40 $O/gpu_tests_all.log; exit 1; }
tail -1 $O/gpu_tests_all.log
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
