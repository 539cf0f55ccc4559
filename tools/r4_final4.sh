#!/bin/bash
# Round 4 final record (after the reset-store and deep-kernel changes) on the shipped build: full GPU suite, smoke, the driver's bench command, rocprofv3
# kernel stats of the step kernel (200 launches), the runner config's kernel stats.
# Outputs under gpurun_out/r4final4/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4final4
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/gpu_tests_all.log 2>&1 || { tail -40 $O/gpu_tests_all.log; exit 1; }
tail -1 $O/gpu_tests_all.log
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || { tail -20 $O/bench_driver_cmd.log; exit 1; }
grep '^{' $O/bench_driver_cmd.log | cut -c1-300
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_step -o step -- \
    python3 bench.py --no-cpu-baseline --no-policy --no-train --no-refconfig --traffic off --steps 200 --warmup 20 > $O/prof_step.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_refconf -o rc -- python3 tools/bench_refconfig.py --label round4 > $O/refconf.log 2>&1 || { tail -30 $O/refconf.log; exit 1; }
grep '^{' $O/refconf.log | cut -c1-330
echo DONE > $O/done.log
