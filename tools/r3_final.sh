#!/bin/bash
# Round-3 end-of-session record on the shipped build: full GPU suite, smoke, the driver's bench command, a
# 200-launch bench and the rocprofv3 kernel-trace summary of the step kernel.  Outputs under gpurun_out/r3final/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3final
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 240 --timeout-method thread \
    > $O/gpu_tests_all.log 2>&1 || { tail -40 $O/gpu_tests_all.log; exit 1; }
tail -1 $O/gpu_tests_all.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || { tail -20 $O/bench_driver_cmd.log; exit 1; }
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-policy --no-train --traffic off --steps 200 --warmup 20 > $O/bench_200.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_step -o step -- \
    python3 bench.py --no-cpu-baseline --no-policy --no-train --traffic off --steps 200 --warmup 20 > $O/prof_step.log 2>&1 || exit 1
echo DONE > $O/done.log
