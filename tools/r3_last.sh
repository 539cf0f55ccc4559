#!/bin/bash
# Round 3, last check of the shipped binary: the whole GPU suite, smoke, the driver's bench command.
set -o pipefail
O=gpurun_out/r3last
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/gpu_tests_all.log 2>&1 || { tail -40 $O/gpu_tests_all.log; exit 1; }
tail -1 $O/gpu_tests_all.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || { tail -20 $O/bench_driver_cmd.log; exit 1; }
