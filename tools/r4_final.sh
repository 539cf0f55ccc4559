#!/bin/bash
# Round 4 record on the shipped build: the driver's bench command, the rocprofv3 kernel-trace summary of the step
# kernel (200 launches) and the PMC passes of the shipped configs[2] update.  Outputs under gpurun_out/r4final2/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4final2
mkdir -p $O
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || { tail -20 $O/bench_driver_cmd.log; exit 1; }
grep '^{' $O/bench_driver_cmd.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_step -o step -- \
    python3 bench.py --no-cpu-baseline --no-policy --no-train --no-refconfig --traffic off --steps 200 --warmup 20 > $O/prof_step.log 2>&1 || exit 1
EPISODES=1048576 PMC_OUT=r4final2/pmc_configs2 bash tools/pmc_grad.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_refconf -o rc -- python3 tools/bench_refconfig.py --label round4 > $O/refconf.log 2>&1 || { tail -30 $O/refconf.log; exit 1; }
grep '^{' $O/refconf.log
echo DONE > $O/done.log
