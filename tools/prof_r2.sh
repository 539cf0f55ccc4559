#!/bin/bash
# Round-2 profiles: rocprofv3 kernel-trace summaries of (1) the headline bench command's step kernel and (2) the
# configs[2] actor-critic training iteration (1,048,576 episodes) split by kernel.  Outputs under gpurun_out/prof_r2/.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/prof_r2
mkdir -p "$O"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/step" -o step -- \
    python3 "$R/bench.py" --no-cpu-baseline --no-policy --no-train --traffic off > "$O/step.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/train2" -o train2 -- \
    python3 "$R/tools/bench_update.py" --episodes 1048576 --repeats 1 --critic > "$O/train2.log" 2>&1
