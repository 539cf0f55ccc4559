#!/bin/bash
# End-of-round profiles of the shipped library: rocprofv3 kernel-trace summaries of (1) the headline bench
# command (step kernel) and (2) the bench with the policy rollout and both training iterations; (3) host-side
# phase timing of rollout_batch.  Outputs under gpurun_out/final/ (copy the summaries into profiles/).
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/final
mkdir -p "$O"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_step" -o step -- \
    python3 "$R/bench.py" --no-cpu-baseline --no-policy --traffic off > "$O/prof_step.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_train" -o train -- \
    python3 "$R/bench.py" --no-cpu-baseline --traffic off > "$O/prof_train.log" 2>&1 &&
timeout -k 10 200 python3 -u "$R/tools/roll_host_timing.py" > "$O/roll_host_timing.log" 2>&1
