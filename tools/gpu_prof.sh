#!/bin/bash
# Round profile: default bench line (incl. PMC traffic passes) + rocprofv3 kernel-trace summary of the same
# bench command.  Outputs under gpurun_out/ (copy the summaries into profiles/).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python3 -u bench.py > gpurun_out/bench_default.log 2>&1; echo "BENCH EXIT $?" >> gpurun_out/bench_default.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1b -o r1 -- python3 bench.py --no-cpu-baseline --no-policy --traffic off > gpurun_out/prof_r1b.log 2>&1; echo "PROF EXIT $?" >> gpurun_out/prof_r1b.log
