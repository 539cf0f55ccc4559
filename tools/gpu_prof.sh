#!/bin/bash
# rocprofv3 kernel-trace summary + PMC traffic (via bench.py --traffic auto) + the fused onehot/Philox variant.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
B="--no-cpu-baseline --no-policy --traffic off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1 -o r1 -- python3 bench.py --steps 50 --warmup 10 $B > gpurun_out/prof.log 2>&1; echo "PROF EXIT $?" >> gpurun_out/prof.log
timeout -k 10 600 python3 -u bench.py --steps 200 --warmup 20 > gpurun_out/bench_full.log 2>&1; echo "BENCH EXIT $?" >> gpurun_out/bench_full.log
timeout -k 10 200 python3 -u bench.py --steps 100 --warmup 10 --rng philox --obs onehot $B > gpurun_out/bench_onehot.log 2>&1; echo "BENCH2 EXIT $?" >> gpurun_out/bench_onehot.log
timeout -k 10 200 python3 -u bench.py --steps 100 --warmup 10 --rng philox --obs none $B > gpurun_out/bench_core.log 2>&1; echo "BENCH3 EXIT $?" >> gpurun_out/bench_core.log
ls -R gpurun_out/prof_r1 | head -20 >> gpurun_out/prof.log
