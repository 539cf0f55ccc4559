#!/bin/bash
# Round 3 step-kernel A/B: env parity on the shipped build, then interleaved bench runs of the given libraries
# against the shipped one, then SQ VALU counters of the shipped build.   bash tools/r3_ab.sh OUT lib...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_env.py tests/test_gpu_ref_fixtures.py tests/test_gpu_env_large.py -m gpu -x -q \
    -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
O=$O bash tools/ab_libs.sh "$@" rl-2048-with-reinforce-and-actor-critic_amd/libg2048.so || exit 1
B="--no-cpu-baseline --no-policy --no-train --traffic off --steps 20 --warmup 100"
timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $O/pmc -o p -- python3 bench.py $B > $O/pmc.log 2>&1 || echo "PMC FAIL" >> $O/ab.log
echo DONE >> $O/ab.log
