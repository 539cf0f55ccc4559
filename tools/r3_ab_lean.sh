#!/bin/bash
# Round 3: env parity on the shipped (lean) build, then interleaved step-kernel A/B against the round-start build
# (tools/libg2048_base.so) and the same sources without the lean path (tools/libg2048_nolean.so); SQ counters.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_lean
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_env.py tests/test_gpu_ref_fixtures.py tests/test_gpu_env_large.py -m gpu -x -q \
    -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SHIP=rl-2048-with-reinforce-and-actor-critic_amd/libg2048.so
O=$O bash tools/ab_libs.sh tools/libg2048_base.so tools/libg2048_nolean.so $SHIP || exit 1
B="--no-cpu-baseline --no-policy --no-train --traffic off --steps 20 --warmup 100"
timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $O/pmc -o p -- python3 bench.py $B > $O/pmc.log 2>&1 || echo "PMC FAIL" >> $O/ab.log
echo DONE >> $O/ab.log
