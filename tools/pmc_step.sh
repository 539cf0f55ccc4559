#!/bin/bash
# SQ counter pass on the step kernel (kernel-trace only, no other tracing domains), two modes.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_sq
B="--no-cpu-baseline --no-policy --traffic off --steps 20 --warmup 5"
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"
timeout -k 10 200 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_sq/a -o a -- python3 bench.py $B --rng philox --obs none > gpurun_out/pmc_sq/a.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sq/b -o b -- python3 bench.py $B --rng philox --obs none > gpurun_out/pmc_sq/b.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_sq/c -o c -- python3 bench.py $B --rng pcg64 --obs log2 > gpurun_out/pmc_sq/c.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_sq/f -o f -- python3 bench.py $B --rng pcg64 --obs log2 > gpurun_out/pmc_sq/f.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_sq/w -o w -- python3 bench.py $B --rng pcg64 --obs log2 > gpurun_out/pmc_sq/w.log 2>&1
echo "PMC EXIT $?" > gpurun_out/pmc_sq/done.log
