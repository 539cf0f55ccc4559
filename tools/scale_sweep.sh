#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
B="--no-cpu-baseline --no-policy --traffic off --steps 100 --warmup 10"
for mode in "--rng pcg64 --obs log2" "--rng philox --obs none"; do
 for n in 262144 524288 1048576 2097152 4194304 8388608; do
  echo "== $mode n=$n" >> gpurun_out/scale.log
  timeout -k 10 120 python -u bench.py $B $mode --boards $n >> gpurun_out/scale.log 2>&1 || { echo "FAIL $?" >> gpurun_out/scale.log; exit 1; }
 done
done
export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"
timeout -k 10 200 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_sq2/a -o a -- python3 bench.py --no-cpu-baseline --no-policy --traffic off --steps 20 --warmup 5 --rng philox --obs none > gpurun_out/pmc_sq2_a.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sq2/b -o b -- python3 bench.py --no-cpu-baseline --no-policy --traffic off --steps 20 --warmup 5 --rng philox --obs none > gpurun_out/pmc_sq2_b.log 2>&1
echo "SCALE DONE $?" >> gpurun_out/scale.log
