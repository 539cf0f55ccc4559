#!/bin/bash
# SQ counter passes on the step kernel (kernel-trace only; no other tracing domains), bench config.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/pmc_sq2
mkdir -p $D
B="--no-cpu-baseline --no-policy --traffic off --steps 20 --warmup 5 ${PMC_MODE:---rng pcg64 --obs log2}"
timeout -k 10 120 rocprofv3 --list-avail > $D/list_avail.txt 2>&1 || true
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
         "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_INST_CYCLES_SALU" ; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $C --output-format csv -d $D/p$i -o p -- python3 bench.py $B > $D/p$i.log 2>&1 || { echo "PMC FAIL $i $?" >> $D/done.log; exit 1; }
done
echo "PMC EXIT 0" >> $D/done.log
