#!/bin/bash
# Round-3 step-kernel attribution: per-workgroup phases (diag build, raw per-block stamps kept) and SQ counters.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r3diag
mkdir -p $D
G2048_DIAG_LIB=tools/libg2048_dg.so timeout -k 10 120 python -u tools/diag_phases.py --warmup 120 --launches 4 > $D/phases.log 2>&1 || exit 1
mv gpurun_out/phases_raw_*.npy $D/ || true
B="--no-cpu-baseline --no-policy --no-train --traffic off --steps 20 --warmup 100"
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
         "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  timeout -s KILL 100 rocprofv3 --pmc $C --output-format csv -d $D/p$i -o p -- python3 bench.py $B > $D/p$i.log 2>&1 || { echo "PMC FAIL $i $?" >> $D/done.log; exit 1; }
done
timeout -k 10 60 rocprofv3 --list-avail > $D/list_avail.txt 2>&1 || true
echo "DONE" >> $D/done.log
