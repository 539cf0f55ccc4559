#!/bin/bash
# PMC of step launches after the synthetic start (S = 5) vs later (S = 40): tools/step_state_pmc.py
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4sp
rm -rf $O; mkdir -p $O
P="--kernel-trace --output-format csv"
for S in 5 40; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY $P -d $O/sq$S -o run -- python3 tools/step_state_pmc.py --skip $S > $O/sq$S.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE $P -d $O/f$S -o run -- python3 tools/step_state_pmc.py --skip $S > $O/f$S.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE $P -d $O/w$S -o run -- python3 tools/step_state_pmc.py --skip $S > $O/w$S.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum $P -d $O/wr$S -o run -- python3 tools/step_state_pmc.py --skip $S > $O/wr$S.log 2>&1
done
echo done
