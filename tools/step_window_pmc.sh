#!/bin/bash
# PMC of the step kernel's start window: the launches after S = 5 vs S = 40 untimed steps from
# bench.py's synthetic random-state start (tools/step_state_pmc.py), one counter group per pass, each pass under its
# own time limit.  A pass whose counter names this rocprofv3 does not know fails fast and is skipped; a time limit
# ends the script.  Outputs under gpurun_out/$RUN/swp; summary: tools/step_window_summary.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${RUN:-swp}/swp
mkdir -p "$O"
P="--kernel-trace --output-format csv"
PASSES=(
  "sq1:SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
  "sq2:SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVES SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
  "ea:TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum"
  "hit:TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
  "tcp:TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum"
  "wr:WRITE_SIZE"
)
for S in 5 40; do
  for p in "${PASSES[@]}"; do
    name=${p%%:*}
    ctrs=${p#*:}
    # shellcheck disable=SC2086
    timeout -s KILL 90 rocprofv3 --pmc $ctrs $P -d "$O/$name$S" -o run -- python3 tools/step_state_pmc.py --skip $S > "$O/$name$S.log" 2>&1
    rc=$?
    if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then echo "pass $name S=$S timed out"; exit 1; fi
    [ $rc -eq 0 ] || echo "pass $name S=$S failed (rc $rc): $(grep -m1 -i error "$O/$name$S.log" | cut -c1-160)"
  done
done
python3 tools/step_window_summary.py "$O"
