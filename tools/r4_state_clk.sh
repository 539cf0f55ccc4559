#!/bin/bash
# chip clock over the step launches after the synthetic start (S = 5) vs later (S = 40)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4sc
rm -rf $O; mkdir -p $O
for S in 5 40; do
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/g$S -o run -- python3 tools/step_state_pmc.py --skip $S > $O/g$S.log 2>&1
done
echo done
