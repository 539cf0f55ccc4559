#!/bin/bash
# PMC passes over one actor-critic iteration (tools/bench_update.py, EPISODES=65536 default; PMC_OUT names the dir): MFMA busy
# cycles and HBM traffic of grad_kernel, one counter group per run (MI355X_MICROARCH.md: TCC limits), each pass
# under its own time limit.  Outputs under gpurun_out/pmc_grad/; tools/pmc_grad_summary.py reads them.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/${PMC_OUT:-pmc_grad}
mkdir -p "$O"
CMD="python3 $R/tools/bench_update.py --episodes ${EPISODES:-65536} --repeats 1 --critic"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- $CMD > "$O/trace.log" 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE \
    --output-format csv -d "$O/sq" -o run -- $CMD > "$O/sq.log" 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o run -- $CMD > "$O/fetch.log" 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o run -- $CMD > "$O/write.log" 2>&1
