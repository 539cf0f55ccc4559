#!/bin/bash
# End-of-round evidence on one box: rocprofv3 kernel-trace summaries of the headline bench command and of the
# configs[2] training iteration, then a 2-rank rehearsal of the bench's torchrun launch (both ranks on the one
# GPU: checks the N>1 code path -- RCCL barrier / max-over-ranks timing / gradient all-reduce -- not scaling).
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/final
mkdir -p "$O"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/step" -o step -- \
    python3 "$R/bench.py" --no-cpu-baseline --no-policy --no-train --traffic off > "$O/step.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/train2" -o train2 -- \
    python3 "$R/tools/bench_update.py" --episodes 1048576 --repeats 1 --critic > "$O/train2.log" 2>&1 &&
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 5 --train-episodes 65536 > "$O/bench_2rank.log" 2>&1
