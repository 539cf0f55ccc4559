#!/bin/bash
# Round 4, first GPU check: the new lean-kernel rare-branch parity tests, the touched env / runner / C-ABI tests,
# the at-size tests with the ReLU-pattern flip bound, then a 2-rank torchrun (gloo) rehearsal of bench.py on the
# one GPU (rank 0 runs the PMC passes and the CPU baseline before any GPU call).  Outputs under gpurun_out/r4c1/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lean_rare.py tests/test_gpu_env.py tests/test_capi.py -m gpu -v -s \
    -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_env.log 2>&1 || { tail -40 $O/tests_env.log; exit 1; }
tail -1 $O/tests_env.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs_at_size.py "tests/test_gpu_ref_fixtures.py::test_runner_matches_reference_training_and_evaluation" \
    -m gpu -v -s -p no:cacheprovider --timeout 400 --timeout-method thread > $O/tests_at_size.log 2>&1 || { tail -40 $O/tests_at_size.log; exit 1; }
tail -1 $O/tests_at_size.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --steps 20 --warmup 5 --no-train > $O/bench_2rank.log 2>&1 || { tail -30 $O/bench_2rank.log; exit 1; }
tail -c 3000 $O/bench_2rank.log
echo DONE > $O/done.log
