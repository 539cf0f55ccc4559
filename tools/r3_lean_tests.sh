#!/bin/bash
# Round 3: the GPU parity tests that run the lean (log2-reward, no-score) step kernel.
set -o pipefail
O=gpurun_out/lean_tests
mkdir -p $O
timeout -k 10 900 python -u -m pytest "tests/test_gpu_env.py::test_env_step_vs_oracle" tests/test_gpu_env_large.py \
    "tests/test_gpu_configs_at_size.py::test_configs4_shard_philox_onehot_1m_lanes" -m gpu -v -s -p no:cacheprovider \
    --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
exit $rc
