#!/bin/bash
# Gradient-path check on one box: the fused-gradient parity tests (torch backprop, reference fixtures, configs at
# size), then the configs[1] / configs[2] update timings and a kernel-trace summary of configs[2].
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=${O:-$R/gpurun_out/gradchk}
mkdir -p "$O"
timeout -k 10 700 python3 -u -m pytest ${GT:-tests/test_gpu_grad.py tests/test_gpu_ref_fixtures.py tests/test_gpu_configs_at_size.py} \
    -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 &&
timeout -k 10 300 python3 -u tools/bench_update.py --episodes 65536 1048576 --repeats 2 --critic > "$O/update.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/train2" -o train2 -- \
    python3 "$R/tools/bench_update.py" --episodes 1048576 --repeats 1 --critic > "$O/train2.log" 2>&1
rc=$?
tail -3 "$O/tests.log"
exit $rc
