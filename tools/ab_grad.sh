#!/bin/bash
# A/B of grad_kernel build variants tools/libg2048_<variant>.so (built with -D options of csrc/g2048_policy.hip):
#     bash tools/ab_grad.sh <variant to parity-test> <variant> [<variant> ...]
# runs the gradient parity tests on the first variant, then a rocprofv3 kernel-trace summary of the configs[1]
# actor-critic update per listed variant.  Outputs under gpurun_out/ab_grad/.  Past runs: DESIGN.md section 3,
# profiles/round1/ab_grad/ (pipelined tile epilogues, non-temporal column stores, prefetch depth).
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/ab_grad
mkdir -p "$O"
T=$1
shift
G2048_TOOLS_LIB=$R/tools/libg2048_$T.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_grad.py -x -q \
    --timeout 240 --timeout-method thread -p no:cacheprovider > "$O/tests_$T.log" 2>&1 || exit 1
i=0
for v in "$@"; do
    i=$((i + 1))
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$O/$i-$v" -o run -- python3 "$R/tools/bench_update.py" --episodes 65536 --repeats 2 --critic --lib $R/tools/libg2048_$v.so \
        > "$O/$i-$v.log" 2>&1 || exit 1
done
