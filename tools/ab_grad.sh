#!/bin/bash
# A/B of grad_kernel build variants (tools/libg2048_c<CPOL>p<PIPE>.so, built from an experimental source with
# -DG2048_GRAD_CPOL (column-store cache policy) / -DG2048_GRAD_PIPE (pipelined tile epilogues); both were measured
# slower or equal and removed -- DESIGN.md section 3, profiles/round1/ab_grad/): parity of the pipelined variant on the
# gradient tests, then a rocprofv3 kernel-trace summary of the configs[1] actor-critic update per variant.
# Outputs under gpurun_out/ab_grad/.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/ab_grad
mkdir -p "$O"
G2048_DIAG_LIB=$R/tools/libg2048_c0p2.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_grad.py -x -q \
    --timeout 240 --timeout-method thread -p no:cacheprovider > "$O/tests_c0p2.log" 2>&1 || exit 1
for v in c0p0 c0p1 c0p2 c0p0; do
    G2048_DIAG_LIB=$R/tools/libg2048_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$O/$v" -o run -- python3 "$R/tools/bench_update.py" --episodes 65536 --repeats 2 --critic \
        > "$O/$v.log" 2>&1 || exit 1
done
