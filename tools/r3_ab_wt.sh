#!/bin/bash
# Round 3: write-through 16-B stores (G2048_WT=1) against the lean build, interleaved; env parity on the variant.
set -o pipefail
O=gpurun_out/ab_wt
mkdir -p $O
G2048_TOOLS_LIB=tools/libg2048_wt.so timeout -k 10 400 python -u -m pytest tests/test_gpu_env.py tests/test_gpu_ref_fixtures.py -m gpu -x -q \
    -p no:cacheprovider --timeout 240 --timeout-method thread -k "env or step or obs or reset" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
O=$O bash tools/ab_libs.sh tools/libg2048_lean.so tools/libg2048_wt.so || exit 1
echo DONE >> $O/ab.log
