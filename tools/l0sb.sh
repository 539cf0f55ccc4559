#!/bin/bash
# TOOL (GPU box): the layer-0 kernel alone for the shipped library and the G2048_L0_SB=2 / 4 builds
# (tools/build_variants.py --tu g2048_deep.hip sb2=G2048_L0_SB=2 sb4=G2048_L0_SB=4), interleaved twice.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${RUN:-l0sb}
mkdir -p "$O"
for r in 1 2; do
    for v in shipped sb2 sb4; do
        lib=""
        [ "$v" = shipped ] || lib=tools/libg2048_$v.so
        G2048_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$v$r" -o l0 -- \
            python3 tools/bench_l0.py > "$O/$v$r.log" 2>&1 || { tail -5 "$O/$v$r.log"; exit 1; }
        python3 - "$O/$v$r/l0_kernel_stats.csv" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "onehot_l0" in r["Name"]:
        print(sys.argv[2], round(float(r["AverageNs"]) / 1e3, 1), "us", r["Calls"])
PY
    done
done
