#!/bin/bash
# TOOL (GPU box): the one-hot layer-0 kernel alone (tools/bench_l0.py) under rocprofv3 kernel stats, for the shipped
# library and the timing-probe builds (tools/build_variants.py --tu g2048_deep.hip p1=G2048_L0_PROBE=1
# p2=G2048_L0_PROBE=2), plus a one-group-per-CU run (8,192 boards: the launch's fixed cost).  Out: gpurun_out/$RUN/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${RUN:-l0ab}
mkdir -p "$O"
run() {   # name lib [bench args]
    local name=$1 lib=$2
    shift 2
    G2048_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$name" -o l0 -- \
        python3 tools/bench_l0.py "$@" > "$O/$name.log" 2>&1 || { tail -5 "$O/$name.log"; return 1; }
    grep '^{' "$O/$name.log"
    python3 - "$O/$name/l0_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "onehot_l0" in r["Name"] or "deep_hidden" in r["Name"]:
        print("   ", round(float(r["AverageNs"]) / 1e3, 1), "us", r["Calls"], r["Name"][:60])
PY
}
run shipped "" && run small "" --boards 8192 || exit 1
[ "${PROBES:-1}" = 0 ] || { run p1 tools/libg2048_p1.so && run p2 tools/libg2048_p2.so; }
