#!/bin/bash
# one-hot gather with unguarded loads (batches of cells issued back to back): deep suites + runner-config profile
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4c20
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_deep.py > $O/tests_deep.log 2>&1 || { tail -30 $O/tests_deep.log; exit 1; }
tail -2 $O/tests_deep.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_refconf -o rc -- python3 tools/bench_refconfig.py --label gather > $O/refconf.log 2>&1 || { tail -30 $O/refconf.log; exit 1; }
grep '^{' $O/refconf.log | cut -c1-330
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/r4c20/prof_refconf/rc_kernel_stats.csv")):
    if any(k in r["Name"] for k in ("deep_", "onehot")):
        print(r["Name"][:60], r["Calls"], round(float(r["TotalDurationNs"]) / 1e6, 1), "ms")
PY
