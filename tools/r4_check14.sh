#!/bin/bash
# Round 4: the deep critic by time rows (no V(s') forward) and the paired one-hot dW1 scatter -- deep-kernel tests
# and the reference runner config (timing + kernel stats).  Outputs under gpurun_out/r4c14/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c14
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_deep.py -m gpu -v -s -p no:cacheprovider -k "onehot or rollout" --timeout 300 \
    --timeout-method thread > $O/tests_deep.log 2>&1 || { tail -60 $O/tests_deep.log; exit 1; }
tail -1 $O/tests_deep.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_refconf -o rc -- python3 tools/bench_refconfig.py --label round4 > $O/refconf.log 2>&1 || { tail -30 $O/refconf.log; exit 1; }
grep '^{' $O/refconf.log | cut -c1-330
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r4c14/prof_refconf/*kernel_stats.csv")[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:6]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.1f} ms {int(r['Calls']):6d} calls {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:90]}")
PY
echo DONE > $O/done.log
