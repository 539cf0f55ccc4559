#!/bin/bash
# One GPU session: parity tests, smoke, a short bench.  Each GPU step has its own time limit; the steps are
# chained with && so nothing else runs on the GPU after a failure (the script exits with that step's status).
set -o pipefail
O=${O:-gpurun_out}
mkdir -p $O
T=${T:-tests}
timeout -k 10 ${TT:-900} python -u -m pytest $T -m gpu -x --tb=short -v -p no:cacheprovider --timeout 240 \
        --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1
rc=$?
echo "GPU ROUND EXIT $rc"
exit $rc
