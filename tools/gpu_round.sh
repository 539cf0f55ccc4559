#!/bin/bash
# One GPU session: parity tests, smoke, a short bench and a rocprofv3 kernel-trace profile.  Each GPU step has
# its own time limit; steps are chained with && so nothing else runs on the GPU after a failure.
set -o pipefail
mkdir -p gpurun_out
T=${T:-tests/test_gpu_env.py tests/test_gpu_agent.py}
timeout -k 10 500 python -u -m pytest $T -m gpu --tb=short -v -p no:cacheprovider --timeout 240 > gpurun_out/tests.log 2>&1; echo "TESTS EXIT $?" >> gpurun_out/tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "SMOKE EXIT $?" >> gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --traffic off > gpurun_out/bench.log 2>&1; echo "BENCH EXIT $?" >> gpurun_out/bench.log
