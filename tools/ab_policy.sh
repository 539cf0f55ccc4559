set -o pipefail
O=gpurun_out/abpol
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_policy.py tests/test_gpu_ref_fixtures.py tests/test_gpu_grad.py tests/test_gpu_agent.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do for lib in tools/libg2048_prev.so rl-2048-with-reinforce-and-actor-critic_amd/libg2048.so; do
  echo "== $lib" >> $O/ab.log
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-train --traffic off --steps 50 --warmup 5 --lib $lib >> $O/ab.log 2>&1 || exit 1
done; done
