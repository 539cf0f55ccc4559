set -o pipefail
O=gpurun_out/r7c
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/gap_c2 -o run -- python3 tools/bench_update.py --episodes 1048576 --repeats 1 --critic > $O/gap_c2.log 2>&1 &&
python3 tools/gap_profile.py $O/gap_c2 --after grad_coop_kernel > $O/gap_c2_summary.txt && cat $O/gap_c2_summary.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/gap_rc -o run -- python3 tools/bench_refconfig.py --episodes 1048576 > $O/gap_rc.log 2>&1 &&
python3 tools/gap_profile.py $O/gap_rc --after onehot_l0_mfma_kernel > $O/gap_rc_summary.txt && cat $O/gap_rc_summary.txt &&
python3 tools/gap_profile.py $O/gap_rc --after deep_rollout_kernel --before deep_rollout_kernel > $O/gap_rc_rollout_summary.txt && cat $O/gap_rc_rollout_summary.txt
rc=$?
find $O -name '*_kernel_trace.csv' -size +4M -delete
exit $rc
