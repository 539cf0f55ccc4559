#!/bin/bash
# One parameterised GPU-box script (replaces round 3/4's one-off r3_*.sh / r4_*.sh checks): runs the named steps in
# order, each under its own time limit, and stops at the first failure.  Outputs under gpurun_out/$RUN/.
#
#   RUN=r5a tools/gpu.sh tests:tests/test_gpu_deep.py refconf pmc_refconf:262144 bench smoke prof_step
#
# steps:
#   tests[:ARGS]        pytest -m gpu over ARGS (shell-parsed after the colon; default: the whole suite)
#   smoke               __graft_entry__.smoke()
#   bench               the driver's bench command (bench.py --gpus 1 --steps 20 --warmup 5)
#   prof_step           rocprofv3 kernel stats of 200 step-kernel launches (bench.py step leg only)
#   trace_bench         the driver's bench command under a rocprofv3 kernel trace; tools/trace_window.py reads the
#                       timed launches back (headline + configs[4] legs) beside the line's kernel_ms
#   rehearse8           bench.py under torchrun with 8 ranks sharing the one GPU (gloo): the N = 8 flow end to end
#   prof_c4             rocprofv3 kernel stats of 200 launches of configs[4]'s Philox + one-hot step leg
#   refconf[:EPISODES]  tools/bench_refconfig.py under rocprofv3 --kernel-trace --stats; the top kernels printed
#   pmc_refconf[:E]     PMC passes over the runner config at E episodes (default 262144): SQ busy / LDS, SQ waits,
#                       FETCH_SIZE, WRITE_SIZE, TCC hit / miss -- one counter group per run; tools/pmc_grad_summary.py
#   pmc_configs2        the same passes over one configs[2] update (tools/bench_update.py, 1,048,576 episodes)
#   abref:LIB[:N]       N (default 2) interleaved runner-config iterations: the shipped library, then LIB
#   abmulti:L1,L2,..[:N] N interleaved runner-config rounds: shipped, then each library
#   abstep:LIB[:N[:ARGS]] N interleaved rounds of bench.py's step leg alone, shipped then LIB (ARGS: e.g. --rng philox --obs onehot)
#   cmd:'...'           any other command (its own timeout inside)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${RUN:-gpu}
mkdir -p "$O"

top_kernels() {   # $1 = kernel_stats.csv
    python3 - "$1" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.1f} ms {int(r['Calls']):6d} calls {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:96]}")
PY
}

pmc_passes() {   # $1 = dir, rest = command
    local d=$1
    shift
    local P="--kernel-trace --output-format csv"
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$d/trace" -o run -- "$@" > "$d/trace.log" 2>&1 &&
    timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS \
        SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE $P -d "$d/sq" -o run -- "$@" > "$d/sq.log" 2>&1 &&
    timeout -s KILL 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
        SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_COEXEC_CYCLES $P -d "$d/sqw" -o run -- "$@" > "$d/sqw.log" 2>&1 &&
    timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE $P -d "$d/fetch" -o run -- "$@" > "$d/fetch.log" 2>&1 &&
    timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE $P -d "$d/write" -o run -- "$@" > "$d/write.log" 2>&1 &&
    timeout -s KILL 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum $P -d "$d/tcc" -o run -- "$@" > "$d/tcc.log" 2>&1 &&
    python3 tools/pmc_grad_summary.py "$d" > "$d/summary.jsonl" && cat "$d/summary.jsonl" &&
    # the per-dispatch CSVs run to 100s of MiB (gpurun copies back at most 64 MiB): keep the summary and the stats
    find "$d" \( -name '*_counter_collection.csv' -o -name '*_kernel_trace.csv' \) -size +4M -delete
}

for step in "$@"; do
    name=${step%%:*}
    arg=""
    [[ "$step" == *:* ]] && arg=${step#*:}
    echo "=== $step" | cut -c1-200
    case $name in
    tests)
        # ARGS is shell-parsed (quote a -k expression inside it: "tests:tests/x.py -k 'a or b'")
        eval "timeout -k 10 900 python3 -u -m pytest ${arg:-tests} -m gpu -v -s -p no:cacheprovider --timeout 300 \
            --timeout-method thread" > "$O/tests_${RUN:-gpu}_$SECONDS.log" 2>&1
        rc=$?
        tail -3 "$(ls -t "$O"/tests_*.log | head -1)" || true
        [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" "$(ls -t "$O"/tests_*.log | head -1)" | head -40; exit 1; }
        ;;
    smoke)
        timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > "$O/smoke.log" 2>&1 ||
            { tail -20 "$O/smoke.log"; exit 1; }
        tail -1 "$O/smoke.log"
        ;;
    bench)
        timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver_cmd.log" 2>&1 ||
            { tail -20 "$O/bench_driver_cmd.log"; exit 1; }
        grep '^{' "$O/bench_driver_cmd.log" | cut -c1-400
        ;;
    trace_bench)
        # the driver's bench command itself under a rocprofv3 kernel trace: its timed launches read back
        # (tools/trace_window.py) beside the line's HIP-event kernel_ms; then the per-kernel stats of the same run
        timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_bench" -o tb -- \
            python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$O/trace_bench.log" 2>&1 ||
            { tail -20 "$O/trace_bench.log"; exit 1; }
        grep '^{' "$O/trace_bench.log" | cut -c1-300
        python3 tools/trace_window.py "$O/trace_bench" "$O/trace_bench.log" --keep "$O/trace_bench_step_rows.csv" \
            > "$O/trace_window.json" && cat "$O/trace_window.json"
        top_kernels "$O/trace_bench/tb_kernel_stats.csv"
        find "$O/trace_bench" -name '*_kernel_trace.csv' -size +4M -delete
        ;;
    prof_c4)
        # rocprofv3 kernel stats of configs[4]'s step leg alone (Philox + one-hot obs + int8 mask, 1M boards)
        timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_c4" -o c4 -- \
            python3 bench.py --rng philox --obs onehot --no-cpu-baseline --no-policy --no-train --no-configs4 \
            --traffic off --steps 200 --warmup 20 > "$O/prof_c4.log" 2>&1 || { tail -20 "$O/prof_c4.log"; exit 1; }
        grep '^{' "$O/prof_c4.log" | cut -c1-300
        top_kernels "$O/prof_c4/c4_kernel_stats.csv"
        ;;
    rehearse8)
        # bench.py's N = 8 flow on ONE GPU (8 ranks share it: the gloo fallback) -- rank 0's PMC children and CPU
        # baseline before init_process_group, every leg's barriers and max-over-ranks reduce; value is not scaling
        HSA_ENABLE_IPC_MODE_LEGACY=0 timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
            --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --steps 20 --warmup 5 --boards 65536 \
            --train-episodes 4096 > "$O/rehearse8.log" 2>&1 || { tail -30 "$O/rehearse8.log"; exit 1; }
        grep '^{' "$O/rehearse8.log" | cut -c1-400
        ;;
    prof_step)
        timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_step" -o step -- \
            python3 bench.py --no-cpu-baseline --no-policy --no-train --no-refconfig --no-configs4 --traffic off --steps 200 --warmup 20 \
            > "$O/prof_step.log" 2>&1 || { tail -20 "$O/prof_step.log"; exit 1; }
        grep '^{' "$O/prof_step.log" | cut -c1-300
        top_kernels "$O/prof_step/step_kernel_stats.csv"
        ;;
    refconf)
        # shellcheck disable=SC2086
        timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_refconf" -o rc -- \
            python3 tools/bench_refconfig.py --label "${RUN:-gpu}" ${arg:+--episodes $arg} > "$O/refconf.log" 2>&1 ||
            { tail -30 "$O/refconf.log"; exit 1; }
        grep '^{' "$O/refconf.log" | cut -c1-330
        top_kernels "$O/prof_refconf/rc_kernel_stats.csv"
        ;;
    pmc_refconf)
        mkdir -p "$O/pmc_refconf"
        pmc_passes "$O/pmc_refconf" python3 tools/bench_refconfig.py --episodes "${arg:-262144}" || exit 1
        ;;
    pmc_configs2)
        mkdir -p "$O/pmc_configs2"
        pmc_passes "$O/pmc_configs2" python3 tools/bench_update.py --episodes 1048576 --repeats 1 --critic || exit 1
        ;;
    abref)
        lib=${arg%%:*}
        n=2
        [[ "$arg" == *:* ]] && n=${arg#*:}
        tag=ab$SECONDS
        for r in $(seq "$n"); do
            timeout -k 10 300 python3 tools/bench_refconfig.py --label shipped > "$O/${tag}_shipped_$r.log" 2>&1 || exit 1
            G2048_LIB=$lib timeout -k 10 300 python3 tools/bench_refconfig.py --label "$(basename "$lib")" > "$O/${tag}_var_$r.log" 2>&1 || exit 1
        done
        grep -h '^{' "$O"/"$tag"_*.log | cut -c1-220
        ;;
    abmulti)
        # abmulti:LIB1,LIB2,...[:N] -- N interleaved rounds of the runner config: the shipped library, then each LIB
        libs=${arg%%:*}
        n=2
        [[ "$arg" == *:* ]] && n=${arg#*:}
        tag=abm$SECONDS
        for r in $(seq "$n"); do
            timeout -k 10 300 python3 tools/bench_refconfig.py --label shipped > "$O/${tag}_shipped_$r.log" 2>&1 || exit 1
            for lib in ${libs//,/ }; do
                G2048_LIB=$lib timeout -k 10 300 python3 tools/bench_refconfig.py --label "$(basename "$lib")" \
                    > "$O/${tag}_$(basename "$lib" .so)_$r.log" 2>&1 || exit 1
            done
        done
        grep -h '^{' "$O"/"$tag"_*.log | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l)
    if d['episodes'] > 100000:
        print(f\"{d['label'][:24]:24s} rep {d['rep']} update {d['update_s']:.4f} rollout {d['rollout_s']:.4f}\")"
        ;;
    abstep)
        # abstep:LIB[:N[:BENCH ARGS]] -- N interleaved rounds of the step leg alone (200 launches), shipped then LIB
        lib=${arg%%:*}
        rest=""
        [[ "$arg" == *:* ]] && rest=${arg#*:}
        n=${rest%%:*}
        n=${n:-3}
        extra=""
        [[ "$rest" == *:* ]] && extra=${rest#*:}
        tag=abstep$SECONDS
        for r in $(seq "$n"); do
            # shellcheck disable=SC2086
            timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-policy --no-train --no-configs4 --traffic off \
                --steps 200 --warmup 20 $extra > "$O/${tag}_shipped_$r.log" 2>&1 || exit 1
            # shellcheck disable=SC2086
            timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-policy --no-train --no-configs4 --traffic off \
                --steps 200 --warmup 20 $extra --lib "$lib" > "$O/${tag}_var_$r.log" 2>&1 || exit 1
        done
        for f in "$O"/"$tag"_*.log; do
            python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1].split('/')[-1], round(d['roofline']['kernel_ms']*1e3, 2), 'us', round(d['roofline']['frac'], 4))" "$f"
        done
        ;;
    cmd)
        bash -o pipefail -c "$arg" || exit 1
        ;;
    *)
        echo "unknown step $step"
        exit 2
        ;;
    esac
done
echo DONE > "$O/done.log"
