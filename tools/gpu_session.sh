#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel-trace stats.
# Every GPU step has its own time limit; a crash, abort or timeout (exit code
# other than 0, or 1 = "tests failed") ends the session so nothing else runs on
# a possibly faulted GPU.  Output lands in gpurun_out/<tag>/.
#   tools/gpu_session.sh <tag> [steps...]   steps: test smoke bench prof pmc e2e_c4 e2e_ref ...
set -u
TAG=${1:-r01}
shift || true
STEPS=${*:-test smoke bench prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ok_or_fail() {  # rc, step
    if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then
        echo "step $2 ended with $1 (crash/timeout): stopping" | tee -a "$OUT/session.log"
        exit "$1"
    fi
}
for s in $STEPS; do
    echo "== $s $(date +%T)" | tee -a "$OUT/session.log"
    case $s in
    test)
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rfs --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
        rc=$?; tail -5 "$OUT/pytest_gpu.log"; ok_or_fail $rc test ;;
    tk)  # a subset of the GPU suite: TK = a -k expression, TKPATH = test files (default tests)
        timeout -k 10 600 python -u -m pytest -m gpu -x -v -rfs --timeout 240 --timeout-method thread -k "${TK:-}" ${TKPATH:-tests} > "$OUT/pytest_tk.log" 2>&1
        rc=$?; tail -8 "$OUT/pytest_tk.log"; ok_or_fail $rc tk ;;
    ctx)  # the in-process multi-GPU children at the GPUs this box has, each with its parity object
        for A in "range northstar" "rs northstar" "rs c4" "range c5 --h2d"; do
            set -- $A
            H=""; [ "${3:-}" = "--h2d" ] && H="--h2d --steps 2 --warmup 1"
            timeout -k 10 240 python bench.py --ctx-multi $1 --workload $2 $H >> "$OUT/ctx.jsonl" 2>> "$OUT/ctx.err"
            rc=$?; tail -c 700 "$OUT/ctx.jsonl"; echo; ok_or_fail $rc "ctx $A"
        done ;;
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
        rc=$?; tail -3 "$OUT/smoke.log"; ok_or_fail $rc smoke ;;
    bench)
        FA_BENCH_FULL="$OUT/bench_full.json" timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
        rc=$?; cat "$OUT/bench.json"; wc -c "$OUT/bench.json"; tail -3 "$OUT/bench.err"; ok_or_fail $rc bench ;;
    prof)
        timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
            python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-live-pmc > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
        rc=$?; tail -3 "$OUT/prof.err"; ok_or_fail $rc prof ;;
    pmc)
        for c in FETCH_SIZE WRITE_SIZE; do
            timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$OUT/pmc_$c" -o run -- \
                python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-live-pmc > "$OUT/pmc_$c.json" 2> "$OUT/pmc_$c.err"
            rc=$?; tail -2 "$OUT/pmc_$c.err"; ok_or_fail $rc pmc_$c
        done ;;
    pmcw)  # the same passes for the secondary workloads whose traffic bench.py reports
        bash tools/pmc_workloads.sh "$TAG" ${PMC_WORKLOADS:-c2 c3 c4 c4r c5 c5r ns_w2 ns_w4 ns_w8}
        rc=$?; ok_or_fail $rc pmcw ;;
    layouts)
        for L in rs chain; do
            timeout -k 10 300 python bench.py --layout $L --steps 10 --no-cpu-baseline --no-secondary --no-live-pmc > "$OUT/bench_$L.json" 2> "$OUT/bench_$L.err"
            rc=$?; cat "$OUT/bench_$L.json"; tail -2 "$OUT/bench_$L.err"; ok_or_fail $rc layout_$L
        done ;;
    h2d)
        for G in 1 2 4; do
            timeout -k 10 600 python tools/h2d_rate.py 8 26 3 $G >> "$OUT/h2d.jsonl" 2>> "$OUT/h2d.err"
            rc=$?; tail -1 "$OUT/h2d.jsonl"; tail -2 "$OUT/h2d.err"; ok_or_fail $rc h2d_$G
        done ;;
    ranks)  # multi-rank rehearsal of the driver's N>1 launch: bench.py spawns 2 ranks, which share the one GPU over gloo
        timeout -k 10 600 python bench.py --gpus 2 --steps 5 --warmup 2 > "$OUT/bench_2ranks.json" 2> "$OUT/bench_2ranks.err"
        rc=$?; cat "$OUT/bench_2ranks.json"; tail -3 "$OUT/bench_2ranks.err"; ok_or_fail $rc ranks ;;
    rslaunch)  # local launch pattern of the rs / chain layouts at 4 and 8 ranks (tools/rs_launch.py)
        for W in 8 4; do
            timeout -k 10 300 python tools/rs_launch.py $W 16 10 >> "$OUT/rs_launch.jsonl" 2>> "$OUT/rs_launch.err"
            rc=$?; tail -1 "$OUT/rs_launch.jsonl"; ok_or_fail $rc rslaunch_$W
        done ;;
    slices)  # one rank's share of the strong-scaled north star at W = 1, 2, 4, 8 (tools/strong_slices.py)
        timeout -k 10 300 python tools/strong_slices.py 20 > "$OUT/slices.jsonl" 2> "$OUT/slices.err"
        rc=$?; cat "$OUT/slices.jsonl"; tail -2 "$OUT/slices.err"; ok_or_fail $rc slices ;;
    rounds)  # one aggregator round on its own buckets, batched vs per part (tools/rounds.py) + kernel trace
        timeout -k 10 300 python tools/rounds.py 20 round_c2,round_c3,round_c4 > "$OUT/rounds.jsonl" 2> "$OUT/rounds.err"
        rc=$?; cat "$OUT/rounds.jsonl"; tail -2 "$OUT/rounds.err"; ok_or_fail $rc rounds
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rounds_prof" -o run -- \
            python3 tools/rounds.py 20 round_c2,round_c3 > "$OUT/rounds_prof.jsonl" 2> "$OUT/rounds_prof.err"
        rc=$?; tail -2 "$OUT/rounds_prof.err"; ok_or_fail $rc rounds_prof ;;
    markers)  # roctx ranges of the host entries (fa_submit / fa_finalize / fa_copy_output) beside kernels and copies
        # D2H copies are HIP blit kernels here (kernel trace: __amd_rocclr_copyBuffer), H2D copies SDMA
        # (memory-copy trace); tools/copy_stats.py puts both directions in one table
        H2D_MODES=${H2D_MODES:-pinned_io} timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --memory-copy-trace \
            --stats --output-format csv -d "$OUT/markers" -o run -- python3 tools/h2d_rate.py 8 24 3 > "$OUT/markers.jsonl" 2> "$OUT/markers.err"
        rc=$?; tail -2 "$OUT/markers.err"; ok_or_fail $rc markers
        python3 tools/copy_stats.py "$OUT/markers" "$OUT/markers_copy_stats.csv" > "$OUT/markers_breakdown.json" ;;
    e2e)
        timeout -k 10 900 python tools/e2e_bench.py 4 3 > "$OUT/e2e_bench.json" 2> "$OUT/e2e_bench.err"
        rc=$?; cat "$OUT/e2e_bench.json"; tail -3 "$OUT/e2e_bench.err"; ok_or_fail $rc e2e ;;
    e2e_c4)  # C4's own client count through the drop-in process: D = 64 VGG-19 owners, range / eager / rs layouts
        for L in "" "--eager" "--layout rs"; do
            E2E_NO_REF=1 timeout -k 10 600 python tools/e2e_bench.py 64 3 $L >> "$OUT/e2e_c4.jsonl" 2>> "$OUT/e2e_c4.err"
            rc=$?; tail -c 600 "$OUT/e2e_c4.jsonl"; echo; ok_or_fail $rc "e2e_c4 $L"
        done ;;
    e2e_ref)  # C2 and C3 through the reference's own process and through fa_aggregator, same receipts
        (while true; do date >> "$OUT/heartbeat"; sleep 45; done) &  # a reference leg is silent for minutes
        HB=$!
        for C in c2 c3; do
            timeout -k 10 900 python -u tools/e2e_ref.py $C 2 5 >> "$OUT/e2e_ref.jsonl" 2>> "$OUT/e2e_ref.err"
            rc=$?; tail -c 600 "$OUT/e2e_ref.jsonl"; echo
            [ "$rc" -ne 0 ] && kill $HB
            ok_or_fail $rc "e2e_ref $C"
        done
        kill $HB ;;
    e2e_c4s)  # C4 at D = 64 through the drop-in, streaming ingest off / on (tools/e2e_bench.py)
        for A in "--stream-min-bytes 0" ""; do
            E2E_NO_REF=1 timeout -k 10 600 python tools/e2e_bench.py 64 3 $A >> "$OUT/e2e_c4s.jsonl" 2>> "$OUT/e2e_c4s.err"
            rc=$?; tail -c 600 "$OUT/e2e_c4s.jsonl"; echo; ok_or_fail $rc "e2e_c4s $A"
        done ;;
    stream_ab)  # streaming ingest on / off, alternating, C2 and C3 through the drop-in (tools/e2e_ref.py)
        for C in ${STREAM_CFGS:-c2 c3}; do
            for i in 1 2; do
                for A in "--stream-min-bytes 0" ""; do
                    E2E_ONLY_FA=1 E2E_AGG_ARGS="$A" timeout -k 10 600 python -u tools/e2e_ref.py $C 0 10 >> "$OUT/stream_ab.jsonl" 2>> "$OUT/stream_ab.err"
                    rc=$?; tail -c 400 "$OUT/stream_ab.jsonl"; echo; ok_or_fail $rc "stream_ab $C"
                done
            done
        done ;;
    probe)
        hipcc --offload-arch=gfx950 -O3 tools/hbm_probe.hip -o "$OUT/hbm_probe" > "$OUT/probe_build.log" 2>&1 &&
        timeout -k 10 300 "$OUT/hbm_probe" > "$OUT/hbm_probe.json" 2> "$OUT/probe.err"
        rc=$?; cat "$OUT/hbm_probe.json"; ok_or_fail $rc probe ;;
    sweep)
        timeout -k 10 600 python tools/sweep.py northstar > "$OUT/sweep_northstar.jsonl" 2> "$OUT/sweep.err"
        rc=$?; head -5 "$OUT/sweep_northstar.jsonl"; ok_or_fail $rc sweep
        timeout -k 10 600 python tools/sweep.py c2 > "$OUT/sweep_c2.jsonl" 2>> "$OUT/sweep.err"
        rc=$?; head -5 "$OUT/sweep_c2.jsonl"; ok_or_fail $rc sweep_c2 ;;
    unroll)  # unroll sweep per workload (block 128, sc1 stores), 3 pools each, interleaved in one process
        for W in c2 c3 northstar; do
            SWEEP_BLOCKS=128 SWEEP_STORES=3 SWEEP_UNROLLS=4,8,16 timeout -k 10 300 python tools/sweep.py $W \
                > "$OUT/sweep_unroll_$W.jsonl" 2>> "$OUT/sweep.err"
            rc=$?; cat "$OUT/sweep_unroll_$W.jsonl"; ok_or_fail $rc unroll_$W
        done ;;
    walk)  # grid walk sweep per workload (block 128, unroll 16, sc1 stores), 3 pools, one process
        for W in northstar c3 c4 c5r c2; do
            SWEEP_BLOCKS=128 SWEEP_STORES=3 SWEEP_UNROLLS=16 SWEEP_WALKS=${WALKS:-2,4} timeout -k 10 300 python tools/sweep.py $W \
                > "$OUT/sweep_walk_$W.jsonl" 2>> "$OUT/sweep.err"
            rc=$?; cat "$OUT/sweep_walk_$W.jsonl"; ok_or_fail $rc walk_$W
        done ;;
    bench3)  # three bench runs (fresh process each): the spread of pool placement
        for i in 1 2 3; do
            timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --no-live-pmc > "$OUT/bench3_$i.json" 2> "$OUT/bench3_$i.err"
            rc=$?; cat "$OUT/bench3_$i.json"; ok_or_fail $rc bench3_$i
        done ;;
    *)
        echo "unknown step $s" ;;
    esac
done
echo "== done $(date +%T)" | tee -a "$OUT/session.log"
