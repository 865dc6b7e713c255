#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel-trace stats.
# Every GPU step has its own time limit; a crash, abort or timeout (exit code
# other than 0, or 1 = "tests failed") ends the session so nothing else runs on
# a possibly faulted GPU.  Output lands in gpurun_out/<tag>/.
#   tools/gpu_session.sh <tag> [steps...]   steps: test smoke bench prof pmc
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
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
        rc=$?; tail -3 "$OUT/smoke.log"; ok_or_fail $rc smoke ;;
    bench)
        timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
        rc=$?; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"; ok_or_fail $rc bench ;;
    prof)
        timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
            python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
        rc=$?; tail -3 "$OUT/prof.err"; ok_or_fail $rc prof ;;
    pmc)
        for c in FETCH_SIZE WRITE_SIZE; do
            timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$OUT/pmc_$c" -o run -- \
                python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > "$OUT/pmc_$c.json" 2> "$OUT/pmc_$c.err"
            rc=$?; tail -2 "$OUT/pmc_$c.err"; ok_or_fail $rc pmc_$c
        done ;;
    layouts)
        for L in rs chain; do
            timeout -k 10 300 python bench.py --layout $L --steps 10 --no-cpu-baseline --no-secondary > "$OUT/bench_$L.json" 2> "$OUT/bench_$L.err"
            rc=$?; cat "$OUT/bench_$L.json"; tail -2 "$OUT/bench_$L.err"; ok_or_fail $rc layout_$L
        done ;;
    h2d)
        timeout -k 10 600 python tools/h2d_rate.py 8 26 3 > "$OUT/h2d.jsonl" 2> "$OUT/h2d.err"
        rc=$?; cat "$OUT/h2d.jsonl"; tail -2 "$OUT/h2d.err"; ok_or_fail $rc h2d ;;
    outexp)
        timeout -k 10 600 python tools/exp_out.py 25 10 > "$OUT/exp_out.jsonl" 2> "$OUT/exp_out.err"
        rc=$?; cat "$OUT/exp_out.jsonl"; tail -2 "$OUT/exp_out.err"; ok_or_fail $rc outexp ;;
    ranks)  # multi-rank rehearsal of the driver's N>1 launch: bench.py spawns 2 ranks, which share the one GPU over gloo
        timeout -k 10 600 python bench.py --gpus 2 --steps 5 --warmup 2 > "$OUT/bench_2ranks.json" 2> "$OUT/bench_2ranks.err"
        rc=$?; cat "$OUT/bench_2ranks.json"; tail -3 "$OUT/bench_2ranks.err"; ok_or_fail $rc ranks ;;
    vmm)  # physical placement of the client pool via the VMM API (tools/exp_vmm.hip)
        hipcc --offload-arch=gfx950 -O2 tools/exp_vmm.hip -Iinclude -Lmultihop-federeated-split-learning_amd/lib -lfa \
            -Wl,-rpath,$PWD/multihop-federeated-split-learning_amd/lib -o "$OUT/exp_vmm" > "$OUT/vmm_build.log" 2>&1 &&
        timeout -k 10 400 "$OUT/exp_vmm" ${VMM_ARGS:-26 3} > "$OUT/exp_vmm.jsonl" 2> "$OUT/exp_vmm.err"
        rc=$?; cat "$OUT/exp_vmm.jsonl"; tail -3 "$OUT/exp_vmm.err"; ok_or_fail $rc vmm ;;
    outplace)  # where the output is written (tools/exp_out.hip)
        hipcc --offload-arch=gfx950 -O2 tools/exp_out.hip -Iinclude -Lmultihop-federeated-split-learning_amd/lib -lfa \
            -Wl,-rpath,$PWD/multihop-federeated-split-learning_amd/lib -o "$OUT/exp_out" > "$OUT/out_build.log" 2>&1 &&
        timeout -k 10 400 "$OUT/exp_out" ${OUT_ARGS:-26 4} > "$OUT/exp_out.jsonl" 2> "$OUT/exp_out.err"
        rc=$?; cat "$OUT/exp_out.jsonl"; tail -3 "$OUT/exp_out.err"; ok_or_fail $rc outplace ;;
    pick)  # K pools allocated in sequence, timed interleaved (tools/exp_pick.hip)
        hipcc --offload-arch=gfx950 -O2 tools/exp_pick.hip -Iinclude -Lmultihop-federeated-split-learning_amd/lib -lfa \
            -Wl,-rpath,$PWD/multihop-federeated-split-learning_amd/lib -o "$OUT/exp_pick" > "$OUT/pick_build.log" 2>&1 &&
        timeout -k 10 400 "$OUT/exp_pick" ${PICK_ARGS:-26 8 3} > "$OUT/exp_pick.jsonl" 2> "$OUT/exp_pick.err" &&
        timeout -k 10 400 "$OUT/exp_pick" ${PICK_ARGS2:-26 4 3 100} >> "$OUT/exp_pick.jsonl" 2>> "$OUT/exp_pick.err"
        rc=$?; cat "$OUT/exp_pick.jsonl"; tail -3 "$OUT/exp_pick.err"; ok_or_fail $rc pick ;;
    slow)  # where a slow pool loses its time (tools/exp_slow.hip)
        hipcc --offload-arch=gfx950 -O2 tools/exp_slow.hip -Iinclude -Lmultihop-federeated-split-learning_amd/lib -lfa \
            -Wl,-rpath,$PWD/multihop-federeated-split-learning_amd/lib -o "$OUT/exp_slow" > "$OUT/slow_build.log" 2>&1 &&
        timeout -k 10 400 "$OUT/exp_slow" ${SLOW_ARGS:-26 6 3} > "$OUT/exp_slow.jsonl" 2> "$OUT/exp_slow.err"
        rc=$?; cat "$OUT/exp_slow.jsonl"; tail -3 "$OUT/exp_slow.err"; ok_or_fail $rc slow ;;
    skew)  # per-slot skew inside the same pool (tools/exp_skew.hip)
        hipcc --offload-arch=gfx950 -O2 tools/exp_skew.hip -Iinclude -Lmultihop-federeated-split-learning_amd/lib -lfa \
            -Wl,-rpath,$PWD/multihop-federeated-split-learning_amd/lib -o "$OUT/exp_skew" > "$OUT/skew_build.log" 2>&1 &&
        timeout -k 10 400 "$OUT/exp_skew" ${SKEW_ARGS:-26 6 3} > "$OUT/exp_skew.jsonl" 2> "$OUT/exp_skew.err"
        rc=$?; cat "$OUT/exp_skew.jsonl"; tail -3 "$OUT/exp_skew.err"; ok_or_fail $rc skew ;;
    cross)  # inputs of pool p into the output of pool q (tools/exp_cross.hip)
        hipcc --offload-arch=gfx950 -O2 tools/exp_cross.hip -Iinclude -Lmultihop-federeated-split-learning_amd/lib -lfa \
            -Wl,-rpath,$PWD/multihop-federeated-split-learning_amd/lib -o "$OUT/exp_cross" > "$OUT/cross_build.log" 2>&1 &&
        timeout -k 10 400 "$OUT/exp_cross" ${CROSS_ARGS:-26 5 3} > "$OUT/exp_cross.jsonl" 2> "$OUT/exp_cross.err"
        rc=$?; cat "$OUT/exp_cross.jsonl"; tail -3 "$OUT/exp_cross.err"; ok_or_fail $rc cross ;;
    order)  # walk order of the grid over the buckets vs the slow-pool penalty (tools/exp_order.hip)
        hipcc --offload-arch=gfx950 -O2 tools/exp_order.hip -Iinclude -Lmultihop-federeated-split-learning_amd/lib -lfa \
            -Wl,-rpath,$PWD/multihop-federeated-split-learning_amd/lib -o "$OUT/exp_order" > "$OUT/order_build.log" 2>&1 &&
        timeout -k 10 400 "$OUT/exp_order" ${ORDER_ARGS:-26 5 3} > "$OUT/exp_order.jsonl" 2> "$OUT/exp_order.err"
        rc=$?; cat "$OUT/exp_order.jsonl"; tail -3 "$OUT/exp_order.err"; ok_or_fail $rc order ;;
    phase)  # reads and writes separated in time (tools/exp_phase.hip)
        hipcc --offload-arch=gfx950 -O2 tools/exp_phase.hip -Iinclude -Lmultihop-federeated-split-learning_amd/lib -lfa \
            -Wl,-rpath,$PWD/multihop-federeated-split-learning_amd/lib -o "$OUT/exp_phase" > "$OUT/phase_build.log" 2>&1 &&
        timeout -k 10 300 "$OUT/exp_phase" ${PHASE_ARGS:-26 5 3} > "$OUT/exp_phase.jsonl" 2> "$OUT/exp_phase.err"
        rc=$?; cat "$OUT/exp_phase.jsonl"; tail -3 "$OUT/exp_phase.err"; ok_or_fail $rc phase ;;
    phase2)  # variants of the phased kernel (tools/exp_phase2.hip)
        hipcc --offload-arch=gfx950 -O2 tools/exp_phase2.hip -Iinclude -Lmultihop-federeated-split-learning_amd/lib -lfa \
            -Wl,-rpath,$PWD/multihop-federeated-split-learning_amd/lib -o "$OUT/exp_phase2" > "$OUT/phase2_build.log" 2>&1 &&
        timeout -k 10 300 "$OUT/exp_phase2" ${PHASE_ARGS:-26 4 3} > "$OUT/exp_phase2.jsonl" 2> "$OUT/exp_phase2.err"
        rc=$?; cat "$OUT/exp_phase2.jsonl"; tail -3 "$OUT/exp_phase2.err"; ok_or_fail $rc phase2 ;;
    phase3)  # register-staged phases and soft barriers (tools/exp_phase3.hip)
        hipcc --offload-arch=gfx950 -O2 tools/exp_phase3.hip -Iinclude -Lmultihop-federeated-split-learning_amd/lib -lfa \
            -Wl,-rpath,$PWD/multihop-federeated-split-learning_amd/lib -o "$OUT/exp_phase3" > "$OUT/phase3_build.log" 2>&1 &&
        timeout -k 10 300 "$OUT/exp_phase3" ${PHASE_ARGS:-26 4 3} > "$OUT/exp_phase3.jsonl" 2> "$OUT/exp_phase3.err"
        rc=$?; cat "$OUT/exp_phase3.jsonl"; tail -3 "$OUT/exp_phase3.err"; ok_or_fail $rc phase3 ;;
    rslaunch)  # local launch pattern of the rs / chain layouts at 4 and 8 ranks (tools/rs_launch.py)
        for W in 8 4; do
            timeout -k 10 300 python tools/rs_launch.py $W 16 10 >> "$OUT/rs_launch.jsonl" 2>> "$OUT/rs_launch.err"
            rc=$?; tail -1 "$OUT/rs_launch.jsonl"; ok_or_fail $rc rslaunch_$W
        done ;;
    slices)  # one rank's share of the strong-scaled north star at W = 1, 2, 4, 8 (tools/strong_slices.py)
        timeout -k 10 300 python tools/strong_slices.py 20 > "$OUT/slices.jsonl" 2> "$OUT/slices.err"
        rc=$?; cat "$OUT/slices.jsonl"; tail -2 "$OUT/slices.err"; ok_or_fail $rc slices
        FA_PHASED_MIN_VECS=0 timeout -k 10 300 python tools/strong_slices.py 20 > "$OUT/slices_phased.jsonl" 2>> "$OUT/slices.err"
        rc=$?; cat "$OUT/slices_phased.jsonl"; ok_or_fail $rc slices_phased ;;
    rounds)  # one aggregator round on its own buckets, batched vs per part (tools/rounds.py) + kernel trace
        timeout -k 10 300 python tools/rounds.py 20 round_c2,round_c3,round_c4 > "$OUT/rounds.jsonl" 2> "$OUT/rounds.err"
        rc=$?; cat "$OUT/rounds.jsonl"; tail -2 "$OUT/rounds.err"; ok_or_fail $rc rounds
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rounds_prof" -o run -- \
            python3 tools/rounds.py 20 round_c2,round_c3 > "$OUT/rounds_prof.jsonl" 2> "$OUT/rounds_prof.err"
        rc=$?; tail -2 "$OUT/rounds_prof.err"; ok_or_fail $rc rounds_prof ;;
    e2e)
        timeout -k 10 900 python tools/e2e_bench.py 4 3 > "$OUT/e2e_bench.json" 2> "$OUT/e2e_bench.err"
        rc=$?; cat "$OUT/e2e_bench.json"; tail -3 "$OUT/e2e_bench.err"; ok_or_fail $rc e2e ;;
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
            timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary > "$OUT/bench3_$i.json" 2> "$OUT/bench3_$i.err"
            rc=$?; cat "$OUT/bench3_$i.json"; ok_or_fail $rc bench3_$i
        done ;;
    data)  # value dependence of the reduction time (tools/exp_data.py)
        timeout -k 10 300 python tools/exp_data.py 3 10 > "$OUT/exp_data.jsonl" 2> "$OUT/exp_data.err"
        rc=$?; cat "$OUT/exp_data.jsonl"; tail -2 "$OUT/exp_data.err"; ok_or_fail $rc data ;;
    layout)
        timeout -k 10 600 python tools/exp_layout.py > "$OUT/exp_layout.jsonl" 2> "$OUT/exp_layout.err"
        rc=$?; head -8 "$OUT/exp_layout.jsonl"; tail -3 "$OUT/exp_layout.err"; ok_or_fail $rc layout ;;
    alloc)
        timeout -k 10 600 python tools/exp_alloc.py > "$OUT/exp_alloc.jsonl" 2> "$OUT/exp_alloc.err"
        rc=$?; cat "$OUT/exp_alloc.jsonl"; tail -3 "$OUT/exp_alloc.err"; ok_or_fail $rc alloc ;;
    allocpmc)
        timeout -k 10 600 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum --kernel-trace \
            --output-format csv -d "$OUT/allocpmc1" -o run -- python3 tools/exp_alloc.py 25 3 > "$OUT/allocpmc1.jsonl" 2> "$OUT/allocpmc1.err"
        rc=$?; cat "$OUT/allocpmc1.jsonl"; ok_or_fail $rc allocpmc1
        timeout -k 10 600 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum --kernel-trace \
            --output-format csv -d "$OUT/allocpmc2" -o run -- python3 tools/exp_alloc.py 25 3 > "$OUT/allocpmc2.jsonl" 2> "$OUT/allocpmc2.err"
        rc=$?; cat "$OUT/allocpmc2.jsonl"; ok_or_fail $rc allocpmc2 ;;
    stride)
        timeout -k 10 600 python tools/exp_stride.py 25 > "$OUT/exp_stride.jsonl" 2> "$OUT/exp_stride.err"
        rc=$?; cat "$OUT/exp_stride.jsonl"; tail -2 "$OUT/exp_stride.err"; ok_or_fail $rc stride
        timeout -k 10 600 python tools/exp_stride.py 26 >> "$OUT/exp_stride.jsonl" 2>> "$OUT/exp_stride.err"
        rc=$?; tail -2 "$OUT/exp_stride.jsonl"; ok_or_fail $rc stride26 ;;
    map)
        timeout -k 10 600 python tools/exp_map.py 200 > "$OUT/exp_map.jsonl" 2> "$OUT/exp_map.err"
        rc=$?; cat "$OUT/exp_map.jsonl"; tail -2 "$OUT/exp_map.err"; ok_or_fail $rc map ;;
    counters)
        timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1
        rc=$?; grep -i -E "utcl|tlb|translat" "$OUT/counters.txt" | head -30; ok_or_fail $rc counters ;;
    *)
        echo "unknown step $s" ;;
    esac
done
echo "== done $(date +%T)" | tee -a "$OUT/session.log"
