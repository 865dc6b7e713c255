#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate runs, as the MI355X guide prescribes) of the dominant kernel
# of other bench workloads.  tools/pmc_workloads.sh <tag> workload...
set -u
OUT=gpurun_out/$1; shift; mkdir -p "$OUT"; export TMPDIR=/tmp
for w in "$@"; do
    for c in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$OUT/pmc_${w}_$c" -o run -- \
            python3 bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-live-pmc \
            > "$OUT/pmc_${w}_$c.json" 2> "$OUT/pmc_${w}_$c.err" || exit 1
    done
done
