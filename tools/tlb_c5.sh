#!/bin/bash
# UTCL1 translation hits/misses of the phased kernel: C5 on one GPU (129 GiB resident) vs C5r (16 GiB).
# One --pmc pass per workload (2 TCP counters); output under gpurun_out/<tag>/.
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; export TMPDIR=/tmp
for w in c5r c5; do
    timeout -k 10 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum --kernel-trace \
        --output-format csv -d "$OUT/tlb_$w" -o run -- python3 bench.py --workload $w --steps 5 --warmup 2 \
        --no-cpu-baseline --no-secondary > "$OUT/tlb_$w.json" 2> "$OUT/tlb_$w.err" || exit 1
done
