#!/bin/bash
# Experiment knobs of one build, A/B'd in fresh alternating processes: each variant is an environment
# assignment (or "base").  Output: gpurun_out/<tag>/ab_env.jsonl.
#   tools/ab_env.sh <tag> "<workloads>" variant...
set -u
TAG=$1; W=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for w in $W; do
    for rep in 1 2; do
        for v in "$@"; do
            if [ "$v" = base ]; then
                r=$(timeout -k 10 120 python tools/ab_lib.py multihop-federeated-split-learning_amd $w 40 2>> "$OUT/ab_env.err") || exit 1
            else
                r=$(env $v timeout -k 10 120 python tools/ab_lib.py multihop-federeated-split-learning_amd $w 40 2>> "$OUT/ab_env.err") || exit 1
            fi
            echo "{\"variant\": \"$v\", \"r\": $r}" >> "$OUT/ab_env.jsonl"
        done
    done
done
