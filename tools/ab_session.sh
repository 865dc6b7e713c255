#!/bin/bash
# A/B of the package build in ab_old/ (A) against the in-tree build (B): fresh processes, alternated,
# per workload.  Output: gpurun_out/<tag>/ab.jsonl.   tools/ab_session.sh <tag> [workloads...]
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for w in ${*:-northstar c2 c3 c4 c5r}; do
    for rep in 1 2; do
        for pkg in ab_old multihop-federeated-split-learning_amd; do
            timeout -k 10 120 python tools/ab_lib.py $pkg $w 40 >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || exit 1
        done
    done
done
