#!/bin/bash
# A/B of the phased kernel's dynamic row pool (FA_PHASED_DYN): tools/many_clients.py's product launch per
# config, fresh alternating processes per variant.  Output: gpurun_out/<tag>/ab_dyn.jsonl.
#   tools/ab_dyn.sh <tag> <configs> <reps> variant...     (variant: a pool size, 0 = the static form)
set -u
TAG=$1; CFG=$2; REPS=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for rep in $(seq 1 "$REPS"); do
    for v in "$@"; do
        FA_PHASED_DYN=$v timeout -k 10 200 python tools/many_clients.py 12 "$CFG" 0 > "$OUT/ab_dyn_cur.jsonl" 2>> "$OUT/ab_dyn.err" || exit 1
        python -c "
import json,sys
for l in open('$OUT/ab_dyn_cur.jsonl'):
    d=json.loads(l); d['dyn']=$v; d['rep']=$rep; print(json.dumps(d))" >> "$OUT/ab_dyn.jsonl"
        tail -n +1 "$OUT/ab_dyn_cur.jsonl" | sed "s/^/dyn=$v /"
    done
done
