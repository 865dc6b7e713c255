#!/bin/bash
# BASELINE C1 through fa_aggregator under rocprofv3 (kernel, marker and HIP runtime traces): where the
# aggregator's ~0.35 ms of work per LeNet-5 round goes.  The fake owners drive 40 rounds over loopback.
#   tools/c1_trace.sh <tag> [fedavg|literal]
set -u
TAG=${1:-c1}
MODE=${2:-literal}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BASE=$(( (RANDOM % 200) * 100 + 10000 ))
timeout -k 10 180 rocprofv3 --kernel-trace --marker-trace --hip-runtime-trace --stats --output-format csv \
    -d "$OUT/c1trace" -o agg -- multihop-federeated-split-learning_amd/bin/fa_aggregator -i -1 -d 2 -c 1 \
    --mode "$MODE" --rounds 40 --port-base "$BASE" > "$OUT/c1_agg.jsonl" 2> "$OUT/c1_agg.err" &
AGG=$!
sleep 4
timeout -k 10 120 tests/tools/bin/fa_fake_owners --blobs tests/golden/lenet5_c1 --parts 1,2,3 -d 2 -c 1 \
    --rounds 40 --port-base "$BASE" --model-name 2 --start 6 --end 1 --mode "$MODE" --reply-timeout 30 \
    > "$OUT/c1_owners.json" 2> "$OUT/c1_owners.err"
rc=$?
wait $AGG
arc=$?
tail -c 600 "$OUT/c1_owners.json"
echo "owners rc=$rc aggregator rc=$arc"
