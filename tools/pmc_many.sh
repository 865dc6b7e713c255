#!/bin/bash
# PMC passes of tools/many_clients.py per config (GPU box): read latency / DRAM credits, translation, writes.
#   tools/pmc_many.sh <tag> [configs...]      -> gpurun_out/<tag>/pmc_<config>_<pass>/
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PASSES=(
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE"
  "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_PENDING_STALL_CYCLES_sum"
  "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum"
)
for cfg in "$@"; do
  for i in 0 1 2; do
    timeout -s KILL 120 rocprofv3 --pmc ${PASSES[$i]} --kernel-trace --output-format csv -d "$OUT/pmc_${cfg}_$i" -o run -- \
      python3 tools/many_clients.py 4 "$cfg" 0 > "$OUT/pmc_${cfg}_$i.log" 2>&1
    rc=$?
    echo "$cfg pass $i rc $rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
