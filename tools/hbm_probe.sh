#!/bin/bash
# rocprofv3 passes of a program for the L2 memory-side byte counters (run on the GPU box from the
# repo root), one counter group per run (at most 4 TCC counters a pass):
#   tools/hbm_probe.sh OUTDIR -- PROGRAM [ARGS...]
# Summarise with tools/hbm_probe_summary.py OUTDIR.
set -euo pipefail
export TMPDIR=/tmp
OUT=$1
shift
[ "$1" = "--" ] && shift
mkdir -p "$OUT"
run() {
  local name=$1
  shift
  echo "pass $name"
  timeout -s KILL "${PASS_TIMEOUT:-120}" rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o "$name" -- \
    "${PROG[@]}" > "$OUT/$name.log" 2>&1
}
PROG=("$@")
run kt --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run req --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
run dram --pmc TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_32B_sum TCC_MISS_sum
run hit --pmc TCC_HIT_sum TCC_REQ_sum TCC_READ_sum TCC_EA0_WRREQ_64B_sum
echo "passes done: $OUT"
