#!/bin/bash
# rocprofv3 passes of bench.py for one workload (run on the GPU box from the repo root):
#   tools/run_profiles.sh OUTDIR CONFIG [extra bench.py args]
# One kernel-trace + stats run, then each PMC counter group in its own run (no sys/runtime trace,
# at most 8 SQ / 4 TCC / 2 GRBM counters per pass).  Summarise with tools/summarize_profiles.py.
set -euo pipefail
export TMPDIR=/tmp
OUT=$1
CFG=$2
shift 2
ARGS="--config $CFG --no-cpu-baseline --no-extra $*"
mkdir -p "$OUT"
run() {
  local name=$1
  shift
  echo "pass $name"
  timeout -s KILL "${PASS_TIMEOUT:-300}" rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o "$name" -- \
    python3 bench.py $ARGS > "$OUT/$name.log" 2>&1
}
run kt --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run dram --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum TCC_EA0_WRREQ_64B_sum
run req --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
run sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT
echo "profiles of $CFG done"
