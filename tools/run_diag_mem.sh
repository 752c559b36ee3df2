#!/bin/bash
# Memory-pipeline PMC passes on the render kernel (TA / TCP stalls, L1 traffic); one group per run.
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/diagmem}
ARGS=${BENCH_ARGS:-"--steps 1 --warmup 1 --no-cpu-baseline"}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum --output-format csv -d "$OUT/d" -o d -- python3 bench.py $ARGS > "$OUT/d.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum --output-format csv -d "$OUT/e" -o e -- python3 bench.py $ARGS > "$OUT/e.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VMEM_RD --output-format csv -d "$OUT/c" -o c -- python3 bench.py $ARGS > "$OUT/c.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD --output-format csv -d "$OUT/a" -o a -- python3 bench.py $ARGS > "$OUT/a.log" 2>&1
echo diagmem done
