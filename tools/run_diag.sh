#!/bin/bash
# Diagnostic PMC passes on the render kernel (one counter group per run).
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/diag}
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu-baseline"}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU --output-format csv -d "$OUT/a" -o a -- python3 bench.py $ARGS > "$OUT/a.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD --output-format csv -d "$OUT/b" -o b -- python3 bench.py $ARGS > "$OUT/b.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d "$OUT/c" -o c -- python3 bench.py $ARGS > "$OUT/c.log" 2>&1
echo diag done
