#!/bin/bash
# SQ counter passes on tile renders (tools/tile_loop.py N REPS OPTS), one group per run
set -euo pipefail
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU --output-format csv -d "$OUT/a" -o a -- python3 tools/tile_loop.py "$@" > "$OUT/a.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD --output-format csv -d "$OUT/b" -o b -- python3 tools/tile_loop.py "$@" > "$OUT/b.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_SMEM_NORM SQ_ACTIVE_INST_EXP SQ_INSTS_VMEM_WR --output-format csv -d "$OUT/c" -o c -- python3 tools/tile_loop.py "$@" > "$OUT/c.log" 2>&1
echo diag done
