#!/bin/bash
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/calib}
mkdir -p "$OUT"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU --output-format csv -d "$OUT/a" -o a -- python3 tools/calib_valu.py > "$OUT/a.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d "$OUT/b" -o b -- python3 tools/calib_valu.py > "$OUT/b.log" 2>&1
