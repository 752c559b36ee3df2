#!/bin/bash
# round-3 GPU session WS: wave-level loop statistics (traversal vs shading cycles, SIMD efficiency) of C3 / C4 / C5
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/wave_stats.py C3,C4,C5 "" > gpurun_out/ws.log 2>&1 || { tail -5 gpurun_out/ws.log; exit 1; }
grep '^{' gpurun_out/ws.log
echo "session WS done"
