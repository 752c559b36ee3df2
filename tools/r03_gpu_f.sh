#!/bin/bash
# round-3 GPU session F: RCCL one-rank test, deferred-leaf variants (RT_LEAF_DEFER = 16 / 32 / 48 lanes)
# vs base on C3 / C4
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_boundary.py -x -q --timeout 280 --timeout-method thread -k rccl > gpurun_out/f_rccl.log 2>&1 || { tail -30 gpurun_out/f_rccl.log; exit 1; }
tail -1 gpurun_out/f_rccl.log
VAR_CONFIGS=C3,C4 timeout -k 10 900 python3 -u tools/variants.py run base d16 d32 d48 base > gpurun_out/f_defer.log 2>&1 || { tail -20 gpurun_out/f_defer.log; exit 1; }
cat gpurun_out/f_defer.log
echo "session F done"
