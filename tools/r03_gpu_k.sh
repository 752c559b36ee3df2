#!/bin/bash
# round-3 GPU session K: small-tile pilot auto (tests + tile scaling C3 / C4)
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "team or pilot or full_size" > gpurun_out/k_tests.log 2>&1 || { tail -30 gpurun_out/k_tests.log; exit 1; }
tail -1 gpurun_out/k_tests.log
for c in C3 C4; do
  timeout -k 10 300 python3 -u tools/occupancy_probe.py $c 1,2,4,8 "" > gpurun_out/k_tiles_$c.log 2>&1 || exit 1
  cat gpurun_out/k_tiles_$c.log
done
echo "session K done"
