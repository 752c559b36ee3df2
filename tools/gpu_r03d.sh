#!/bin/bash
# round-3 GPU session D: tile scaling of C3-C5 at N = 1, 2, 4, 8 with the 64-bit LDS stack entries, then
# the default bench.  Stop at the first failure.
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in C5 C3 C4; do
  timeout -k 10 400 python3 -u tools/occupancy_probe.py $c 1,2,4,8 "" > gpurun_out/d_tiles_$c.log 2>&1 || { tail -5 gpurun_out/d_tiles_$c.log; exit 1; }
  grep '^{' gpurun_out/d_tiles_$c.log | cut -c1-300
done
timeout -k 10 600 python3 -u bench.py > gpurun_out/d_bench.log 2>&1 || { tail -20 gpurun_out/d_bench.log; exit 1; }
tail -1 gpurun_out/d_bench.log | cut -c1-300
echo "session D done"
