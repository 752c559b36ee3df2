#!/bin/bash
# round-3 GPU session FIN: tile scaling of C2-C5 at N = 1, 2, 4, 8 with the final r03 build, then the bench
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in C2 C3 C4 C5; do
  timeout -k 10 400 python3 -u tools/occupancy_probe.py $c 1,2,4,8 "" > gpurun_out/fin_tiles_$c.log 2>&1 || { tail -5 gpurun_out/fin_tiles_$c.log; exit 1; }
  grep '^{' gpurun_out/fin_tiles_$c.log
done
timeout -k 10 600 python3 -u bench.py > gpurun_out/fin_bench.log 2>&1 || { tail -20 gpurun_out/fin_bench.log; exit 1; }
tail -1 gpurun_out/fin_bench.log | cut -c1-600
echo "session FIN done"
