#!/bin/bash
# round-3 GPU session Q: C3 / C4 row tiles with and without the pilot order (N = 2, 4)
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in C3 C4; do
  timeout -k 10 400 python3 -u tools/occupancy_probe.py $c 2,4 "pilot=-1;pilot=0" > gpurun_out/q_pilot_$c.log 2>&1 || { tail -5 gpurun_out/q_pilot_$c.log; exit 1; }
  cat gpurun_out/q_pilot_$c.log
done
echo "session Q done"
