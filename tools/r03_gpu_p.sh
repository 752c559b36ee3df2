#!/bin/bash
# round-3 GPU session P: C5 row tiles with and without the two-pass pilot order
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 -u tools/occupancy_probe.py C5 2,4,8 "pilot=-1;pilot=0" > gpurun_out/p_c5_pilot.log 2>&1 || { tail -5 gpurun_out/p_c5_pilot.log; exit 1; }
cat gpurun_out/p_c5_pilot.log
echo "session P done"
