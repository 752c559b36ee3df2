#!/bin/bash
# round-3 GPU session J: two-pass pilot ordering on 1/8 tiles with teams (C3 / C4)
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/occupancy_probe.py C4 8 "pilot=-1;pilot=64;pilot=32;pilot=128" > gpurun_out/j_pilot_C4.log 2>&1 || exit 1
cat gpurun_out/j_pilot_C4.log
timeout -k 10 300 python3 -u tools/occupancy_probe.py C3 8 "pilot=-1;pilot=32;pilot=16;pilot=64" > gpurun_out/j_pilot_C3.log 2>&1 || exit 1
cat gpurun_out/j_pilot_C3.log
echo "session J done"
