#!/bin/bash
# round-3 GPU session L: C2 1/8 and 1/4 tiles -- brute-force teams with and without the pilot order
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/occupancy_probe.py C2 4,8 "team=1;team=2;team=4;team=8;team=4,pilot=8;team=4,pilot=4;team=2,pilot=8;team=1,pilot=8;team=4,pilot=8,pilot_chunk=1" > gpurun_out/l_c2.log 2>&1 || exit 1
cat gpurun_out/l_c2.log
echo "session L done"
