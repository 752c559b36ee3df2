#!/bin/bash
# round-3 GPU session B: C2 small tiles -- brute force vs tree walk with teams
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/occupancy_probe.py C2 1,2,4,8,16 "brute_max=64;brute_max=0,walk_team=1;brute_max=0,walk_team=2;brute_max=0,walk_team=4;brute_max=0,walk_team=4,resume_min=16;brute_max=0,walk_team=4,resume_min=56" > gpurun_out/b_c2_team.log 2>&1 || { tail -20 gpurun_out/b_c2_team.log; exit 1; }
cat gpurun_out/b_c2_team.log
echo "session B done"
