#!/bin/bash
# round-3 GPU session I: resume threshold with teams on small tiles (C3 / C4, N = 4, 8)
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in C3 C4; do
  timeout -k 10 400 python3 -u tools/occupancy_probe.py $c 4,8 "resume_min=-1;resume_min=16;resume_min=24;resume_min=48;resume_min=56" > gpurun_out/i_resume_$c.log 2>&1 || exit 1
  cat gpurun_out/i_resume_$c.log
done
echo "session I done"
