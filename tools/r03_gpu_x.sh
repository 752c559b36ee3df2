#!/bin/bash
# round-3 GPU session X: resume threshold re-check after the prefix / shadow-ray caches (C3, C4, C5 at N=1)
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in C3 C4; do
  timeout -k 10 300 python3 -u tools/occupancy_probe.py $c 1 ";resume_min=28;resume_min=44;resume_min=52" > gpurun_out/x_$c.log 2>&1 || { tail -5 gpurun_out/x_$c.log; exit 1; }
  grep '^{' gpurun_out/x_$c.log
done
timeout -k 10 300 python3 -u tools/occupancy_probe.py C5 1 ";resume_min=40;resume_min=56" > gpurun_out/x_C5.log 2>&1 || { tail -5 gpurun_out/x_C5.log; exit 1; }
grep '^{' gpurun_out/x_C5.log
echo "session X done"
