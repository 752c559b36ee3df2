#!/bin/bash
# round-3 GPU session I: resume threshold re-swept with the predicated steps (C5: 40 / 48 / 56; C3, C4: 28 / 36 / 44)
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_CFGS=C5 timeout -k 10 400 python3 -u tools/ab_walk.py base:0,base@resume_min=40:0,base@resume_min=56:0 > gpurun_out/i_c5.log 2>&1 || { tail -20 gpurun_out/i_c5.log; exit 1; }
grep '^{' gpurun_out/i_c5.log | cut -c1-110
AB_CFGS=C3,C4 timeout -k 10 300 python3 -u tools/ab_walk.py base:0,base@resume_min=28:0,base@resume_min=44:0,base:0 > gpurun_out/i_c34.log 2>&1 || { tail -20 gpurun_out/i_c34.log; exit 1; }
grep '^{' gpurun_out/i_c34.log | cut -c1-110
echo "session I done"
