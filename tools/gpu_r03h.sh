#!/bin/bash
# round-3 GPU session H: A/B of the two-entry pop (variant pop2) on C3/C4, then rocprofv3 passes of C3, C4
# and C5 with the final r03c build.  Stop at the first failure.
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_CFGS=C3,C4 timeout -k 10 400 python3 -u tools/ab_walk.py base:0,pop2:0,base:0,pop2:0 > gpurun_out/ab_r03h.log 2>&1 || { tail -20 gpurun_out/ab_r03h.log; exit 1; }
grep '^{' gpurun_out/ab_r03h.log | cut -c1-120
PASS_TIMEOUT=200 timeout -k 10 500 tools/run_profiles.sh gpurun_out/prof_C3g C3 || exit 1
PASS_TIMEOUT=200 timeout -k 10 500 tools/run_profiles.sh gpurun_out/prof_C4g C4 || exit 1
PASS_TIMEOUT=240 timeout -k 10 900 tools/run_profiles.sh gpurun_out/prof_C5g C5 --steps 1 --warmup 1 || exit 1
echo "session H done"
