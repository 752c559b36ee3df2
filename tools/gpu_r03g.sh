#!/bin/bash
# round-3 GPU session G: rocprofv3 kernel trace + PMC passes of C3, C4 and C5 with the final r03c build
# (64-bit LDS stack entries, select-form steps).  Stop at the first failure.
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
PASS_TIMEOUT=200 timeout -k 10 500 tools/run_profiles.sh gpurun_out/prof_C3g C3 || exit 1
PASS_TIMEOUT=200 timeout -k 10 500 tools/run_profiles.sh gpurun_out/prof_C4g C4 || exit 1
PASS_TIMEOUT=240 timeout -k 10 900 tools/run_profiles.sh gpurun_out/prof_C5g C5 --steps 1 --warmup 1 || exit 1
echo "session G done"
