#!/bin/bash
# round-3 GPU session Y2: C4 / C5 profiles with the prefix and shadow-ray caches
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
PASS_TIMEOUT=200 tools/run_profiles.sh gpurun_out/prof_C4 C4 --steps 3 --warmup 1 --no-counts || exit 1
PASS_TIMEOUT=240 tools/run_profiles.sh gpurun_out/prof_C5 C5 --steps 1 --warmup 0 --no-counts || exit 1
echo "session Y2 done"
