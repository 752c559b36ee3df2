#!/bin/bash
# round-3 GPU session Y1: the full GPU suite, then C2 / C3 profiles with the prefix and shadow-ray caches
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/y1_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/y1_tests.log; exit 1; }
tail -1 gpurun_out/y1_tests.log
PASS_TIMEOUT=200 tools/run_profiles.sh gpurun_out/prof_C2 C2 --steps 10 --warmup 2 --no-counts || exit 1
PASS_TIMEOUT=200 tools/run_profiles.sh gpurun_out/prof_C3 C3 --steps 3 --warmup 1 --no-counts || exit 1
echo "session Y1 done"
