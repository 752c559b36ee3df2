#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "auto_tile" > gpurun_out/r_tests.log 2>&1 || { tail -30 gpurun_out/r_tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r_tests.log | tail -5
