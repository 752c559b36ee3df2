#!/bin/bash
# Round-end style check on one MI355X: the whole -m gpu suite, smoke(), then the default bench.
# Every GPU step under its own time limit; stop at the first failure.
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/verify_tests.log 2>&1 || { tail -40 gpurun_out/verify_tests.log; exit 1; }
tail -3 gpurun_out/verify_tests.log
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/verify_smoke.log 2>&1 || { tail -20 gpurun_out/verify_smoke.log; exit 1; }
tail -2 gpurun_out/verify_smoke.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/verify_bench.log 2>&1 || { tail -20 gpurun_out/verify_bench.log; exit 1; }
tail -1 gpurun_out/verify_bench.log | cut -c1-400
echo "verify done"
