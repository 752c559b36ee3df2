#!/bin/bash
# round-3 GPU session N: final validation -- GPU test suite, smoke, default bench
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/n_tests.log 2>&1 || { tail -30 gpurun_out/n_tests.log; exit 1; }
tail -1 gpurun_out/n_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/n_smoke.log 2>&1 || { tail -20 gpurun_out/n_smoke.log; exit 1; }
tail -2 gpurun_out/n_smoke.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/n_bench.log 2>&1 || { tail -20 gpurun_out/n_bench.log; exit 1; }
tail -1 gpurun_out/n_bench.log | cut -c1-600
echo "session N done"
