#!/bin/bash
# round-3 GPU session F (select-form steps): the whole -m gpu suite, tile scaling of C3-C5 at N = 1, 2, 4, 8,
# then the default bench.  Stop at the first failure.
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/f_tests.log 2>&1 || { tail -40 gpurun_out/f_tests.log; exit 1; }
tail -2 gpurun_out/f_tests.log
for c in C5 C3 C4; do
  timeout -k 10 400 python3 -u tools/occupancy_probe.py $c 1,2,4,8 "" > gpurun_out/f_tiles_$c.log 2>&1 || { tail -5 gpurun_out/f_tiles_$c.log; exit 1; }
  grep '^{' gpurun_out/f_tiles_$c.log | cut -c1-200
done
timeout -k 10 600 python3 -u bench.py > gpurun_out/f_bench.log 2>&1 || { tail -20 gpurun_out/f_bench.log; exit 1; }
tail -1 gpurun_out/f_bench.log | cut -c1-200
echo "session F done"
