#!/bin/bash
# round-3 GPU session E: the select-form item step (RT_FLAT_STEP) -- the whole -m gpu suite, then C3/C4
# row tiles at N = 1, 4, 8 with it and without it (variant flat0).  Stop at the first failure.
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e_tests.log 2>&1 || { tail -40 gpurun_out/e_tests.log; exit 1; }
tail -2 gpurun_out/e_tests.log
for c in C3 C4; do
  timeout -k 10 400 python3 -u tools/occupancy_probe.py $c 1,4,8 "" > gpurun_out/e_tiles_$c.log 2>&1 || { tail -5 gpurun_out/e_tiles_$c.log; exit 1; }
  grep '^{' gpurun_out/e_tiles_$c.log | cut -c1-200
  ENSEM3A_RT_LIB=$PWD/ensem3a_openclraytracer_amd/lib/variants/libflat0.so timeout -k 10 400 python3 -u tools/occupancy_probe.py $c 1,4,8 "" > gpurun_out/e_tiles0_$c.log 2>&1 || { tail -5 gpurun_out/e_tiles0_$c.log; exit 1; }
  grep '^{' gpurun_out/e_tiles0_$c.log | sed 's/^/flat0 /' | cut -c1-200
done
echo "session E done"
