#!/bin/bash
# round-3 GPU session D: team-gated pass-2 launches (tests + tiles), C3/C4 profiles, the full bench
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "team or pilot or full_size_fast or full_size_rows" > gpurun_out/d_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/d_tests.log; exit 1; }
tail -1 gpurun_out/d_tests.log
for c in C3 C4; do
  timeout -k 10 300 python3 -u tools/occupancy_probe.py $c 1,2,4,8 "" > gpurun_out/d_tiles_$c.log 2>&1 || exit 1
  cat gpurun_out/d_tiles_$c.log
done
for c in C3 C4; do
  PASS_TIMEOUT=200 tools/run_profiles.sh gpurun_out/prof_$c $c --steps 3 --warmup 1 --no-counts || exit 1
done
timeout -k 10 600 python3 -u bench.py > gpurun_out/d_bench.log 2>&1 || { tail -20 gpurun_out/d_bench.log; exit 1; }
tail -1 gpurun_out/d_bench.log
echo "session D done"
