#!/bin/bash
# round-3 GPU session B: team-walk tests (2/4/8 lanes) and full-size FAST-vs-REF pixel counts,
# C2 small tiles (brute force vs team tree walk), C3/C4 tiles with 4/8-lane teams, probe re-run
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 300 --timeout-method thread -k "team_walk or full_size_fast" > gpurun_out/b_tests.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error|assert|config" gpurun_out/b_tests.log | tail -30; exit 1; }
grep -E '^\{"config"|passed|failed' gpurun_out/b_tests.log
timeout -k 10 300 python3 -u tools/occupancy_probe.py C2 1,2,4,8,16 "brute_max=64;brute_max=0,walk_team=1;brute_max=0,walk_team=4;brute_max=0,walk_team=8" > gpurun_out/b_c2_team.log 2>&1 || { tail -20 gpurun_out/b_c2_team.log; exit 1; }
cat gpurun_out/b_c2_team.log
for c in C3 C4; do
  timeout -k 10 300 python3 -u tools/occupancy_probe.py $c 2,4,8 "walk_team=4;walk_team=8" > gpurun_out/b_team8_$c.log 2>&1 || exit 1
  cat gpurun_out/b_team8_$c.log
done
timeout -k 10 300 tools/hbm_probe.sh gpurun_out/hbm_probe2 -- tools/bin/hbm_probe || exit 1
echo "session B done"
