#!/bin/bash
# round-3 GPU session A: team-walk parity, counter calibration probe, tile scaling (C2-C5, N=1/2/4/8),
# team-walk tiles (C3/C4).  Every GPU step under its own time limit; stop at the first failure.
set -uo pipefail
mkdir -p gpurun_out
(nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python3 -c "import os; print(len(os.sched_getaffinity(0)), os.cpu_count())"; env | grep -E "OMP|MAX_JOBS") > gpurun_out/host_cpu.txt 2>&1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "team_walk" > gpurun_out/a_team_tests.log 2>&1 || { echo "team tests failed"; tail -30 gpurun_out/a_team_tests.log; exit 1; }
tail -3 gpurun_out/a_team_tests.log
timeout -k 10 300 tools/hbm_probe.sh gpurun_out/hbm_probe -- tools/bin/hbm_probe || exit 1
for c in C2 C3 C4 C5; do
  timeout -k 10 240 python3 -u tools/occupancy_probe.py $c 1,2,4,8 "" > gpurun_out/tiles_$c.log 2>&1 || exit 1
  cat gpurun_out/tiles_$c.log
done
for c in C3 C4; do
  timeout -k 10 300 python3 -u tools/occupancy_probe.py $c 1,2,4,8 "walk_team=1;walk_team=2;walk_team=4" > gpurun_out/tiles_team_$c.log 2>&1 || exit 1
  cat gpurun_out/tiles_team_$c.log
done
echo "session A done"
