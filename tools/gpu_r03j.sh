#!/bin/bash
# round-3 GPU session J: C5 item steps vs descend-until-leaf rounds (option step=2) with the predicated
# step; C3/C4 row tiles at N = 4, 8 with the team step predicated (default) and branchy (variant ft0)
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_CFGS=C5 timeout -k 10 300 python3 -u tools/ab_walk.py base:0,base@step=2:0 > gpurun_out/j_c5.log 2>&1 || { tail -20 gpurun_out/j_c5.log; exit 1; }
grep '^{' gpurun_out/j_c5.log | cut -c1-110
for c in C3 C4; do
  timeout -k 10 300 python3 -u tools/occupancy_probe.py $c 4,8 "" > gpurun_out/j_tiles_$c.log 2>&1 || { tail -5 gpurun_out/j_tiles_$c.log; exit 1; }
  grep '^{' gpurun_out/j_tiles_$c.log | cut -c1-200
  ENSEM3A_RT_LIB=$PWD/ensem3a_openclraytracer_amd/lib/variants/libft0.so timeout -k 10 300 python3 -u tools/occupancy_probe.py $c 4,8 "" > gpurun_out/j_tiles0_$c.log 2>&1 || { tail -5 gpurun_out/j_tiles0_$c.log; exit 1; }
  grep '^{' gpurun_out/j_tiles0_$c.log | sed 's/^/ft0 /' | cut -c1-200
  timeout -k 10 300 python3 -u tools/occupancy_probe.py $c 4,8 "" > gpurun_out/j_tiles2_$c.log 2>&1 || { tail -5 gpurun_out/j_tiles2_$c.log; exit 1; }
  grep '^{' gpurun_out/j_tiles2_$c.log | cut -c1-200
done
echo "session J done"
