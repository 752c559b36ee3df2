#!/bin/bash
# round-3 GPU session U: sun_cache option -- parity, then same-box A/B on C2 / C3 / C4 frames and tiles
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "sun or fixed_point or team or pilot or auto_tile" > gpurun_out/u_tests.log 2>&1 || { tail -30 gpurun_out/u_tests.log; exit 1; }
tail -1 gpurun_out/u_tests.log
for c in C2 C3 C4; do
  timeout -k 10 300 python3 -u tools/occupancy_probe.py $c 1,8 "sun_cache=1;sun_cache=0;sun_cache=1;sun_cache=0" > gpurun_out/u_tiles_$c.log 2>&1 || exit 1
  grep '^{' gpurun_out/u_tiles_$c.log
done
echo "session U done"
