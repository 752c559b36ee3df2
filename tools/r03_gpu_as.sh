#!/bin/bash
# round-3 GPU session AS: wave assist (finished lanes walk other lanes' subtrees) -- parity, then C3 / C4 A/B
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "assist" > gpurun_out/as_tests.log 2>&1 || { tail -30 gpurun_out/as_tests.log; exit 1; }
tail -1 gpurun_out/as_tests.log
for c in C3 C4; do
  timeout -k 10 400 python3 -u tools/occupancy_probe.py $c 1,2,8 "assist=0;assist=1" > gpurun_out/as_$c.log 2>&1 || { tail -5 gpurun_out/as_$c.log; exit 1; }
  grep '^{' gpurun_out/as_$c.log
done
echo "session AS done"
