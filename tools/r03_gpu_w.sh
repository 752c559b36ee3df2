#!/bin/bash
# round-3 GPU session W: C5 after the shadow-ray cache -- waves per SIMD of the 4-wide walk (6 / 7 / 8) and the pilot
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/occupancy_probe.py C5 1 ";pilot=128" > gpurun_out/w_base.log 2>&1 || { tail -5 gpurun_out/w_base.log; exit 1; }
grep '^{' gpurun_out/w_base.log
for v in w6 w8; do
  ENSEM3A_RT_LIB=ensem3a_openclraytracer_amd/lib/variants/lib$v.so timeout -k 10 300 python3 -u tools/occupancy_probe.py C5 1 "" > gpurun_out/w_$v.log 2>&1 || { tail -5 gpurun_out/w_$v.log; exit 1; }
  echo "$v $(grep '^{' gpurun_out/w_$v.log)"
done
echo "session W done"
