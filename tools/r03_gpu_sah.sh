#!/bin/bash
# round-3 GPU session SAH: a finer SAH build (exact sweep up to 4096 leaves, 256 bins above) vs the default
# (exact sweep up to 64, 32 bins): node visits and frame times of C3 / C4 / C5
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in base sah; do
  if [ $v = sah ]; then export ENSEM3A_RT_LIB=$PWD/ensem3a_openclraytracer_amd/lib/variants/libsah.so; else unset ENSEM3A_RT_LIB; fi
  timeout -k 10 500 python3 -u tools/wave_stats.py C3,C4 "" > gpurun_out/sah_ws_$v.log 2>&1 || { tail -5 gpurun_out/sah_ws_$v.log; exit 1; }
  echo "$v"; grep '^{' gpurun_out/sah_ws_$v.log | cut -c1-200
  for c in C3 C4 C5; do
    timeout -k 10 300 python3 -u tools/occupancy_probe.py $c 1 "" > gpurun_out/sah_t_${v}_$c.log 2>&1 || { tail -5 gpurun_out/sah_t_${v}_$c.log; exit 1; }
    echo "$v $(grep '^{' gpurun_out/sah_t_${v}_$c.log)"
  done
done
echo "session SAH done"
