#!/bin/bash
# per variant library: tile times (N = 1, 8, 128) with auto and single-lane teams; VP_N / VP_SETS override
N=${VP_N:-1,8,128}
SETS=${VP_SETS:-"team=0;team=1"}
CFG=${VP_CFG:-C2}
for v in "$@"; do
  if [ "$v" = base ]; then lib=ensem3a_openclraytracer_amd/lib/libensem3a_rt.so; else lib=ensem3a_openclraytracer_amd/lib/variants/lib$v.so; fi
  echo "== $v"
  ENSEM3A_RT_LIB=$lib timeout -k 10 300 python tools/occupancy_probe.py $CFG $N "$SETS" || exit 1
done
