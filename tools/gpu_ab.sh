#!/bin/bash
# A/B of variant libraries (tools/variants.py build ...) on the tree-walk configs: bit-identity at 4 spp
# against the default library, then timing.   tools/gpu_ab.sh CFGS NAME:block[,NAME:block...]
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_CFGS=$1 timeout -k 10 900 python3 -u tools/ab_walk.py $2 > gpurun_out/ab_$3.log 2>&1 || { tail -20 gpurun_out/ab_$3.log; exit 1; }
grep '^{' gpurun_out/ab_$3.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['variant'], d['cfg'], d['Msamples/s'], d['ms'], d['identical_4spp'])"
