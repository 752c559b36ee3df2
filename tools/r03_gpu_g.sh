#!/bin/bash
# round-3 GPU session G: SQ / TA counters of the deferred-leaf variant vs base on C3 (lanes active per
# VALU instruction, TA busy), the counts of the same launches in the bench lines
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in base d16; do
  mkdir -p gpurun_out/g_$v
  ENSEM3A_RT_LIB=$PWD/ensem3a_openclraytracer_amd/lib/variants/lib$v.so timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD TA_TA_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/g_$v/sq -o sq -- python3 bench.py --config C3 --steps 2 --warmup 1 --no-extra --no-cpu-baseline > gpurun_out/g_$v/bench.log 2>&1 || { tail -20 gpurun_out/g_$v/bench.log; exit 1; }
  tail -1 gpurun_out/g_$v/bench.log | cut -c1-200
done
echo "session G done"
