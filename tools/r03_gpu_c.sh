#!/bin/bash
# round-3 GPU session C: the GPU test suite, tile scaling with the auto team rule, rocprofv3 passes
# (kernel trace + calibrated memory-side bytes + SQ) of C2-C5, and the C5 spill A/B: the 4-wave build
# (no scratch, 20 LDS stack entries) vs the default 7-wave one
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/c_tests.log; exit 1; }
tail -2 gpurun_out/c_tests.log
for c in C3 C4; do
  timeout -k 10 300 python3 -u tools/occupancy_probe.py $c 1,2,4,8 "" > gpurun_out/c_tiles_$c.log 2>&1 || exit 1
  cat gpurun_out/c_tiles_$c.log
done
for c in C2 C3 C4; do
  PASS_TIMEOUT=200 tools/run_profiles.sh gpurun_out/prof_$c $c --steps 3 --warmup 1 --no-counts || exit 1
done
PASS_TIMEOUT=240 tools/run_profiles.sh gpurun_out/prof_C5 C5 --steps 1 --warmup 0 --no-counts || exit 1
ENSEM3A_RT_LIB=$PWD/ensem3a_openclraytracer_amd/lib/variants/libw4.so PASS_TIMEOUT=240 \
  tools/run_profiles.sh gpurun_out/prof_C5w4 C5 --steps 1 --warmup 0 --no-counts --option stack_lds=20 || exit 1
echo "session C done"
