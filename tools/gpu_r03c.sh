#!/bin/bash
# round-3 GPU session C (after the 64-bit LDS stack entries): the whole -m gpu suite, then C5 profiles of
# the default build and of the spill-free 4-wave build (useful bytes).  Stop at the first failure.
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/c_tests.log 2>&1 || { tail -40 gpurun_out/c_tests.log; exit 1; }
tail -2 gpurun_out/c_tests.log
PASS_TIMEOUT=240 timeout -k 10 900 tools/run_profiles.sh gpurun_out/prof_C5c C5 --steps 1 --warmup 1 || exit 1
ENSEM3A_RT_LIB=$PWD/ensem3a_openclraytracer_amd/lib/variants/libw4.so PASS_TIMEOUT=240 \
  timeout -k 10 900 tools/run_profiles.sh gpurun_out/prof_C5w4c C5 --steps 1 --warmup 0 --no-counts --option stack_lds=20 || exit 1
echo "session C done"
