#!/bin/bash
# round-3 GPU session H: separate C5's register-spill bytes from its stack-overflow bytes: the
# spill-free 4-wave build with the default build's 11 LDS stack levels (deeper entries in HBM)
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ENSEM3A_RT_LIB=$PWD/ensem3a_openclraytracer_amd/lib/variants/libw4.so PASS_TIMEOUT=240 \
  tools/run_profiles.sh gpurun_out/prof_C5w4s11 C5 --steps 1 --warmup 0 --no-counts --option stack_lds=11 || exit 1
echo "session H done"
