#!/bin/bash
# round-3 GPU session Z: the spill-free 4-wave build of the 4-wide walk profiled on C5 (useful bytes)
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ENSEM3A_RT_LIB=$PWD/ensem3a_openclraytracer_amd/lib/variants/libw4.so PASS_TIMEOUT=240 \
  tools/run_profiles.sh gpurun_out/prof_C5w4 C5 --steps 1 --warmup 0 --no-counts --option stack_lds=20 || exit 1
echo "session Z done"
