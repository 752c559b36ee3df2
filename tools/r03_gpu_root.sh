#!/bin/bash
# round-3 GPU session ROOT: the root node tested at ray start from scalar loads (RT_ROOT_STEP) -- full GPU
# suite, then A/B against the build without it (noroot) and with it on the 4-wide walk too (rootw)
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/root_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/root_tests.log; exit 1; }
tail -1 gpurun_out/root_tests.log
ENSEM3A_RT_LIB=$PWD/ensem3a_openclraytracer_amd/lib/variants/libroot2.so timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "fast or fixed_point or pilot or sun or team or wide" > gpurun_out/root2_tests.log 2>&1 || { echo "root2 tests failed"; tail -30 gpurun_out/root2_tests.log; exit 1; }
tail -1 gpurun_out/root2_tests.log
for v in root noroot rootw root2; do
  if [ $v = root ]; then unset ENSEM3A_RT_LIB; else export ENSEM3A_RT_LIB=$PWD/ensem3a_openclraytracer_amd/lib/variants/lib$v.so; fi
  for c in C3 C4; do
    timeout -k 10 300 python3 -u tools/occupancy_probe.py $c 1,8 "" > gpurun_out/root_${v}_$c.log 2>&1 || { tail -5 gpurun_out/root_${v}_$c.log; exit 1; }
    echo "$v $(grep '^{' gpurun_out/root_${v}_$c.log | tr '\n' ' ')"
  done
  if [ $v != noroot ] || true; then
    timeout -k 10 300 python3 -u tools/occupancy_probe.py C5 1 "" > gpurun_out/root_${v}_C5.log 2>&1 || { tail -5 gpurun_out/root_${v}_C5.log; exit 1; }
    echo "$v $(grep '^{' gpurun_out/root_${v}_C5.log)"
  fi
done
echo "session ROOT done"
