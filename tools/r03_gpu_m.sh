#!/bin/bash
# round-3 GPU session M: C5 with the pixel sum kept in the output buffer (RT_WIDE_LEAN) vs base:
# parity on the wide layout (small cases vs the oracle), then the C5 frame
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in base lean; do
  ENSEM3A_RT_LIB=$PWD/ensem3a_openclraytracer_amd/lib/variants/lib$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 280 --timeout-method thread -k "wide_layout or two_pass_pilot_renders or full_size_fast_vs_ref_pixel_counts and C5" > gpurun_out/m_tests_$v.log 2>&1 || { tail -30 gpurun_out/m_tests_$v.log; exit 1; }
  tail -1 gpurun_out/m_tests_$v.log
done
for v in base lean base lean; do
  ENSEM3A_RT_LIB=$PWD/ensem3a_openclraytracer_amd/lib/variants/lib$v.so timeout -k 10 300 python3 -u bench.py --config C5 --steps 1 --warmup 1 --no-extra --no-cpu-baseline --no-counts > gpurun_out/m_bench_$v.log 2>&1 || { tail -20 gpurun_out/m_bench_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/m_bench_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
echo "session M done"
