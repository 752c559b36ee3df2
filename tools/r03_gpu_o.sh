#!/bin/bash
# round-3 GPU session O: 4-wide node with a partial child sort (RT_WIDE_PARTIAL_SORT) vs base on C5
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ENSEM3A_RT_LIB=$PWD/ensem3a_openclraytracer_amd/lib/variants/libps.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 280 --timeout-method thread -k "wide_layout or shadow_rays_end" > gpurun_out/o_tests.log 2>&1 || { tail -30 gpurun_out/o_tests.log; exit 1; }
tail -1 gpurun_out/o_tests.log
for v in base ps base ps; do
  ENSEM3A_RT_LIB=$PWD/ensem3a_openclraytracer_amd/lib/variants/lib$v.so timeout -k 10 300 python3 -u bench.py --config C5 --steps 1 --warmup 1 --no-extra --no-cpu-baseline --no-counts > gpurun_out/o_bench_$v.log 2>&1 || { tail -20 gpurun_out/o_bench_$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/o_bench_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
echo "session O done"
