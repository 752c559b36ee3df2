#!/bin/bash
# round-3 GPU session V: sun_cache on the 4-wide walk -- parity, C5 same-box A/B, C5 bench with counts
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "sun or wide or fixed_point" > gpurun_out/v_tests.log 2>&1 || { tail -30 gpurun_out/v_tests.log; exit 1; }
tail -1 gpurun_out/v_tests.log
timeout -k 10 400 python3 -u tools/occupancy_probe.py C5 1 "sun_cache=1;sun_cache=0" > gpurun_out/v_tiles_C5.log 2>&1 || { tail -5 gpurun_out/v_tiles_C5.log; exit 1; }
grep '^{' gpurun_out/v_tiles_C5.log
timeout -k 10 400 python3 -u bench.py --config C5 --steps 1 --warmup 1 --no-extra --no-cpu-baseline > gpurun_out/v_bench_C5.log 2>&1 || { tail -20 gpurun_out/v_bench_C5.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/v_bench_C5.log').read().strip().splitlines()[-1]); print('C5', d['value'], d['ms_per_step'], d['roofline'].get('counts_per_sample'))"
echo "session V done"
