#!/bin/bash
# round-3 GPU session T: first-bounce shadow-ray cache -- parity, then C3 / C4 frames and tiles
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "sun or fixed_point or team or pilot or full_size or auto_tile or fast_traversal_matches or work_counters or edge_cases or stack" > gpurun_out/t_tests.log 2>&1 || { tail -30 gpurun_out/t_tests.log; exit 1; }
tail -1 gpurun_out/t_tests.log
grep -E '^\{"config"' gpurun_out/t_tests.log || true
for c in C2 C3 C4; do
  timeout -k 10 300 python3 -u bench.py --config $c --steps 3 --warmup 1 --no-extra --no-cpu-baseline > gpurun_out/t_bench_$c.log 2>&1 || { tail -20 gpurun_out/t_bench_$c.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/t_bench_$c.log').read().strip().splitlines()[-1]); print('$c', d['value'], d['mt_per_step'], d['roofline']['countt_per_sample']['rays'])"
  timeout -k 10 300 python3 -u tools/occupancy_probe.py $c 1,8 "fixed_point=1;fixed_point=0" > gpurun_out/t_tilet_$c.log 2>&1 || exit 1
  cat gpurun_out/t_tilet_$c.log
done
echo "session T done"
