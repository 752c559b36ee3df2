#!/bin/bash
# quick A/B timing of the C2 workload (no CPU baseline), several variants in one box call
set -e
for t in fast ref; do for b in 64 128 256; do
  echo "traversal=$t block=$b $(timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --traversal $t --block $b 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "Msamples/s", d["roofline"]["kernel_ms"], "ms/kernel")')"
done; done
