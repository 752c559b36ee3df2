#!/bin/bash
# round-3 GPU session E: the N>1 bench path rehearsed on one GPU (2 ranks on device 0, gloo
# collectives: BENCH_SAME_DEVICE=1) with the per-config multi-GPU lines, then the GPU test suite
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
BENCH_SAME_DEVICE=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --check > gpurun_out/e_rehearsal.log 2>&1 || { tail -30 gpurun_out/e_rehearsal.log; exit 1; }
grep '^{"metric"' gpurun_out/e_rehearsal.log | cut -c1-1500
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/e_tests.log 2>&1 || { tail -30 gpurun_out/e_tests.log; exit 1; }
tail -1 gpurun_out/e_tests.log
echo "session E done"
