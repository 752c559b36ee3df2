#!/bin/bash
# rocprofv3 passes for the benchmark workload (run on the GPU box from the repo root).
# Kernel trace + stats in one run; each PMC counter group in its own run (no sys/runtime trace).
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
ARGS=${BENCH_ARGS:-"--steps 10 --warmup 2 --no-cpu-baseline"}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python3 bench.py $ARGS > "$OUT/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum --output-format csv -d "$OUT/dram" -o dram -- python3 bench.py $ARGS > "$OUT/dram.log" 2>&1
echo profiles done
