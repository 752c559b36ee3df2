set -o pipefail
timeout -k 10 300 python bench.py > gpurun_out/bench_C2.json 2> gpurun_out/bench.err &&
timeout -k 10 300 python bench.py --config C3 --steps 3 --warmup 1 > gpurun_out/bench_C3.json 2>> gpurun_out/bench.err &&
timeout -k 10 300 python bench.py --config C4 --steps 3 --warmup 1 > gpurun_out/bench_C4.json 2>> gpurun_out/bench.err &&
timeout -k 10 400 python bench.py --config C5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/bench_C5.json 2>> gpurun_out/bench.err
r=$?; cat gpurun_out/bench_C*.json; tail -5 gpurun_out/bench.err; exit $r
