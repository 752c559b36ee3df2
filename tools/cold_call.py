"""Repeat bench.py's cold_call (a fresh KernelLauncher's first launch_Raytracing into host memory, split
into packing / uploads / IBL / render + read-back) on a config: the spread of a one-off cost.

    python tools/cold_call.py CONFIG[,CONFIG...] [REPS]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    for cfg in sys.argv[1].split(","):   # CONFIG[,CONFIG...]: in this order, in one process
        for r in range(reps):
            print(json.dumps({"config": cfg, "rep": r, **bench.cold_call(cfg, 0)}), flush=True)


if __name__ == "__main__":
    main()
