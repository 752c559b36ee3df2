"""Collect row-tile timings (tools/occupancy_probe.py JSON lines, e.g. gpurun_out/SESSION_n_tiles.log) into a
committed tile-scaling profile: the N-GPU speed-up each config's tile times predict (rank 0's tile,
rows 0::N, rendered alone on one MI355X with the product defaults; the RCCL gather adds ~0.1 ms).

    python tools/tile_scaling.py OUT.json "NOTE" LOG [LOG ...]
"""
import json
import sys


def main():
    out, note, logs = sys.argv[1], sys.argv[2], sys.argv[3:]
    rows = []
    for path in logs:
        with open(path, errors="replace") as f:
            for ln in f:
                if ln.startswith("{"):
                    r = json.loads(ln)
                    if not r.get("opts"):   # product defaults only
                        rows.append(dict(r, source=path.split("/")[-1]))
    t = {(r["config"], r["n"]): r["tile_ms"] for r in rows}
    pred = {}
    for cfg in sorted({c for c, _ in t}):
        if (cfg, 1) in t:
            pred[cfg] = {f"N={n}": round(t[cfg, 1] / t[cfg, n], 2) for n in (2, 4, 8) if (cfg, n) in t}
    res = {"source": "tools/occupancy_probe.py on one MI355X via tools/gpu_session.py (tiles= steps): rank 0's row "
                     "tile (rows 0::N) rendered alone with the product defaults; 3 reps at N=1, 5 otherwise",
           "note": note, "predicted_speedup": pred, "rows": rows}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(pred, indent=1))


if __name__ == "__main__":
    main()
