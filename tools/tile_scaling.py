"""Predict strong scaling of the row-interleaved frame split on one GPU: time the tile one rank of
an N-GPU run renders (rows r::N) for N = 1, 2, 4, 8 and report T(1) / (N * T(N)).
With TEAMS="0 1" (rt_set_option "team" values) each tile is rendered once per value, timed
separately, and checked bit-identical against the first value.

    [TEAMS="0 1"] python tools/tile_scaling.py [CONFIG]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from ensem3a_openclraytracer_amd import _native
    from ensem3a_openclraytracer_amd import distributed as D
    from ensem3a_openclraytracer_amd import workloads as W
    name = sys.argv[1] if len(sys.argv) > 1 else "C2"
    sc, cam, env, npix, spp, mb, ibl = W.CONFIGS[name].inputs()
    ctx = _native.Context(device_ids=[0])
    ctx.set_scene(sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.BVH.exportArray)
    ctx.set_env(ibl)
    width = int(cam[6])
    teams = [int(t) for t in os.environ.get("TEAMS", "0").split()]
    t1 = {}
    for n in (1, 2, 4, 8):
        rows = D.max_tile_rows(npix, width, n)
        out = torch.empty(3 * width * rows, dtype=torch.float32, device="cuda")
        first = {}
        for team in teams:
            ctx.set_option("team", team)
            worst, same = 0.0, True
            for r in (0, n - 1):
                ctx.render_device(cam, env, npix, spp, mb, r, n, out.data_ptr())
                torch.cuda.synchronize()
                if r not in first:
                    first[r] = out.clone()
                else:
                    same = same and torch.equal(first[r], out)
                t0 = time.perf_counter()
                for _ in range(5):
                    ctx.render_device(cam, env, npix, spp, mb, r, n, out.data_ptr())
                torch.cuda.synchronize()
                worst = max(worst, (time.perf_counter() - t0) / 5)
            t1.setdefault(team, worst)
            print(json.dumps({"config": name, "team": team, "n": n, "tile_ms": round(worst * 1e3, 3),
                              "predicted_efficiency": round(t1[team] / (n * worst), 3),
                              "vs_n1_team_first": round(t1[teams[0]] / (n * worst), 3),
                              "identical_to_first_team": same}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
