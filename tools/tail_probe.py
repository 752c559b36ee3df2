"""Tail of a frame launch: time one frame alone and K frames launched back to back on K streams
(independent launches that overlap on the GPU); tail ~ (K * T1 - TK) / (K - 1).

    python tools/tail_probe.py [CONFIG] [K]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from ensem3a_openclraytracer_amd import _native, workloads as W
    name = sys.argv[1] if len(sys.argv) > 1 else "C2"
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    sc, cam, env, npix, spp, mb, ibl = W.CONFIGS[name].inputs()
    ctxs = []
    for _ in range(K):   # one context per stream: each launch has its own work block
        c = _native.Context(device_ids=[0])
        c.set_scene(sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.BVH.exportArray)
        c.set_env(ibl)
        ctxs.append(c)
    outs = [torch.empty(3 * npix, dtype=torch.float32, device="cuda") for _ in range(K)]
    streams = [torch.cuda.Stream() for _ in range(K)]

    def run(k, reps=5):
        for c, o, s in zip(ctxs[:k], outs, streams):
            c.render_device(cam, env, npix, spp, mb, 0, 1, o.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            for c, o, s in zip(ctxs[:k], outs, streams):
                c.render_device(cam, env, npix, spp, mb, 0, 1, o.data_ptr(), s.cuda_stream)
            torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3

    t1 = run(1)
    tk = run(K)
    same = all(torch.equal(outs[0], o) for o in outs[1:])
    print(json.dumps({"config": name, "K": K, "one_ms": round(t1, 3), "K_overlapped_ms": round(tk, 3),
                      "tail_ms_est": round((K * t1 - tk) / (K - 1), 3), "identical": same}), flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
