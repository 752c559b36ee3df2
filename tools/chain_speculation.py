"""Price sample-parallel speculation for small tiles, on the CPU oracle.

A pixel's samples form one chain: sample k starts at RNG offset D_k (draws consumed by samples
0..k-1) and its colour and draw count are a function of D_k alone (the primary hit is cached,
Raytracing.cl:184-206).  T lanes per pixel could run trails from guessed offsets G_t and stitch
the chain where it lands on a computed offset (trails merge once they share an offset), keeping
the frame bit-identical.  This script measures, per sampled pixel, the chain latency in traced
rays for T = 1..4 with G_t = t * spp / T * mu (static guesses), against the serial chain.

    python tools/chain_speculation.py [CONFIG] [PIXELS] [MU]   (MU 0: per pixel, from a spp/8 pilot)
"""
import ctypes
import heapq
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def trails(osc, cam, env, npix, mb, pixels, P):
    import oracle.oracle as O
    L = O.lib()
    vp = ctypes.c_void_p
    L.oracle_sample_trail.argtypes = [ctypes.POINTER(O._Scene), vp, vp, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_int32, ctypes.c_int32, vp, vp, vp]
    out = []
    for i in pixels:
        col = np.zeros(3 * P, np.float32)
        nd = np.zeros(P, np.int32)
        nr = np.zeros(P, np.int32)
        L.oracle_sample_trail(ctypes.byref(osc.c), cam.ctypes.data, env.ctypes.data, int(npix), int(mb), int(i),
                              int(P), col.ctypes.data, nd.ctypes.data, nr.ctypes.data)
        out.append((int(i), col.reshape(P, 3), nd, nr))
    return out


def chain(nd, spp):
    D, seq = 0, []
    for _ in range(spp):
        seq.append(D)
        if nd[D // 2] == 0:
            seq += [D] * (spp - len(seq))
            break
        D += nd[D // 2]
    return seq


def pilot_mu(nd, spp, k):
    """Draws per sample over the chain's first k samples (what a pilot pass of k samples knows)."""
    seq = chain(nd, k + 1)
    return max(seq[-1] / k, 2.0)


def modal_draws(nd, k):
    """The most frequent draw count of the chain's first k samples (what a pilot pass of k samples saw)."""
    seq = chain(nd, k)
    vals, cnt = np.unique([int(nd[D // 2]) for D in seq], return_counts=True)
    return int(vals[np.argmax(cnt)])


def speculate(nd, nr, spp, T, mu, k=0, snap=0):
    """Event simulation: lanes walk trails from G_t, a lane stops on an offset already computed or
    being computed; returns (time the chain is complete, total rays traced) in rays.
    k > 0: the chain's first k samples are already done (a pilot pass, rt_spec.hip): trail 0 continues
    from their end offset D0 and trail t > 0 starts at D0 + ahead_t, ahead_t = t (spp - k) / T * mu
    draws; snap > 0 rounds ahead_t to a multiple of snap draws (the pixel's modal draws per sample), so
    that a trail starts on the chain's own offsets wherever the samples between D0 and it all drew
    the modal count (C2's samples mostly draw 10)."""
    P = len(nd)
    cost = lambda p: max(int(nr[p // 2]), 1)   # noqa: E731
    done, claim, ev, work = {}, {}, [], 0
    pre = chain(nd, k + 1) if k > 0 else [0]
    D0 = pre[-1]
    t0 = 0   # the pilot's samples run serially first (pass 1), their rays are work too
    for q in dict.fromkeys(pre[:-1]):
        t0 += cost(q)
        done[q] = t0
    work += t0
    for t in range(T):
        ahead = t * (spp - k) / T * mu
        g = D0 + (int(round(ahead / snap)) * snap if snap > 0 else int(round(ahead / 2)) * 2)
        if g // 2 < P and g not in claim and g not in done:
            claim[g] = t
            heapq.heappush(ev, (t0 + cost(g), t, g))
    seq = chain(nd, spp)
    tnow = 0
    while ev:
        tnow, t, p = heapq.heappop(ev)
        done[p] = tnow
        work += cost(p)
        if all(q in done for q in seq):
            return max(done[q] for q in seq), work
        q = p + int(nd[p // 2])
        if nd[p // 2] == 0 or q // 2 >= P or q in done or q in claim:
            continue
        claim[q] = t
        heapq.heappush(ev, (tnow + cost(q), t, q))
    tt = tnow
    for q in seq:   # chain left every trail: finish it serially
        if q not in done:
            tt += cost(q)
            work += cost(q)
            done[q] = tt
    return max(done[q] for q in seq), work


def main():
    import oracle.oracle as O
    from ensem3a_openclraytracer_amd import workloads as W
    name = sys.argv[1] if len(sys.argv) > 1 else "C2"
    npx = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    mu = float(sys.argv[3]) if len(sys.argv) > 3 else 6.0
    sc, cam, env, npix, spp, mb, ibl = W.CONFIGS[name].inputs()
    osc = O.OracleScene.from_scene(sc, ibl)
    cam = np.ascontiguousarray(cam, np.float32)
    env = np.ascontiguousarray(env, np.float32)
    P = spp * (mb + 1) + 64
    pixels = np.random.default_rng(1).choice(npix, npx, replace=False)
    tr = trails(osc, cam, env, npix, mb, pixels, P)
    # the stitched chain reproduces the oracle's pixel bit for bit
    W_ = int(cam[6])
    for i, col, nd, nr in tr[:16]:
        acc = np.zeros(3, np.float32)
        for D in chain(nd, spp):
            acc = acc + col[D // 2]
        got = np.clip(acc / np.float32(spp), 0, 1).astype(np.float32)
        ref = O.render(osc, cam, env, npix, spp, mb, row0=i // W_, row_step=npix).reshape(-1, 3)[i % W_]
        assert np.array_equal(got, ref), i
    # the serial chain as the product traces it: a sample that draws nothing repeats for the rest of the
    # pixel and is traced once (fixed_point), so every distinct offset is counted once
    ser = np.array([sum(max(int(nr[D // 2]), 1) for D in set(chain(nd, spp))) for _, _, nd, nr in tr])
    mus = np.array([chain(nd, spp + 1)[-1] / spp for _, _, nd, _ in tr])
    print(f"{name}: {npx} pixels, draws/sample mean {mus.mean():.2f} (std {mus.std():.2f}); serial chain "
          f"mean {ser.mean():.1f} rays, max {ser.max()}")
    k = max(spp // 8, 1)
    modes = os.environ.get("SPEC_MODES", "static").split(",")
    for mode in modes:
        # static: guesses from offset 0, no pilot (r03 pricing); pilot: trails after a spp/8 pilot, as the
        # r04 kernel runs them; snap: the pilot's guesses rounded to multiples of the modal draw count
        for T in [int(x) for x in os.environ.get("SPEC_TRAILS", "2,3,4").split(",")]:
            r = []
            for _, _, nd, nr in tr:
                m = mu if mu > 0 else pilot_mu(nd, spp, k)
                if mode == "static":
                    r.append(speculate(nd, nr, spp, T, m))
                else:
                    r.append(speculate(nd, nr, spp, T, m, k=k, snap=modal_draws(nd, k) if mode == "snap" else 0))
            lat = np.array([a for a, _ in r], float)
            wk = np.array([b for _, b in r], float)
            # the pilot modes count the pilot's rays too (they are part of the tile's time)
            print(f"{mode} T={T}: latency mean {lat.mean():.1f} p99 {np.percentile(lat, 99):.1f} max {lat.max():.0f} "
                  f"rays (max {ser.max() / lat.max():.2f}x shorter than serial), work {wk.sum() / ser.sum():.3f}x",
                  flush=True)


if __name__ == "__main__":
    main()
