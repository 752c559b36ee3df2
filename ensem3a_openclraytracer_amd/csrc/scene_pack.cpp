// Host-side scene preparation (scene_pack.h): the reference's flat arrays -> the device layouts.
// Host-only C++ (no HIP), so the sanitizer build (oracle/Makefile asan) covers it.
#include "scene_pack.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <atomic>
#include <map>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/rt_api.h"
#include "../../include/rt_debug.h"
#include "../../include/rt_scene.h"
#include "bvh_sah.h"

using rt::HostScene;

namespace {

inline int32_t as_i32(float f) {
    int32_t i;
    std::memcpy(&i, &f, 4);
    return i;
}
inline float as_f32(int32_t i) {
    float f;
    std::memcpy(&f, &i, 4);
    return f;
}

// Reference index stored as float -> int, like (int)BVH[...] in MathLib.cl.
// Returns false for values the kernel could not use safely.
inline bool fidx(float v, int64_t limit, int32_t* out) {
    if (!(v == v) || v < -1.0f || v >= (float)limit + 1.0f) return false;
    const int32_t i = (int32_t)v;
    if (i < -1 || i >= limit) return false;
    *out = i;
    return true;
}

// p + q * s in fp32 (q * s is exact: s is a power of two): a quantised box bound, exactly as the
// kernels dequantise it (rt_kernels.hip wide_step; this file is built with -ffp-contract=off).
inline float deq(float p, uint32_t q, float s) { return p + (float)q * s; }


// f(begin, end) over [0, n) in chunks of `grain`, on up to 16 host threads (the caller's included)
template <class F>
void parallel_for(int64_t n, int64_t grain, F f) {
    const int64_t chunks = (n + grain - 1) / grain;
    const int nt = (int)std::min<int64_t>(chunks, std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
    if (nt <= 1) {
        if (n > 0) f(0, n);
        return;
    }
    std::atomic<int64_t> next{0};
    auto run = [&]() {
        for (int64_t k; (k = next.fetch_add(1)) < chunks;) f(k * grain, std::min(n, (k + 1) * grain));
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) {
        try {
            pool.emplace_back(run);
        } catch (const std::system_error&) {   // no more threads: the ones started (and this one) do the rest
            break;
        }
    }
    run();
    for (auto& t : pool) t.join();
}

int fail(std::string& msg, int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    msg = buf;
    return code;
}

}  // namespace

// Per-axis quantisation of up to 4 child boxes against their union's lower corner p: a scale
// 2^e and byte bounds whose dequantised box contains each child's exact box.  Returns the
// biased exponent byte (scale = as_float(e << 23)), or -1 when no exponent up to 2^100 gives
// containing bounds (non-finite bounds, or an extent beyond 255 * 2^100): the caller must then not
// use the quantised layout (a dequantised box that is not a superset could cull a hit subtree).
extern "C" int rt_debug_quantise_axis(float p, const float* lo, const float* hi, int n, float gap, uint8_t* qlo,
                                      uint8_t* qhi) {
    if (n < 1 || n > 4 || !lo || !hi || !qlo || !qhi) return -1;
    if (!std::isfinite(p) || !std::isfinite(gap) || gap < 0.0f) return -1;
    double ext = 0.0;
    for (int c = 0; c < n; ++c) {
        if (!std::isfinite(lo[c]) || !std::isfinite(hi[c])) return -1;
        ext = std::max(ext, (double)hi[c] + gap - (double)p);
    }
    int e = ext > 0.0 ? (int)std::ceil(std::log2(ext / 255.0)) : -100;
    e = std::min(std::max(e, -100), 100);
    // a bound with q > 0 lies at least `gap` outside its child's exact bound, in exact arithmetic (the
    // kernels' origin-folded form fma(q, s, p - o) is then conservative, rt_device.h wide_node); q = 0
    // is the corner p itself, which both forms dequantise exactly
    auto lo_ok = [&](uint32_t q, float sc, float l) {
        return deq(p, q, sc) <= l && (q == 0 || (double)p + (double)q * sc <= (double)l - gap);
    };
    auto hi_ok = [&](uint32_t q, float sc, float h) {
        return deq(p, q, sc) >= h && (q == 0 ? (double)p >= h : (double)p + (double)q * sc >= (double)h + gap);
    };
    for (;; ++e) {
        const float sc = std::ldexp(1.0f, e);
        bool ok = true;
        for (int c = 0; c < n && ok; ++c) {
            double fl = std::floor(((double)lo[c] - gap - p) / sc), fh = std::ceil(((double)hi[c] + gap - p) / sc);
            uint32_t a = (uint32_t)std::min(255.0, std::max(0.0, fl));
            uint32_t b = (uint32_t)std::min(255.0, std::max(0.0, fh));
            while (a > 0 && !lo_ok(a, sc, lo[c])) --a;
            while (b < 255 && !hi_ok(b, sc, hi[c])) ++b;
            ok = lo_ok(a, sc, lo[c]) && hi_ok(b, sc, hi[c]);
            qlo[c] = (uint8_t)a;
            qhi[c] = (uint8_t)b;
        }
        if (ok) return e + 127;
        if (e >= 100) return -1;
    }
}

namespace {

// Wide layout of the FAST tree (DevScene::wnodes / wleaves, option "bvh_width" 4): the binary tree
// collapsed to nodes of up to 4 children (the internal child with the largest surface area is
// replaced by its two children while fewer than 4), BFS order, 64 bytes per node:
//   float4 (p.x, p.y, p.z, exponent bytes ex | ey << 8 | ez << 16)    p = the children's lower corner
//   int4   child refs: >= 0 wide node, < 0 leaf ~(64 * rank), INT_MIN = empty slot
//   uint4  (lo.x, lo.y, lo.z, hi.x), uint4 (hi.y, hi.z, 0, 0): one byte per child per word
// A child box dequantises per axis as p + q * 2^(e-127), a superset of the child's exact box, so an
// internal child is never rejected where its leaves would pass.  Leaves, one triangle each, are
// 64-byte records in the reference's DFS rank order (rank = record index, the tie break):
// exact leaf box lo.xyz hi.x | hi.yz a.xy | a.z e1.xyz | e2.xyz triangle index.  The leaf step
// tests the exact box again, so the accepted triangles are those of the binary walk.
void emit_wide(HostScene& hs, const int32_t* L, const int32_t* R, const int32_t* T, const float* box, int64_t nn) {
    hs.wnodes.clear();
    hs.wleaves.clear();
    hs.nwnodes = 0;
    hs.wroot_ref = 0;
    hs.wdepth = 1;
    hs.wdq_omax = 0.0f;
    if (hs.ntri > (1 << 25)) return;   // leaf refs ~(64 * rank) must fit 31 bits: no wide layout
    auto is_inner = [&](int64_t i) { return L[i] >= 0; };
    auto area = [&](int64_t i) {
        const float* b = box + 6 * i;
        const double x = (double)b[3] - b[0], y = (double)b[4] - b[1], z = (double)b[5] - b[2];
        return x * y + y * z + z * x;
    };
    auto kids = [&](int32_t n) {
        std::vector<int32_t> k{L[n], R[n]};
        while (k.size() < 4) {
            int best = -1;
            for (int i = 0; i < (int)k.size(); ++i)
                if (is_inner(k[i]) && (best < 0 || area(k[i]) > area(k[best]))) best = i;
            if (best < 0) break;
            const int32_t c = k[best];
            k[best] = L[c];
            k.insert(k.begin() + best + 1, R[c]);
        }
        return k;
    };
    auto rank_of = [&](int32_t leaf) { return as_i32(hs.tri_geo[12 * (size_t)T[leaf] + 3]); };
    std::vector<int32_t> wide_of(nn, -1), bfs;
    std::vector<std::vector<int32_t>> children;
    if (is_inner(0)) {
        bfs.push_back(0);
        wide_of[0] = 0;
    }
    for (size_t h = 0; h < bfs.size(); ++h) {
        children.push_back(kids(bfs[h]));
        for (int32_t ch : children.back()) {
            if (!is_inner(ch)) continue;
            wide_of[ch] = (int32_t)bfs.size();
            bfs.push_back(ch);
        }
    }
    std::vector<int32_t> need(bfs.size(), 0);
    for (size_t w = bfs.size(); w-- > 0;) {
        int32_t sub = 0;
        for (int32_t ch : children[w])
            if (is_inner(ch)) sub = std::max(sub, need[wide_of[ch]]);
        need[w] = (int32_t)children[w].size() - 1 + sub;
    }
    hs.nwnodes = (int32_t)bfs.size();
    hs.wnodes.assign((size_t)hs.nwnodes * 16, 0.0f);
    int32_t nleaves = 0;
    for (int64_t i = 0; i < nn; ++i)
        if (!is_inner(i) && T[i] >= 0) nleaves = std::max(nleaves, rank_of((int32_t)i) + 1);
    hs.wleaves.assign((size_t)std::max(nleaves, 1) * 16, 0.0f);
    auto leaf_ref = [&](int32_t c) { return ~(64 * rank_of(c)); };
    // the gap of the origin-folded dequantisation: every child bound with q > 0 is
    // quantised at least gap = 2^-17 P outside the exact bound, P = the largest coordinate magnitude of
    // the leaf boxes; that covers the rounding of fma(q, s, p - o) for ray origins up to ~20 P (hit
    // points, and cameras up to DevScene::wdq_omax, checked per frame).  If a node cannot take the gap
    // (no exponent up to 2^100), the whole layout is quantised without it and the exact form runs.
    double pmax = 0.0, bmax = 0.0;   // bmax: the largest |p + q s| the layout holds
    for (int64_t i = 0; i < nn; ++i)
        for (int k = 0; k < 6; ++k) pmax = std::max(pmax, (double)std::fabs(box[6 * i + k]));
    float gap = (std::isfinite(pmax) && pmax > 0x1p-100) ? (float)std::ldexp(pmax, -17) : 0.0f;
    // every node quantises independently: in parallel, with a per-chunk reduction of bmax and of the
    // failure kinds (a node with no room for the gap restarts the whole layout without it)
    auto quantise_all = [&](float g, double* bmax_out) -> int {   // 0 ok, 1 gap failed, 2 no quantisation
        std::atomic<int> fail{0};
        std::mutex mu;
        double bm = 0.0;
        parallel_for((int64_t)bfs.size(), 4096, [&](int64_t w0, int64_t w1) {
            double lbm = 0.0;
            for (int64_t w = w0; w < w1 && fail.load(std::memory_order_relaxed) == 0; ++w) {
                float* o = hs.wnodes.data() + 16 * w;
                const auto& ch = children[w];
                const int n = (int)ch.size();
                float lo[3][4], hi[3][4];
                float p[3];
                for (int a = 0; a < 3; ++a) {
                    p[a] = INFINITY;
                    for (int c = 0; c < n; ++c) {
                        lo[a][c] = box[6 * (int64_t)ch[c] + a];
                        hi[a][c] = box[6 * (int64_t)ch[c] + 3 + a];
                        p[a] = std::min(p[a], lo[a][c]);
                    }
                }
                uint8_t ql[3][4] = {}, qh[3][4] = {};
                uint32_t meta = 0;
                for (int a = 0; a < 3; ++a) {
                    const int ex = rt_debug_quantise_axis(p[a], lo[a], hi[a], n, g, ql[a], qh[a]);
                    if (ex < 0) {
                        fail.store(g > 0.0f ? 1 : 2);
                        return;
                    }
                    meta |= (uint32_t)ex << (8 * a);
                    const double sc = std::ldexp(1.0, ex - 127);
                    for (int c = 0; c < n; ++c)
                        lbm = std::max(lbm, std::max(std::fabs(p[a] + ql[a][c] * sc), std::fabs(p[a] + qh[a][c] * sc)));
                }
                o[0] = p[0]; o[1] = p[1]; o[2] = p[2]; o[3] = as_f32((int32_t)meta);
                for (int c = 0; c < 4; ++c)
                    o[4 + c] = as_f32(c < n ? (is_inner(ch[c]) ? wide_of[ch[c]] : leaf_ref(ch[c])) : INT32_MIN);
                auto pack = [&](const uint8_t* q) {
                    uint32_t v = 0;
                    for (int c = 0; c < 4; ++c) v |= (uint32_t)q[c] << (8 * c);
                    return as_f32((int32_t)v);
                };
                o[8] = pack(ql[0]); o[9] = pack(ql[1]); o[10] = pack(ql[2]); o[11] = pack(qh[0]);
                o[12] = pack(qh[1]); o[13] = pack(qh[2]); o[14] = 0.0f; o[15] = 0.0f;
            }
            std::lock_guard<std::mutex> lk(mu);
            bm = std::max(bm, lbm);
        });
        *bmax_out = bm;
        return fail.load();
    };
    int qf = quantise_all(gap, &bmax);
    if (qf == 1) {   // no room for the gap: quantise without it, exact form only
        gap = 0.0f;
        qf = quantise_all(gap, &bmax);
    }
    if (qf != 0) {   // no containing quantisation: no wide layout (use_wide() keeps the BVH2 walk)
        hs.wnodes.clear();
        hs.wleaves.clear();
        hs.nwnodes = 0;
        hs.wroot_ref = 0;
        hs.wdepth = 1;
        return;
    }
    // origins the gap covers: gap >= u (1 + u) (|p - o| + |p + q s - o| + |b - o|) for every bound, u = 2^-24,
    // with |p|, |b| <= pmax and |p + q s| <= bmax holds for |o| <= (gap / (u (1 + u)) - 2 pmax - bmax) / 3
    // (about 40 pmax); kept 1/2 below that
    {
        const double u = 0x1p-24;
        const double om = gap > 0.0f ? ((double)gap / (u * (1.0 + u)) - 2.0 * pmax - bmax) / 3.0 : 0.0;
        hs.wdq_omax = om > 0.0 ? (float)(0.5 * om) : 0.0f;
    }
    for (int64_t i = 0; i < nn; ++i) {
        if (is_inner(i) || T[i] < 0) continue;
        const int32_t r = rank_of((int32_t)i);
        float* q = hs.wleaves.data() + 16 * (size_t)r;
        const float* b = box + 6 * i;
        const float* g = hs.tri_geo.data() + 12 * (size_t)T[i];
        q[0] = b[0]; q[1] = b[1]; q[2] = b[2]; q[3] = b[3];
        q[4] = b[4]; q[5] = b[5]; q[6] = g[0]; q[7] = g[1];
        q[8] = g[2]; q[9] = g[4]; q[10] = g[5]; q[11] = g[6];
        q[12] = g[8]; q[13] = g[9]; q[14] = g[10]; q[15] = as_f32(T[i]);
    }
    hs.wroot_ref = is_inner(0) ? 0 : leaf_ref(0);
    hs.wdepth = bfs.empty() ? 1 : std::max(1, need[0]);
}

// Emit the FAST node array from a binary tree with one triangle per leaf: internal nodes in BFS
// order, each holding its two children's boxes and refs (rt_internal.h DevScene::nodes).
// box: 6 floats per tree node (lo.xyz, hi.xyz).
void emit_bvh(HostScene& hs, const int32_t* L, const int32_t* R, const int32_t* T, const float* box, int64_t nn) {
    (void)nn;
    auto is_inner = [&](int64_t i) { return L[i] >= 0; };
    std::vector<int32_t> wide_of(nn, -1), bfs;
    if (is_inner(0)) {
        bfs.push_back(0);
        wide_of[0] = 0;
    }
    for (size_t h = 0; h < bfs.size(); ++h) {
        for (int32_t ch : {L[bfs[h]], R[bfs[h]]}) {
            if (!is_inner(ch)) continue;
            wide_of[ch] = (int32_t)bfs.size();
            bfs.push_back(ch);
        }
    }
    // stack bound: a node pushes one entry at most; need = max over root-to-leaf paths of the sum
    // (children are after their parents in BFS order: sweep backwards)
    std::vector<int32_t> need(bfs.size(), 0);
    for (size_t w = bfs.size(); w-- > 0;) {
        int32_t sub = 0;
        for (int32_t ch : {L[bfs[w]], R[bfs[w]]})
            if (is_inner(ch)) sub = std::max(sub, need[wide_of[ch]]);
        need[w] = 1 + sub;
    }
    constexpr int F = 4 * rt::kNodeF4;   // floats per node
    // the FAST traversal's triangle records (DevScene::tri_fast), in the order a depth-first walk of
    // this tree meets its leaves: pos[t] = record of t
    std::vector<int32_t> pos((size_t)hs.ntri, -1);
    {
        int32_t next = 0;
        auto place = [&](int32_t c) {
            if (!is_inner(c) && T[c] >= 0 && pos[T[c]] < 0) pos[T[c]] = next++;
        };
        if (is_inner(0)) {
            std::vector<int32_t> st{0};
            while (!st.empty()) {
                const int32_t n = st.back();
                st.pop_back();
                place(L[n]);
                place(R[n]);
                if (is_inner(R[n])) st.push_back(R[n]);
                if (is_inner(L[n])) st.push_back(L[n]);
            }
        }
        if (!is_inner(0)) place(0);
        for (int32_t t = 0; t < hs.ntri; ++t)
            if (pos[t] < 0) pos[t] = next++;   // unreachable triangles keep their order
        hs.tri_fast.assign(hs.tri_geo.size(), 0.0f);
        for (int32_t t = 0; t < hs.ntri; ++t)
            for (int k = 0; k < 12; ++k) hs.tri_fast[12 * (size_t)pos[t] + k] = hs.tri_geo[12 * (size_t)t + k];
    }
    hs.nnodes = (int32_t)bfs.size();
    hs.nodes.assign((size_t)hs.nnodes * F, 0.0f);
    for (size_t w = 0; w < bfs.size(); ++w) {
        float* o = hs.nodes.data() + (size_t)F * w;
        const int32_t n = bfs[w];
        auto ref = [&](int32_t c) { return is_inner(c) ? wide_of[c] : ~(48 * pos[T[c]]); };
        const float* c0 = box + 6 * (int64_t)L[n];
        const float* c1 = box + 6 * (int64_t)R[n];
        o[0] = c0[0]; o[1] = c0[3]; o[2] = c0[1]; o[3] = c0[4];
        o[4] = c1[0]; o[5] = c1[3]; o[6] = c1[1]; o[7] = c1[4];
        o[8] = c0[2]; o[9] = c0[5]; o[10] = c1[2]; o[11] = c1[5];
        o[12] = as_f32(ref(L[n])); o[13] = as_f32(ref(R[n])); o[14] = 0.0f; o[15] = 0.0f;
    }
    hs.root_ref = is_inner(0) ? 0 : ~(48 * pos[T[0]]);
    for (int k = 0; k < 6; ++k) hs.root_box[k] = box[k];
    hs.depth = bfs.empty() ? 1 : std::max(1, need[0]);
    emit_wide(hs, L, R, T, box, nn);
}

// Pack the FAST layout from the reference export.  Returns false (with
// reason) if the export is not a proper binary tree with one triangle per
// leaf, in which case only the REF traversal is available.  layout
// RT_BVH_REFERENCE keeps the reference's tree, RT_BVH_SAH regroups its leaf
// boxes (bvh_sah.cpp); both give the same hits.
bool pack_fast(HostScene& hs, const float* bvh9, int64_t nn, int64_t ntri, int layout, int brute_max,
               std::string& why) {
    if (nn <= 0) {
        why = "empty BVH";
        return false;
    }
    if (ntri > 0x7fffffff / 48) {  // leaf refs are ~(48 * triangle)
        why = "more than 44.7M triangles";
        return false;
    }
    std::vector<int32_t> L(nn), R(nn), T(nn);
    for (int64_t i = 0; i < nn; ++i) {
        if (!fidx(bvh9[9 * i + 0], nn, &L[i]) || !fidx(bvh9[9 * i + 1], nn, &R[i]) ||
            !fidx(bvh9[9 * i + 8], ntri, &T[i])) {
            why = "index out of range";
            return false;
        }
    }
    // Check the tree shape over the reachable nodes.
    std::vector<uint8_t> seen(nn, 0);
    auto is_leaf = [&](int64_t i) { return L[i] == -1 && R[i] == -1 && T[i] >= 0; };
    auto is_inner = [&](int64_t i) { return L[i] >= 0 && R[i] >= 0 && T[i] == -1; };
    if (!is_leaf(0) && !is_inner(0)) {
        why = "root is neither a one-triangle leaf nor a two-child node";
        return false;
    }
    std::vector<int32_t> tri_seen(ntri, 0), leaves;
    std::vector<int32_t> queue{0};
    seen[0] = 1;
    for (size_t h = 0; h < queue.size(); ++h) {
        const int32_t n = queue[h];
        if (is_leaf(n)) {
            if (tri_seen[T[n]]++) {
                why = "triangle in two leaves";
                return false;
            }
            leaves.push_back(n);
            continue;
        }
        if (!is_inner(n)) {
            why = "node with one child, or with both a triangle and children";
            return false;
        }
        for (int32_t ch : {L[n], R[n]}) {
            if (seen[ch]) {
                why = "node reachable twice (not a tree)";
                return false;
            }
            seen[ch] = 1;
            queue.push_back(ch);
        }
    }
    // Rank of each leaf triangle in the reference visiting order: pre-order
    // DFS, right child first (push left then right, MathLib.cl:269-276).
    std::vector<int32_t> rank(ntri, 0x7fffffff);
    {
        std::vector<int32_t> st;
        st.push_back(0);
        int32_t r = 0;
        while (!st.empty()) {
            const int32_t n = st.back();
            st.pop_back();
            if (T[n] >= 0) rank[T[n]] = r++;
            if (L[n] >= 0) st.push_back(L[n]);
            if (R[n] >= 0) st.push_back(R[n]);
        }
    }
    for (int64_t t = 0; t < ntri; ++t) {
        hs.tri_geo[12 * t + 3] = as_f32(rank[t]);
        hs.tri_geo[12 * t + 7] = as_f32((int32_t)t);   // e1.w: the triangle's own index (FAST hit records)
    }
    // small scenes: brute-force records of the reachable triangles in DFS-rank order
    hs.brute.clear();
    hs.brute_box.clear();
    hs.nbrute = 0;
    hs.nbox = 0;
    if ((int64_t)leaves.size() <= (int64_t)brute_max) {
        std::vector<int32_t> by_rank(leaves.size());
        for (int32_t n : leaves) by_rank[rank[T[n]]] = n;
        hs.brute.assign(16 * by_rank.size(), 0.0f);
        for (size_t q = 0; q < by_rank.size(); ++q) {
            const float* nd = bvh9 + 9 * (int64_t)by_rank[q];
            const int32_t t = T[by_rank[q]];
            const float* g = hs.tri_geo.data() + 12 * t;
            float* r = hs.brute.data() + 16 * q;
            r[0] = nd[2]; r[1] = nd[3]; r[2] = nd[4]; r[3] = nd[5];      // lo.xyz hi.x
            r[4] = nd[6]; r[5] = nd[7]; r[6] = g[0]; r[7] = g[1];        // hi.yz a.xy
            r[8] = g[2]; r[9] = g[4]; r[10] = g[5]; r[11] = g[6];        // a.z e1.xyz
            r[12] = g[8]; r[13] = g[9]; r[14] = g[10]; r[15] = as_f32(t); // e2.xyz tri
        }
        hs.nbrute = (int32_t)by_rank.size();
        // the distinct leaf boxes, 32 bytes each: records whose leaf boxes are bit-identical (the
        // two triangles of an axis-aligned or vertical quad) share one box test, which passes or
        // fails for both.  Each box lists up to two records (the second -1 when alone); padded with
        // never-hit boxes to whole groups of rt::kBoxGroup (the lock-step loop loads a group with
        // one scalar wait).
        std::vector<std::array<int32_t, 2>> groups;
        {
            std::map<std::array<uint32_t, 6>, size_t> open;   // box bits -> group with a free slot
            for (size_t q = 0; q < by_rank.size(); ++q) {
                const float* r = hs.brute.data() + 16 * q;
                std::array<uint32_t, 6> key;
                for (int k = 0; k < 6; ++k) std::memcpy(&key[k], r + k, 4);
                auto it = open.find(key);
                if (it != open.end()) {
                    groups[it->second][1] = (int32_t)q;
                    open.erase(it);
                } else {
                    open[key] = groups.size();
                    groups.push_back({(int32_t)q, -1});
                }
            }
        }
        hs.nbox = (int32_t)groups.size();
        const size_t ng = (groups.size() + rt::kBoxGroup - 1) / rt::kBoxGroup * rt::kBoxGroup;
        hs.brute_box.assign(8 * ng, 0.0f);
        for (size_t g = 0; g < ng; ++g) {
            float* b = hs.brute_box.data() + 8 * g;
            if (g < groups.size()) {
                const float* r = hs.brute.data() + 16 * groups[g][0];   // lo.xyz hi.x | hi.yz ...
                b[0] = r[0]; b[1] = r[3];                                // lo.x hi.x
                b[2] = r[1]; b[3] = r[4];                                // lo.y hi.y
                b[4] = r[2]; b[5] = r[5];                                // lo.z hi.z
                b[6] = as_f32(groups[g][0]); b[7] = as_f32(groups[g][1]);
            } else {
                for (int k = 0; k < 6; ++k) b[k] = 1e30f;                // a point far beyond any k < 1000
                b[6] = as_f32(-1); b[7] = as_f32(-1);
            }
        }
    }
    if (layout == RT_BVH_SAH && leaves.size() > 1) {
        std::vector<float> lb(6 * leaves.size());
        std::vector<int32_t> ids(leaves.size());
        for (size_t q = 0; q < leaves.size(); ++q) {
            const float* nd = bvh9 + 9 * (int64_t)leaves[q];
            for (int k = 0; k < 6; ++k) lb[6 * q + k] = nd[2 + k];
            ids[q] = T[leaves[q]];
        }
        rt::SahTree st;
        rt::sah_build(lb.data(), ids.data(), (int64_t)leaves.size(), st);
        emit_bvh(hs, st.L.data(), st.R.data(), st.leaf.data(), st.box.data(), (int64_t)st.L.size());
        return true;
    }
    std::vector<float> box(6 * nn);
    for (int64_t i = 0; i < nn; ++i)
        for (int k = 0; k < 6; ++k) box[6 * i + k] = bvh9[9 * i + 2 + k];
    emit_bvh(hs, L.data(), R.data(), T.data(), box.data(), nn);
    return true;
}

}  // namespace

namespace rt {

void pack_checked(HostScene& hs, const float* bvh9, int64_t nb, int64_t ntri, int layout, int brute_max,
                  std::string& why) {
    hs.fast_ok = (ntri > 0) ? pack_fast(hs, bvh9, nb, ntri, layout, brute_max, why) : true;
    if (hs.fast_ok && ntri > 0) {
        // the FAST kernels' Moller-Trumbore reciprocal (rt_device.h mt_recip) is IEEE-exact for
        // |a| <= 2^126, a = e1 . (d x e2) with |d| = 1: bound |e1| |e2| (finite edges; an infinite or
        // NaN edge makes a infinite or NaN, which mt_recip also returns exactly) 64x below it
        double m1 = 0.0, m2 = 0.0;
        for (int64_t t = 0; t < ntri; ++t) {
            const float* g = hs.tri_geo.data() + 12 * t;
            const double l1 = std::sqrt((double)g[4] * g[4] + (double)g[5] * g[5] + (double)g[6] * g[6]);
            const double l2 = std::sqrt((double)g[8] * g[8] + (double)g[9] * g[9] + (double)g[10] * g[10]);
            if (std::isfinite(l1)) m1 = std::max(m1, l1);
            if (std::isfinite(l2)) m2 = std::max(m2, l2);
        }
        if (!(m1 * m2 <= std::ldexp(1.0, 120))) {
            hs.fast_ok = false;
            why = "triangle edges beyond 2^60 (the FAST reciprocal needs |e1 . (d x e2)| <= 2^126)";
        }
    }
    if (ntri == 0) {
        hs.nnodes = 0; hs.root_ref = 0; hs.depth = 1; hs.nodes.clear();
        hs.nwnodes = 0; hs.wroot_ref = 0; hs.wdepth = 1; hs.wnodes.clear(); hs.wleaves.clear();
        hs.brute.clear(); hs.brute_box.clear(); hs.nbrute = 0; hs.nbox = 0;
    }
    if (!hs.fast_ok) { hs.brute.clear(); hs.brute_box.clear(); hs.nbrute = 0; hs.nbox = 0; }
    if (!hs.fast_ok || hs.wdepth > 64) { hs.wnodes.clear(); hs.wleaves.clear(); hs.nwnodes = 0; hs.wdepth = 1; }
    // render kernels keep kStackLds entries in LDS and spill deeper ones to HBM; the single-ray
    // debug kernel keeps the whole stack in LDS (int2 entries, 128 lanes): depth <= 64
    if (hs.fast_ok && hs.depth > 64) {
        hs.fast_ok = false;
        why = "tree deeper than 64 levels";
    }
    if (hs.nodes.empty()) hs.nodes.assign(4 * rt::kNodeF4, 0.0f);
    if (hs.brute.empty()) hs.brute.assign(16, 0.0f);
    if (hs.brute_box.empty()) hs.brute_box.assign(8 * rt::kBoxGroup, 1e30f);
}

namespace {

int scene_prepare_(HostScene& hs, const float* vp, int64_t nvp, const float* vn, int64_t nvn, const int32_t* face,
                   int64_t nface, const float* mat, int64_t nmat, const float* bvh9, int64_t nbvh, int layout,
                   int brute_max, std::string& msg, std::string& why) {
    if (nvp < 0 || nvp % 3 || nvn < 0 || nvn % 3 || nface < 0 || nface % 10 || nmat <= 0 || nmat % 6 || nbvh < 0 ||
        nbvh % 9)
        return fail(msg, RT_ERR_ARG,
                       "bad array sizes (V_p %lld, V_n %lld, faceData %lld, materialData %lld, BVH %lld)",
                       (long long)nvp, (long long)nvn, (long long)nface, (long long)nmat, (long long)nbvh);
    if ((nface && (!vp || !vn || !face)) || !mat || (nbvh && !bvh9))
        return fail(msg, RT_ERR_ARG, "null array");
    const int64_t T = nface / 10, NV = nvp / 3, NN = nvn / 3, M = nmat / 6, NB = nbvh / 9;
    if (T > 0x3fffffff || NB > 0x7fffffff) return fail(msg, RT_ERR_ARG, "scene too large");
    if (T > 0 && NB == 0) return fail(msg, RT_ERR_SCENE, "triangles given without a BVH");
    for (int64_t m = 0; m < M; ++m) {
        const float tf = mat[6 * m];
        if (!(tf > -1.0f && tf < 4.0f))
            return fail(msg, RT_ERR_SCENE, "material %lld has type %g; the kernel defines types 0..3", (long long)m,
                           (double)tf);
    }
    hs.ntri = (int32_t)T;
    hs.nmat = (int32_t)M;
    hs.nbvh9 = (int32_t)NB;
    hs.mat.assign((size_t)rt::kMatF * M, 0.0f);   // rows padded to kMatF floats (DevScene::mat)
    for (int64_t m = 0; m < M; ++m) {
        for (int k = 0; k < 6; ++k) hs.mat[(size_t)rt::kMatF * m + k] = mat[6 * m + k];
        for (int k = 1; k < 4; ++k) hs.colors_finite = hs.colors_finite && std::isfinite(mat[6 * m + k]);
        hs.has_glass = hs.has_glass || (int)mat[6 * m] == 3;
    }
    if (bvh9) hs.bvh9.assign(bvh9, bvh9 + nbvh);
    hs.tri_geo.assign((size_t)T * 12, 0.0f);
    hs.tri_shade.assign((size_t)T * 4, 0.0f);
    for (int64_t t = 0; t < T; ++t) {
        const int32_t* f = face + 10 * t;
        if (f[0] < 0 || f[0] >= M)
            return fail(msg, RT_ERR_ARG, "triangle %lld: material %d out of range [0,%lld)", (long long)t, f[0],
                           (long long)M);
        for (int j = 7; j < 10; ++j)
            if (f[j] < 0 || f[j] >= NV)
                return fail(msg, RT_ERR_ARG, "triangle %lld: position index %d out of range", (long long)t, f[j]);
        if (f[4] < 0 || f[4] >= NN)
            return fail(msg, RT_ERR_ARG, "triangle %lld: normal index %d out of range", (long long)t, f[4]);
        const float* a = vp + 3 * (int64_t)f[7];
        const float* b = vp + 3 * (int64_t)f[8];
        const float* c = vp + 3 * (int64_t)f[9];
        float* g = hs.tri_geo.data() + 12 * t;
        g[0] = a[0]; g[1] = a[1]; g[2] = a[2]; g[3] = 0.0f;
        g[4] = b[0] - a[0]; g[5] = b[1] - a[1]; g[6] = b[2] - a[2]; g[7] = 0.0f;
        g[8] = c[0] - a[0]; g[9] = c[1] - a[1]; g[10] = c[2] - a[2]; g[11] = 0.0f;
        const float* n = vn + 3 * (int64_t)f[4];
        float* sh = hs.tri_shade.data() + 4 * t;
        sh[0] = n[0]; sh[1] = n[1]; sh[2] = n[2]; sh[3] = as_f32(f[0]);
    }
    // REF traversal safety: every index the reference would follow must be in range.
    for (int64_t i = 0; i < NB; ++i) {
        int32_t l, r, t;
        if (!fidx(bvh9[9 * i + 0], NB, &l) || !fidx(bvh9[9 * i + 1], NB, &r) || !fidx(bvh9[9 * i + 8], T, &t))
            return fail(msg, RT_ERR_SCENE, "BVH node %lld has an index out of range", (long long)i);
    }
    // The reference loops forever on a cyclic node graph; refuse it instead of hanging the GPU.
    if (NB > 0) {
        std::vector<uint8_t> color(NB, 0);  // 0 new, 1 on path, 2 done
        std::vector<std::pair<int32_t, int>> st;
        st.push_back({0, 0});
        color[0] = 1;
        while (!st.empty()) {
            auto& top = st.back();
            const int32_t n = top.first;
            if (top.second < 2) {
                const int32_t ch = (int32_t)bvh9[9 * (int64_t)n + top.second];
                ++top.second;
                if (ch < 0) continue;
                if (color[ch] == 1) return fail(msg, RT_ERR_SCENE, "BVH node graph has a cycle through node %d", ch);
                if (color[ch] == 0) { color[ch] = 1; st.push_back({ch, 0}); }
            } else {
                color[n] = 2;
                st.pop_back();
            }
        }
    }
    pack_checked(hs, bvh9, NB, T, layout, brute_max, why);
    return RT_OK;
}

}  // namespace

// No C++ exception leaves the C ABI: a scene too large for host memory is an error status.
int scene_prepare(HostScene& hs, const float* vp, int64_t nvp, const float* vn, int64_t nvn, const int32_t* face,
                  int64_t nface, const float* mat, int64_t nmat, const float* bvh9, int64_t nbvh, int layout,
                  int brute_max, std::string& msg, std::string& why) {
    try {
        return scene_prepare_(hs, vp, nvp, vn, nvn, face, nface, mat, nmat, bvh9, nbvh, layout, brute_max, msg, why);
    } catch (const std::bad_alloc&) {
        hs = HostScene();
        return fail(msg, RT_ERR_ARG, "scene too large for host memory");
    } catch (const std::exception& e) {
        hs = HostScene();
        return fail(msg, RT_ERR_ARG, "scene preparation failed: %s", e.what());
    }
}

}  // namespace rt

namespace {
thread_local std::string g_check_error;
}

extern "C" int rt_scene_check(const float* vp, int64_t nvp, const float* vn, int64_t nvn, const int32_t* face,
                              int64_t nface, const float* mat, int64_t nmat, const float* bvh9, int64_t nbvh,
                              int layout, int64_t info[8]) {
    HostScene hs;
    std::string msg, why;
    if (layout != RT_BVH_REFERENCE && layout != RT_BVH_SAH) {
        g_check_error = "layout must be RT_BVH_REFERENCE or RT_BVH_SAH";
        return RT_ERR_ARG;
    }
    const int rc = rt::scene_prepare(hs, vp, nvp, vn, nvn, face, nface, mat, nmat, bvh9, nbvh, layout,
                                     RT_BRUTE_MAX_DEFAULT, msg, why);
    g_check_error = rc != RT_OK ? msg : hs.fast_ok ? std::string() : "FAST traversal unavailable (" + why + ")";
    if (rc == RT_OK && info) {
        info[0] = hs.ntri;
        info[1] = hs.nnodes;
        info[2] = hs.depth;
        info[3] = hs.nwnodes;
        info[4] = hs.wdepth;
        info[5] = hs.nbrute;
        info[6] = hs.nbox;
        info[7] = hs.fast_ok ? 1 : 0;
    }
    return rc;
}

extern "C" const char* rt_scene_last_error(void) { return g_check_error.c_str(); }
