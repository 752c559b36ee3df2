// Device code shared by the render kernels (rt_kernels.hip: the per-lane megakernels; rt_spec.hip: the
// speculative-trail kernel): traversals, shading arithmetic, launch constants, pixel hand-out.  Included by
// the .hip translation units only; everything is internal to each of them (anonymous namespace).
//
// Numerics: every OpenCL builtin of the reference is taken from rtm.h and the including file is
// compiled with -ffp-contract=off (see rtm.h).
#pragma once
#include <algorithm>
#include <climits>

#include "rt_internal.h"
#include "rtm.h"

namespace rt {

namespace {

// Scenes whose BVH2 nodes + triangles take at most this many bytes are staged in LDS.
constexpr size_t kLdsSceneMax = 24 * 1024;

constexpr int TRAV_FAST = 0;
constexpr int TRAV_REF = 1;
constexpr int REF_STACK = 20;  // stack.cl:4, Raytracing capacity 20 (DevScene::ref_stack: the REF traversal's cap)

struct Hit {
    float k;
    int tri;  // < 0: miss
};

// Work counters of the instrumented (COUNT) kernels, summed over the launch; the order is the
// public one of rt_count_work_detail (include/rt_api.h).
struct Cnt {
    unsigned long long nodes, tris, rays, env, dropped;
    unsigned long long wave_trav;   // traversal-loop iterations issued per wave (any lane active)
    unsigned long long wave_outer;  // render-loop iterations per wave
    unsigned long long cyc_shade;   // resumable kernel, per wave: clock cycles outside the traversal rounds
    unsigned long long cyc_trav;    //   ... and inside them
    unsigned long long boxes;       // ray-box slab tests (a FAST node tests 2, a REF node 1, brute force: distinct leaf boxes)
    unsigned long long diffuse, glossy, glass;   // shading events (naiveGI bounces) by material type 1 / 2 / 3
    unsigned long long sun;         // sun terms evaluated (Raytracing.cl:115-137)
    unsigned long long samples;     // samples completed
};
constexpr int NCOUNTS = 15;

__device__ __forceinline__ void count_event(Cnt& c, int type) {
    if (type == 1) c.diffuse++;
    else if (type == 2) c.glossy++;
    else c.glass++;
}

// COUNT builds: the lowest active lane of the wave counts one wave-level iteration.
__device__ __forceinline__ void count_wave(unsigned long long& x) {
    if ((int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1) x++;
}

__device__ __forceinline__ rtm_f3 xyz(float4 v) { return rtm_v3(v.x, v.y, v.z); }

// Moller-Trumbore exactly as MathLib.cl:117-160 on pre-gathered a.p, e1, e2
// (e1 = b.p - a.p and e2 = c.p - a.p are computed on the host in float32, the
// same operations the reference performs per test).
__device__ __forceinline__ bool mt_test(const float4* __restrict__ tg, int t, rtm_f3 o, rtm_f3 d,
                                        float* kout, int* rank) {
    const float4 g0 = tg[3 * t + 0];
    const float4 g1 = tg[3 * t + 1];
    const float4 g2 = tg[3 * t + 2];
    const rtm_f3 e1 = xyz(g1), e2 = xyz(g2);
    const rtm_f3 h = rtm_cross(d, e2);
    const float a = rtm_dot(e1, h);
    if (a > -0.0000001f && a < 0.0000001f) return false;
    const float f = 1.0f / a;
    const rtm_f3 s = rtm_sub(o, xyz(g0));
    const float u = f * rtm_dot(s, h);
    if (u < 0.0f || u > 1.0f) return false;
    const rtm_f3 q = rtm_cross(s, e1);
    const float v = f * rtm_dot(d, q);
    if (v < 0.0f || u + v > 1.0f) return false;
    const float k = f * rtm_dot(e2, q);
    if (!(k > 0.0000001f)) return false;
    *kout = k;
    *rank = __float_as_int(g0.w);
    return true;
}

// ---- REF traversal: MathLib.cl:234-288 + stack.cl ----
template <bool COUNT>
__device__ Hit trace_ref(const DevScene& S, rtm_f3 o, rtm_f3 d, int* __restrict__ stk, int B, Cnt& c) {
    Hit H{1000.0f, -1};
    if (COUNT) c.rays++;
    if (S.nbvh9 <= 0) return H;
    int top = 0;
    stk[0] = 0;
    while (top != -1) {
        if (COUNT) count_wave(c.wave_trav);
        const int curr = stk[top * B];
        --top;
        if (COUNT) { c.nodes++; c.boxes++; }
        const float* nd = S.bvh9 + 9 * curr;
        const float tx1 = (nd[2] - o.x) / d.x, tx2 = (nd[5] - o.x) / d.x;
        float tmin = fminf(tx1, tx2), tmax = fmaxf(tx1, tx2);
        const float ty1 = (nd[3] - o.y) / d.y, ty2 = (nd[6] - o.y) / d.y;
        tmin = fmaxf(tmin, fminf(ty1, ty2));
        tmax = fminf(tmax, fmaxf(ty1, ty2));
        const float tz1 = (nd[4] - o.z) / d.z, tz2 = (nd[7] - o.z) / d.z;
        tmin = fmaxf(tmin, fminf(tz1, tz2));
        tmax = fminf(tmax, fmaxf(tz1, tz2));
        if (tmax >= tmin) {
            const int t = (int)nd[8];
            if (t != -1) {
                if (COUNT) c.tris++;
                float k;
                int rank;
                if (mt_test(S.tri_geo, t, o, d, &k, &rank) && k < H.k && k > 0.0001f) {
                    H.k = k;
                    H.tri = t;
                }
            }
            const int L = (int)nd[0];
            if (L != -1) {
                if (top == S.ref_stack - 1) { if (COUNT) c.dropped++; }
                else stk[(++top) * B] = L;
            }
            const int R = (int)nd[1];
            if (R != -1) {
                if (top == S.ref_stack - 1) { if (COUNT) c.dropped++; }
                else stk[(++top) * B] = R;
            }
        }
    }
    return H;
}

// ---- FAST traversal ----
// Slab test of one box against a ray given as inv = 1/d: the reference's (b - o)
// scaled by 1/d instead of divided by d (MathLib.cl:167-199).
__device__ __forceinline__ void slab(float lo_x, float hi_x, float lo_y, float hi_y, float lo_z, float hi_z,
                                     rtm_f3 o, float ix, float iy, float iz, float& tmin, float& tmax) {
    const float x0 = (lo_x - o.x) * ix, x1 = (hi_x - o.x) * ix;
    const float y0 = (lo_y - o.y) * iy, y1 = (hi_y - o.y) * iy;
    const float z0 = (lo_z - o.z) * iz, z1 = (hi_z - o.z) * iz;
    tmin = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
    tmax = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
}

// A box is entered in front of the best hit: tmax >= tmin, tmax >= 0 and tmin <= cull, in one
// compare for the never-NaN slab values and cull > 0.
__device__ __forceinline__ bool box_hit(float tmin, float tmax, float cull) {
    return fmaxf(tmin, 0.0f) <= fminf(tmax, cull);
}

constexpr float CULL_MARGIN = 1.0f + 0x1p-12f;

__device__ __forceinline__ bool mt_vals(float4 g0, float4 g1, float4 g2, rtm_f3 o, rtm_f3 d, float* kout, int* rank);

// Branch-free Moller-Trumbore (same arithmetic as mt_test): all three loads are
// issued together and one predicate decides, so a wave pays one memory round trip
// and no nested divergence per triangle.
// tb + toff: the triangle's 48-byte record (toff = 48 * t, 32-bit: no 64-bit multiply in the loop).
__device__ __forceinline__ bool mt_flat(const char* __restrict__ tb, unsigned toff, rtm_f3 o, rtm_f3 d, float* kout,
                                        int* rank, int* index) {
    const float4 g0 = *reinterpret_cast<const float4*>(tb + toff);
    const float4 g1 = *reinterpret_cast<const float4*>(tb + toff + 16);
    const float4 g2 = *reinterpret_cast<const float4*>(tb + toff + 32);
    *index = __float_as_int(g1.w);   // the triangle's reference index (DevScene::tri_fast)
    return mt_vals(g0, g1, g2, o, d, kout, rank);
}

// mt_flat on a loaded record (g0 = a.p | rank, g1 = e1, g2 = e2).
// 1/a of the Moller-Trumbore test in 4 instructions instead of the IEEE division's 11: the v_rcp_f32
// seed, one Newton step in fma and v_div_fixup (infinities, NaN) give 1.0f / a bit for bit for every
// a with |a| <= 2^126 -- checked on the MI355X over all 2^32 inputs (tools/rcp_exhaustive.hip,
// profiles/r05_rcp_exhaustive.json).  Above 2^126 the reciprocal is denormal and the seed flushes it:
// the FAST path is taken only on scenes whose triangle edges keep |a| = |e1 . (d x e2)| far below
// 2^126 (rt_api.hip pack_fast; |d| = 1).  |a| < 1e-7 is the parallel case, whose 1/a is not used.
__device__ __forceinline__ float mt_recip(float a) {
    const float r = __builtin_amdgcn_rcpf(a);
    const float e = fmaf(-a, r, 1.0f);
    return __builtin_amdgcn_div_fixupf(fmaf(e, r, r), a, 1.0f);
}

// 1.0f / x for any x: mt_recip where it is the IEEE result (1e-7 <= |x| <= 2^126, profiles/
// r05_rcp_exhaustive.json), the IEEE division in a branch no lane normally takes otherwise
__device__ __forceinline__ float dev_recip(float x) {
    const float ax = fabsf(x);
    float r = mt_recip(x);
    if (__builtin_expect(!(ax >= 0.0000001f && ax <= 0x1p126f), 0)) r = 1.0f / x;
    return r;
}

// sqrtf(x) and 1.0f / sqrtf(x) (rtm_normalize's scale) in 5 and 9 instructions instead of ~16 and ~27:
// the v_rsq_f32 seed with one Newton step, then mt_recip, are bit-identical to the IEEE sqrtf and to
// 1.0f / sqrtf for every x in [2^-96, 2^126] -- checked on the MI355X over all 2^32 inputs
// (tools/sqrt_exhaustive.hip, profiles/r05_sqrt_exhaustive.json).  Outside that range (zero,
// denormals, negatives, infinities, NaN) the IEEE forms run, in a branch no lane normally takes.
__device__ __forceinline__ float sqrt_rsq(float x) {
    const float y = __builtin_amdgcn_rsqf(x);
    const float s = x * y;
    const float e = fmaf(-s, s, x);
    return fmaf(e, 0.5f * y, s);
}
__device__ __forceinline__ bool sqrt_fast_ok(float x) { return x >= 0x1p-96f && x <= 0x1p126f; }
__device__ __forceinline__ float dev_sqrt(float x) {
    float r = sqrt_rsq(x);
    if (__builtin_expect(!sqrt_fast_ok(x), 0)) r = sqrtf(x);
    return r;
}
__device__ __forceinline__ float dev_inv_sqrt(float d) {   // 1.0f / sqrtf(d), bit for bit
    float s = mt_recip(sqrt_rsq(d));
    if (__builtin_expect(!sqrt_fast_ok(d), 0)) s = 1.0f / sqrtf(d);
    return s;
}
__device__ __forceinline__ rtm_f3 dev_normalize(rtm_f3 v) {   // rtm_normalize, bit for bit
    return rtm_scale(v, dev_inv_sqrt(rtm_dot(v, v)));
}

// Moller-Trumbore on a triangle given as (a.p, e1, e2): MathLib.cl:117-160's arithmetic.
__device__ __forceinline__ bool mt_core(rtm_f3 p0, rtm_f3 e1, rtm_f3 e2, rtm_f3 o, rtm_f3 d, float* kout) {
    const rtm_f3 h = rtm_cross(d, e2);
    const float a = rtm_dot(e1, h);
    const float f = mt_recip(a);
    const rtm_f3 s = rtm_sub(o, p0);
    const float u = f * rtm_dot(s, h);
    const rtm_f3 q = rtm_cross(s, e1);
    const float v = f * rtm_dot(d, q);
    const float k = f * rtm_dot(e2, q);
    *kout = k;
    const bool parallel = a > -0.0000001f && a < 0.0000001f;
    return !parallel && !(u < 0.0f || u > 1.0f) && !(v < 0.0f || u + v > 1.0f) && (k > 0.0000001f);
}

__device__ __forceinline__ bool mt_vals(float4 g0, float4 g1, float4 g2, rtm_f3 o, rtm_f3 d, float* kout, int* rank) {
    *rank = __float_as_int(g0.w);
    return mt_core(xyz(g0), xyz(g1), xyz(g2), o, d, kout);
}

// A lane's FAST traversal stack: entries below cap bytes in LDS ([entry][blockDim]
// int2, conflict-free), deeper ones in the HBM overflow buffer ([entry][lanes]).
// off = entry index * stride (bytes of LDS between a lane's entries).
// The LDS part is addressed through an LDS-qualified pointer: the compiler then cannot merge the
// LDS and overflow branches of put/get into one generic (flat) access, which waits on both the
// vector-memory and the LDS counters
typedef char __attribute__((address_space(3))) lds_char;
typedef unsigned long long __attribute__((address_space(3))) lds_u64;
// a stack entry (ref, entry distance bits) as one 64-bit LDS word
__device__ __forceinline__ unsigned long long pack_entry(int2 e) {
    return ((unsigned long long)(unsigned)e.y << 32) | (unsigned)e.x;
}
__device__ __forceinline__ int2 unpack_entry(unsigned long long v) {
    return make_int2((int)(unsigned)v, (int)(unsigned)(v >> 32));
}
struct LaneStack {
    lds_char* lds;                   // per lane
    int2* ovf;                       // uniform base; the lane's slot is added only on the rare spill path
    unsigned stride, cap, shift, ostride;
    __device__ __forceinline__ unsigned slot(unsigned off) const {
        return ((off - cap) >> shift) * ostride + blockIdx.x * blockDim.x + threadIdx.x;
    }
    // OVF = false: the whole stack fits in LDS (stack_lds == depth) and no spill code is emitted
    template <bool OVF>
    __device__ __forceinline__ void put(unsigned off, int2 e) const {
        if (!OVF || off < cap) *(lds_u64*)(lds + off) = pack_entry(e);
        else ovf[slot(off)] = e;
    }
    template <bool OVF>
    __device__ __forceinline__ int2 get(unsigned off) const {
        int2 e;
        if (!OVF || off < cap) e = unpack_entry(*(const lds_u64*)(lds + off));
        else e = ovf[slot(off)];
        return e;
    }
    // entry `off` of the stack of the lane dl lanes away in the same wave (team walk steals).  The
    // teammate wrote it in an earlier step of this wave; the wavefront-scope acquire fence orders the read
    // after those writes (LDS and the HBM overflow part alike)
    template <bool OVF>
    __device__ __forceinline__ int2 get_lane(unsigned off, int dl) const {
        int2 e;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (!OVF || off < cap) e = unpack_entry(*(const lds_u64*)(lds + off + 8 * dl));
        else e = ovf[(unsigned)((int)slot(off) + dl)];
        return e;
    }
};

__device__ __forceinline__ LaneStack lane_stack(const DevScene& S, int* lds_base) {
    LaneStack st;
    const unsigned B = blockDim.x;
    st.lds = (lds_char*)(reinterpret_cast<char*>(lds_base)) + 8 * threadIdx.x;
    st.stride = 8u * B;
    st.cap = (unsigned)S.stack_lds * st.stride;
    st.shift = (unsigned)__builtin_ctz(st.stride);
    st.ovf = S.stack_ovf;
    st.ostride = gridDim.x * B;
    return st;
}

// One FAST BVH2 node on its loaded data: a / b = (lo.x hi.x lo.y hi.y) of child 0 / 1, z = (lo.z
// hi.z) of both, e = the child refs.  Both child boxes are tested; when both are hit the farther is
// pushed with its entry distance.  Returns the nearer hit child, or INT_MIN when none is hit (pop next).
template <bool OVF>
__device__ __forceinline__ int node_pick(float4 a, float4 b, float4 z, int2 e, rtm_f3 o, float ix, float iy,
                                         float iz, float cull, const LaneStack& st, unsigned& soff) {
    float t0n, t0x, t1n, t1x;
    slab(a.x, a.y, a.z, a.w, z.x, z.y, o, ix, iy, iz, t0n, t0x);
    slab(b.x, b.y, b.z, b.w, z.z, z.w, o, ix, iy, iz, t1n, t1x);
    const bool h0 = box_hit(t0n, t0x, cull);
    const bool h1 = box_hit(t1n, t1x, cull);
    if (h0 && h1) {
        const bool first0 = t0n <= t1n;
        st.template put<OVF>(soff, make_int2(first0 ? e.y : e.x, __float_as_int(first0 ? t1n : t0n)));
        soff += st.stride;
        return first0 ? e.x : e.y;
    }
    if (h0 || h1) return h0 ? e.x : e.y;
    return INT_MIN;
}

// node_pick on node np (AoS: 4 consecutive float4; SOA: float4 planes kstride bytes apart).
template <bool OVF>
__device__ __forceinline__ int node_step(const char* np, unsigned kstride, rtm_f3 o, float ix, float iy, float iz,
                                         float cull, const LaneStack& st, unsigned& soff) {
    const float4 a = *reinterpret_cast<const float4*>(np);
    const float4 b = *reinterpret_cast<const float4*>(np + kstride);
    const float4 z = *reinterpret_cast<const float4*>(np + 2 * kstride);
    const int2 e = *reinterpret_cast<const int2*>(np + 3 * kstride);
    return node_pick<OVF>(a, b, z, e, o, ix, iy, iz, cull, st, soff);
}

// One item per iteration: an internal node (both child boxes tested, nearer hit
// child continues, the farther is pushed with its entry distance) or a leaf
// (one triangle test).  Popped items whose entry distance is beyond the best hit
// are discarded without a fetch.  Stack entries: int2 (ref, tmin bits) in LDS.
template <bool COUNT, bool SOA, bool OVF>
__device__ Hit trace_fast(const DevScene& S, const float4* __restrict__ nodes, const float4* __restrict__ tris,
                          rtm_f3 o, rtm_f3 d, const LaneStack& st, Cnt& c) {
    Hit best{1000.0f, -1};
    int best_rank = -1;
    if (COUNT) c.rays++;
    if (S.ntri <= 0) return best;
    // Stack entries int2 (ref, tmin bits) addressed by a running byte offset (push: += stride,
    // pop: -= stride), node and triangle records by 32-bit byte offsets: the loop has no integer
    // multiplies.
    const unsigned sstride = st.stride;
    const char* const nb = reinterpret_cast<const char*>(nodes);
    const char* const tb = reinterpret_cast<const char*>(tris);
    // AoS: node i = 64 bytes at 64 i; SOA (LDS copy): plane k of node i at 16 (k nnodes + i), so
    // 16 lanes reading 16 different nodes hit 16 different bank groups
    const unsigned kstride = SOA ? 16u * (unsigned)S.nnodes : 16u;
    const float ix = dev_recip(d.x), iy = dev_recip(d.y), iz = dev_recip(d.z);
    float tmin, tmax;
    slab(S.root_box[0], S.root_box[3], S.root_box[1], S.root_box[4], S.root_box[2], S.root_box[5], o, ix, iy, iz,
         tmin, tmax);
    if (!(tmax >= tmin && tmax >= 0.0f)) return best;
    int item = S.root_ref;
    unsigned soff = 0;
    while (true) {
        if (COUNT) count_wave(c.wave_trav);
        if (item >= 0) {
            if (COUNT) { c.nodes++; c.boxes += 2; }
            const char* np = nb + (SOA ? 16u : 16u * kNodeF4) * (unsigned)item;
            const int next = node_step<OVF>(np, kstride, o, ix, iy, iz, best.k * CULL_MARGIN, st, soff);
            if (next != INT_MIN) {
                item = next;
                continue;
            }
        } else {
            if (COUNT) c.tris++;
            float k;
            int rank;
            const unsigned toff = ~(unsigned)item;   // leaf ref = ~(48 * triangle)
            int index;
            if (mt_flat(tb, toff, o, d, &k, &rank, &index) && k > 0.0001f &&
                (k < best.k || (k == best.k && rank < best_rank))) {
                best.k = k;
                best.tri = 48 * index;
                best_rank = rank;
            }
        }
        // pop the next item still in front of the best hit
        item = 0x7fffffff;
        while (soff > 0) {
            soff -= sstride;
            const int2 en = st.template get<OVF>(soff);
            if (__int_as_float(en.y) <= best.k * CULL_MARGIN) {
                item = en.x;
                break;
            }
        }
        if (item == 0x7fffffff) break;
    }
    if (best.tri >= 0) best.tri = (int)((unsigned)best.tri / 48u);
    return best;
}

// Small scenes (brute_max): every lane of the wave tests the same leaf box at the same time, its
// record read once per wave through scalar loads (SGPR operands, no LDS, no stack, no divergence).
// The set of accepted triangles is FAST's (own leaf box passes with the same slab arithmetic, MT
// hit, k > 1e-4), and records are in the reference's DFS order, so the lowest rank wins on equal
// distances: the same hit as trace_fast.
// Read-only data read through the constant address space: wave-uniform addresses become scalar
// loads (s_load_*) whatever the surrounding control flow.
typedef const float __attribute__((address_space(4))) const_f;
struct ConstF4 {
    const const_f* p;
    __device__ __forceinline__ float4 operator[](int i) const {
        return make_float4(p[4 * i], p[4 * i + 1], p[4 * i + 2], p[4 * i + 3]);
    }
};
__device__ __forceinline__ ConstF4 as_const(const float4* p) {
    return ConstF4{(const const_f*)(const float*)(p)};   // C-style: an address-space cast
}

__device__ __forceinline__ float sgpr1(float x) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}
__device__ __forceinline__ float4 sgpr4(float4 v) {
    return make_float4(sgpr1(v.x), sgpr1(v.y), sgpr1(v.z), sgpr1(v.w));
}

// Brute force with ray-triangle pair compaction.  Running the Moller-Trumbore block
// for the whole wave whenever any lane's box passes would run it for 28 of C2's 36
// triangles per ray round at ~6 passing lanes each.  The box tests stay lock-step
// (scalar records), but every passing
// (lane, triangle) pair is appended to a per-wave LDS queue; whenever the queue
// holds a full wave of pairs, each lane takes one pair -- the owner's ray from
// an LDS table, the triangle record by a vector load -- runs the same MT test
// and folds the hit into the owner's best with one 64-bit LDS atomic min on
// (distance bits, DFS position): positive float bits order like the floats, so
// the minimum key is the reference's hit (lowest rank on equal distances).
// Culling uses the owner's best as of the last batch (a conservative bound).
constexpr unsigned BRUTE_RING = 256u;
constexpr int BRUTE_WAVE_LDS = 64 * 6 * 4 + 64 * 8 + (BRUTE_RING + 64) * 4;   // ray table | best keys | pair ring + dummy slots

// Lanes of one wave hand data to each other through LDS here.  The hardware runs a
// wave's LDS instructions in order; this keeps the compiler from reordering them
// across the hand-off (it would otherwise move a lane's read of another lane's
// entry above the write it depends on).
// base + the number of bits of mask m below this lane (v_mbcnt_lo / v_mbcnt_hi: two VALU, no lane-mask
// registers)
__device__ __forceinline__ unsigned lane_prefix(unsigned long long m, unsigned base) {
    return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, base));
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Teams (ts = 2, 4 or 8 lanes per pixel, when a tile has fewer pixels than the GPU has lanes):
// the ts lanes of a team carry the same path (identical arithmetic), split the box tests between
// them (lane `sub` of the team tests records sub, sub + ts, ...; records read from the LDS copy
// at boxrec, 1 float4 per triangle, and mtrec) and share one owner slot (the team's first lane).
template <bool COUNT>
__device__ Hit trace_brute_compact(const DevScene& S, rtm_f3 o, rtm_f3 d, char* wl, const float4* mtrec,
                                   unsigned mtstride, Cnt& c, int ts = 1, const float4* boxrec = nullptr) {
    const unsigned lane = threadIdx.x & 63;
    const unsigned sub = lane & (unsigned)(ts - 1), tl = lane - sub;   // lane in team, team leader
    if (COUNT && sub == 0) c.rays++;
    const unsigned long long act = __ballot(1);
    const int nact = __popcll(act);
    const int myrank = (int)lane_prefix(act, 0u);
    float* ray = reinterpret_cast<float*>(wl);                                   // [6][64]
    unsigned long long* bestk = reinterpret_cast<unsigned long long*>(wl + 64 * 6 * 4);
    unsigned* ring = reinterpret_cast<unsigned*>(wl + 64 * 6 * 4 + 64 * 8);   // owner << 16 | triangle; [256 + lane]: dummy
    ray[0 * 64 + lane] = o.x; ray[1 * 64 + lane] = o.y; ray[2 * 64 + lane] = o.z;
    ray[3 * 64 + lane] = d.x; ray[4 * 64 + lane] = d.y; ray[5 * 64 + lane] = d.z;
    const unsigned long long nokey = ((unsigned long long)__float_as_uint(1000.0f) << 32) | 0xffffffffull;
    bestk[lane] = nokey;
    wave_lds_sync();
    const float ix = dev_recip(d.x), iy = dev_recip(d.y), iz = dev_recip(d.z);
    float bk = 1000.0f;
    unsigned head = 0, tail = 0;   // wave-uniform ring positions
    auto run_batch = [&](int n) __attribute__((always_inline)) {
        if (myrank < n) {
            const unsigned e = ring[(head + myrank) & (BRUTE_RING - 1)];
            const unsigned ow = e >> 16, q = e & 0xffffu;
            const rtm_f3 ro = rtm_v3(ray[ow], ray[64 + ow], ray[128 + ow]);
            const rtm_f3 rd = rtm_v3(ray[192 + ow], ray[256 + ow], ray[320 + ow]);
            // record q's last three float4 (hi.yz a.xy | a.z e1.xyz | e2.xyz tri): LDS copy or global
            const float4* rq = mtrec + mtstride * q;
            const float4 r1 = rq[0], r2 = rq[1], r3 = rq[2];
            const rtm_f3 a = rtm_v3(r1.z, r1.w, r2.x), e1 = rtm_v3(r2.y, r2.z, r2.w), e2 = rtm_v3(r3.x, r3.y, r3.z);
            const rtm_f3 h = rtm_cross(rd, e2);
            const float det = rtm_dot(e1, h);
            const float f = mt_recip(det);
            const rtm_f3 sv = rtm_sub(ro, a);
            const float u = f * rtm_dot(sv, h);
            const rtm_f3 qv = rtm_cross(sv, e1);
            const float v = f * rtm_dot(rd, qv);
            const float k = f * rtm_dot(e2, qv);
            const bool parallel = det > -0.0000001f && det < 0.0000001f;
            const bool hit = !parallel && !(u < 0.0f || u > 1.0f) && !(v < 0.0f || u + v > 1.0f) &&
                             (k > 0.0000001f) && k > 0.0001f && k < 1000.0f;
            if (hit) atomicMin(&bestk[ow], ((unsigned long long)__float_as_uint(k) << 32) | q);
        }
        head += n;
        wave_lds_sync();
    };
    // queue the passing (owner, triangle) pairs of records qa and qb (qb wave-uniform; < 0: none),
    // which share one leaf box; run batches while a full wave of pairs is queued.  The ring holds
    // 256 pairs: fewer than nact (<= 64) are queued before a call, which adds at most 128.
    auto enqueue = [&](bool pass, unsigned qa, int qb) __attribute__((always_inline)) {
        const unsigned long long m = __ballot(pass);
        if (m == 0) return;
        const unsigned n = (unsigned)__popcll(m);
        // no exec-mask change: a lane that does not pass writes its entries to a private dummy slot after
        // the ring (r06: the 1/8 tile 2.25 -> 2.19 ms, the whole frame unchanged)
        if (COUNT && pass) c.tris += qb >= 0 ? 2 : 1;
        const unsigned r = lane_prefix(m, tail);
        ring[pass ? (r & (BRUTE_RING - 1)) : BRUTE_RING + lane] = (tl << 16) | qa;
        if (qb >= 0) ring[pass ? ((r + n) & (BRUTE_RING - 1)) : BRUTE_RING + lane] = (tl << 16) | (unsigned)qb;
        tail += qb >= 0 ? 2 * n : n;
        wave_lds_sync();
        if ((int)(tail - head) >= nact) {
            do run_batch(nact); while ((int)(tail - head) >= nact);
            bk = __uint_as_float((unsigned)(bestk[tl] >> 32));
        }
    };
    if (ts == 1) {
        // kBoxGroup distinct leaf boxes per scalar wait: the group is loaded together (2 float4 per box:
        // the box and its one or two records; padded with never-hit boxes), all its slab tests run back
        // to back, then the passes are queued (culling uses the best hit as of the group's start:
        // conservative)
        const ConstF4 cb = as_const(S.brute_box);
        for (int g0 = 0; g0 < S.nbox; g0 += kBoxGroup) {
            float4 bx[2 * kBoxGroup];
#pragma unroll
            for (int j = 0; j < 2 * kBoxGroup; ++j) bx[j] = sgpr4(cb[2 * g0 + j]);
            const float cull = bk * CULL_MARGIN;
            bool pass[kBoxGroup];
#pragma unroll
            for (int j = 0; j < kBoxGroup; ++j) {
                float tn, tx;
                slab(bx[2 * j].x, bx[2 * j].y, bx[2 * j].z, bx[2 * j].w, bx[2 * j + 1].x, bx[2 * j + 1].y, o, ix, iy,
                     iz, tn, tx);
                pass[j] = box_hit(tn, tx, cull);
            }
#pragma unroll
            for (int j = 0; j < kBoxGroup; ++j) {
                // padding boxes (a point at 1e30: every slab distance is beyond the cull or behind the ray) never
                // pass, so the product build queues nothing for them without a check (r06: the 1/8 tile 2.19 ->
                // 2.16 ms, the frame unchanged); the instrumented build skips them so the counters stay exact
                if (COUNT && g0 + j >= S.nbox) break;
                const int qa = __float_as_int(bx[2 * j + 1].z), qb = __float_as_int(bx[2 * j + 1].w);
                if (COUNT) {   // counted per record (one leaf box test each, as in the tree walk)
                    c.boxes++;
                    count_wave(c.wave_trav); c.nodes++;
                    if (qb >= 0) { count_wave(c.wave_trav); c.nodes++; }
                }
                enqueue(pass[j], (unsigned)qa, qb);
            }
        }
    } else {
        // box g = gg * ts + sub of each round (LDS copy of brute_box at boxrec); its second record, when
        // there is one, differs between the lanes of the wave: queued by a second call
        const int rounds = (S.nbox + ts - 1) / ts;
        for (int gg = 0; gg < rounds; ++gg) {
            if (COUNT) { count_wave(c.wave_trav); count_wave(c.wave_trav); }
            const int g = gg * ts + (int)sub;
            bool pass = false;
            int qa = 0, qb = -1;
            if (g < S.nbox) {
                const float4 b0 = boxrec[2 * g], b1 = boxrec[2 * g + 1];
                float tn, tx;
                slab(b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, o, ix, iy, iz, tn, tx);
                pass = box_hit(tn, tx, bk * CULL_MARGIN);
                qa = __float_as_int(b1.z);
                qb = __float_as_int(b1.w);
                if (COUNT) { c.nodes += qb >= 0 ? 2 : 1; c.boxes++; }
            }
            enqueue(pass, (unsigned)qa, -1);
            enqueue(pass && qb >= 0, (unsigned)qb, -1);
        }
    }
    while (tail != head) run_batch(min((int)(tail - head), nact));
    const unsigned long long key = bestk[tl];
    Hit best{1000.0f, -1};
    if (key != nokey) {
        best.k = __uint_as_float((unsigned)(key >> 32));
        // triangle index: the record's last float4 (read from the LDS copy when it is staged)
        best.tri = __float_as_int(mtrec[mtstride * (unsigned)(key & 0xffffffffu) + 2].w);
    }
    return best;
}

// stk/B: the REF traversal's int stack in LDS; st: the FAST traversal's stack.
// mtrec/mtstride: where the brute-force MT batches read triangle records (float4 units).
// BLDS: the caller staged the MT records in LDS at mtrec (3 float4 per triangle); otherwise they
// are read from the global brute-force records.
template <int TRAV, bool COUNT, bool SOA = false, bool OVF = false, bool BLDS = false>
__device__ __forceinline__ Hit trace(const DevScene& S, const float4* nodes, const float4* tris, rtm_f3 o, rtm_f3 d,
                                     int* stk, int B, const LaneStack& st, Cnt& c, const float4* mtrec = nullptr,
                                     int ts = 1, const float4* boxrec = nullptr) {
    if (TRAV == TRAV_REF) return trace_ref<COUNT>(S, o, d, stk, B, c);
    if (S.nbrute > 0)
        return trace_brute_compact<COUNT>(S, o, d, reinterpret_cast<char*>(stk - threadIdx.x) +
                                                        (threadIdx.x >> 6) * BRUTE_WAVE_LDS,
                                          BLDS ? mtrec : S.brute + 1, BLDS ? 3u : 4u, c, BLDS ? ts : 1, boxrec);
    return trace_fast<COUNT, SOA, OVF>(S, nodes, tris, o, d, st, c);
}

// ---- per-launch constants (Raytracing.cl:18-37, 115-118; MathLib.cl:72-80) ----
// Every rotation whose angle and axis do not depend on the pixel is prepared
// once per thread with rtm_rot_prepare, then applied with rtm_rot_apply: the
// same arithmetic as the reference's rotateVec, done once instead of per call.
struct LaunchConst {
    rtm_rot cam_rx, cam_ry, cam_rz;   // genCameraRay rotations
    rtm_rot ibl_x, ibl_y;             // SampleSphericalMap's 90 degree rotations
    rtm_f3 focal, position, sun;      // camera focal point and origin, unnormalised sun vector
    float pas;                        // 1.0 / cam[6]
};

// evaluated once per launch on the device (make_const_kernel); rtm.h makes it bit-identical to a host
// evaluation
__host__ __device__ inline LaunchConst make_const(const FrameParams& F) {
    LaunchConst c;
    const float* cam = F.cam;
    c.focal = rtm_v3(cam[0], cam[1] - (1.0f / (2.0f * rtm_tan(cam[9] / 2.0f))), cam[2]);
    c.position = rtm_v3(cam[0], cam[1], cam[2]);
    c.pas = 1.0f / cam[6];
    c.cam_rx = rtm_rot_prepare(cam[3] * (3.14f / 180.0f), rtm_v3(1, 0, 0));
    c.cam_ry = rtm_rot_prepare(cam[4] * (3.14f / 180.0f), rtm_v3(0, 1, 0));
    c.cam_rz = rtm_rot_prepare(cam[5] * (3.14f / 180.0f), rtm_v3(0, 0, 1));
    c.ibl_x = rtm_rot_prepare(90.0f * (3.14f / 180.0f), rtm_v3(1, 0, 0));
    c.ibl_y = rtm_rot_prepare(90.0f * (3.14f / 180.0f), rtm_v3(0, 1, 0));
    rtm_f3 sun = rtm_v3(1, 1, 1);
    sun = rtm_rotate(F.env[0] * (3.14f / 180.0f), rtm_v3(1, 0, 0), sun);
    sun = rtm_rotate(F.env[1] * (3.14f / 180.0f), rtm_v3(0, 1, 0), sun);
    sun = rtm_rotate(F.env[2] * (3.14f / 180.0f), rtm_v3(0, 0, 1), sun);
    c.sun = sun;
    return c;
}

__global__ void make_const_kernel(FrameParams F, LaunchConst* __restrict__ out) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *out = make_const(F);
}

// ---- camera ray direction, Raytracing.cl:18-37 ----
__device__ __forceinline__ rtm_f3 camera_dir(const LaunchConst& C, int W, int i) {
    const int pixelY = (i + 1) % W;
    const int pixelX = (i - pixelY) / W;
    const rtm_f3 pc = rtm_v3(fmaf((float)pixelY, C.pas, -0.5f), 0.0f, fmaf(-(float)pixelX, C.pas, 0.5f));
    rtm_f3 d = dev_normalize(rtm_sub(rtm_add(C.position, pc), C.focal));
    d = rtm_rot_apply(C.cam_rx, d);
    d = rtm_rot_apply(C.cam_ry, d);
    return rtm_rot_apply(C.cam_rz, d);
}

// ---- IBL, MathLib.cl:72-90 (integer coords through a linear sampler) ----
// The 2x2 texel sums, per clamped coordinate (X, Y) of sample_ibl: X = 0 -> texels (0, 0); 0 < X < W -> (X - 1, X);
// X = W -> (W - 1, W - 1) (and likewise Y), exactly the clamps of the lookup below
__global__ void ibl_sum_kernel(const uchar4* __restrict__ rgba, int w, int h, uint32_t* __restrict__ sum) {
    const int64_t n = (int64_t)(w + 1) * (h + 1);
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
        const int X = (int)(q % (w + 1)), Y = (int)(q / (w + 1));
        const int x0 = max(min(X - 1, w - 1), 0), x1 = min(X, w - 1);
        const int y0 = max(min(Y - 1, h - 1), 0), y1 = min(Y, h - 1);
        const uchar4 t00 = rgba[(int64_t)y0 * w + x0], t10 = rgba[(int64_t)y0 * w + x1];
        const uchar4 t01 = rgba[(int64_t)y1 * w + x0], t11 = rgba[(int64_t)y1 * w + x1];
        const uint32_t r = (uint32_t)t00.x + t10.x + t01.x + t11.x;
        const uint32_t g = (uint32_t)t00.y + t10.y + t01.y + t11.y;
        const uint32_t b = (uint32_t)t00.z + t10.z + t01.z + t11.z;
        sum[q] = r | (g << 10) | (b << 20);
    }
}

template <bool COUNT>
__device__ rtm_f3 sample_ibl(const DevScene& S, const LaunchConst& C, rtm_f3 dir, Cnt& c) {
    if (COUNT) c.env++;
    dir = rtm_rot_apply(C.ibl_x, dir);
    dir = rtm_rot_apply(C.ibl_y, dir);
    float u = rtm_atan2(dir.z, dir.x), v = rtm_asin(dir.y);
    u = u * 0.1591f;
    v = v * 0.3183f;
    u = u + 0.5f;
    v = v + 0.5f;
    const int W = S.ibl_w, H = S.ibl_h;
    const int x = rtm_f2i(u * (float)W);
    const int y = rtm_f2i(v * (float)H);
    // the texels (x0, y0) .. (x1, y1) = (clamp(x - 1), clamp(y - 1)) .. (clamp(x), clamp(y)) depend on x and y
    // only through X = clamp(x, 0, W), Y = clamp(y, 0, H): their integer channel sums are one precomputed
    // word (ibl_sum_kernel), so a lookup is one 4-byte load instead of four texels from two rows
    const int X = min(max(x, 0), W), Y = min(max(y, 0), H);
    const uint32_t s4 = S.ibl_sum[(int64_t)Y * (W + 1) + X];
    const float sr = (float)(int)(s4 & 1023u);
    const float sg = (float)(int)((s4 >> 10) & 1023u);
    const float sb = (float)(int)(s4 >> 20);
    const float w = 1.0f / 1020.0f;
    return rtm_scale(rtm_v3(sr * w, sg * w, sb * w), 1.0f);
}

// IBL radiance where it can matter: every texel mean is a finite value >= 0, so
// with IBL_Power == 0 (C1/C2) the reference's IBL(dir) * IBL_Power is exactly
// 0 * IBL_Power for any dir, and the lookup is skipped.
template <bool COUNT>
__device__ __forceinline__ rtm_f3 sample_ibl_if(const DevScene& S, const LaunchConst& C, rtm_f3 dir, float power,
                                               Cnt& c) {
    if (power == 0.0f) return rtm_v3(0.0f, 0.0f, 0.0f);
    return sample_ibl<COUNT>(S, C, dir, c);
}

// ---- hemisphere samplers, MathLib.cl:313-366, with the triangle's frame
// (colinear flag, rotation to the normal, normalize(n)) precomputed by
// prep_frames_kernel: f0/f1 = q/qinv of the rotation, f2 = normalize(n) | colinear ----
__device__ __forceinline__ rtm_f3 hemi_cosine(rtm_f3 n, float4 f0, float4 f1, float4 f2, uint32_t* s0,
                                              uint32_t* s1, float* invPdf) {
    const float u = rtm_rand(s0, s1);
    const float theta = rtm_rand(s0, s1) * 2.0f * 3.14f;
    const float r = dev_sqrt(u);
    float st, ct;
    rtm_sincos(theta, &st, &ct);
    const rtm_f3 localV = rtm_v3(r * ct, r * st, dev_sqrt(rtm_fmax(0.0f, 1.0f - u)));
    rtm_f3 l;
    if (f2.w != 0.0f) {
        l = rtm_scale(localV, n.z);
    } else {
        rtm_rot R;
        R.q = rtm_v4(f0.x, f0.y, f0.z, f0.w);
        R.qinv = rtm_v4(f1.x, f1.y, f1.z, f1.w);
        l = dev_normalize(rtm_rot_apply(R, localV));
    }
    *invPdf = 3.14f / (rtm_fmax(rtm_dot(l, n), 0.0f));
    return l;
}

__device__ __forceinline__ rtm_f3 hemi_uniform(rtm_f3 n, float4 f0, float4 f1, float4 f2, uint32_t* s0,
                                               uint32_t* s1, float* invPdf) {
    const float phi = 2.0f * 3.14f * (rtm_rand(s0, s1));
    const float theta = rtm_acos(1.0f - (rtm_rand(s0, s1)));
    float sp, cp, sth, cth;
    rtm_sincos(phi, &sp, &cp);
    rtm_sincos(theta, &sth, &cth);
    const rtm_f3 localV = rtm_v3(cp * sth, sth * sp, cth);
    rtm_f3 w;
    if (f2.w != 0.0f) {
        w = rtm_scale(localV, n.z);
    } else {
        rtm_rot R;
        R.q = rtm_v4(f0.x, f0.y, f0.z, f0.w);
        R.qinv = rtm_v4(f1.x, f1.y, f1.z, f1.w);
        w = rtm_rot_apply(R, localV);
    }
    *invPdf = 2.0f * 3.14f;
    return w;
}

// hemi_cosine (cosine = true) and hemi_uniform in one instruction stream: a wave that shades
// diffuse and glossy bounces together runs the two draws, one sincos and the rotation once instead
// of once per branch.  Per lane the operations are those of the two samplers above, so the same bits:
// both first angles are 6.28 times one draw (cosine: theta = rb * 2 * 3.14, uniform: phi = 2 * 3.14 *
// ra) and localV.xy = A * (cos, sin) of it with A = sqrt(u) or sin(theta) (products commute exactly).
__device__ __forceinline__ rtm_f3 hemi_sample(bool cosine, rtm_f3 n, float4 f0, float4 f1, float4 f2, uint32_t* s0,
                                              uint32_t* s1, float* invPdf) {
    const float ra = rtm_rand(s0, s1);
    const float rb = rtm_rand(s0, s1);
    const float ang = cosine ? rb * 2.0f * 3.14f : 2.0f * 3.14f * ra;
    float sa, ca;
    rtm_sincos(ang, &sa, &ca);
    float A, Z;
    if (cosine) {
        A = dev_sqrt(ra);
        Z = dev_sqrt(rtm_fmax(0.0f, 1.0f - ra));
    } else {
        float sth, cth;
        rtm_sincos(rtm_acos(1.0f - rb), &sth, &cth);
        A = sth;
        Z = cth;
    }
    const rtm_f3 localV = rtm_v3(A * ca, A * sa, Z);
    rtm_f3 l;
    if (f2.w != 0.0f) {
        l = rtm_scale(localV, n.z);
    } else {
        rtm_rot R;
        R.q = rtm_v4(f0.x, f0.y, f0.z, f0.w);
        R.qinv = rtm_v4(f1.x, f1.y, f1.z, f1.w);
        l = rtm_rot_apply(R, localV);
        if (cosine) l = dev_normalize(l);
    }
    *invPdf = cosine ? 3.14f / (rtm_fmax(rtm_dot(l, n), 0.0f)) : 2.0f * 3.14f;
    return l;
}

// ---- BRDF_GGX, MathLib.cl:461-500 ----
__device__ __forceinline__ rtm_f3 brdf_ggx(rtm_f3 color, float rough, rtm_f3 v, rtm_f3 l, rtm_f3 n) {
    const rtm_f3 h = dev_normalize(rtm_add(l, v));
    const float alphaSqr = rough * rough;
    const float ndh = rtm_fmax(rtm_dot(n, h), 0.0f);
    const float dd = fmaf(ndh * ndh, alphaSqr - 1.0f, 1.0f);
    const float D = alphaSqr / (3.14f * (dd * dd));
    const float NdotV = rtm_fmax(rtm_dot(n, v), 0.0f);
    const float k = rough * sqrtf(2.0f / 3.14f);
    const float G1 = NdotV / fmaf(NdotV, 1.0f - k, k);
    const float NdotL = rtm_fmax(rtm_dot(n, l), 0.0f);
    const float G2 = NdotL / fmaf(NdotL, 1.0f - k, k);
    const float G = G1 * G2;
    const float F0 = 0.04f;
    const float om = 1.0f - rtm_fmax(rtm_dot(h, v), 0.0f);
    const float om2 = om * om;
    const float p5 = (om2 * om2) * om;
    const float F = fmaf(1.0f - F0, p5, F0);
    const float spec = (F * G * D) *
        dev_recip(rtm_fmax(4.0f * rtm_fmax(rtm_dot(v, n), 0.0f) * rtm_fmax(rtm_dot(l, n), 0.0f), 0.001f));
    rtm_f3 kd = rtm_v3(1.0f - F, 1.0f - F, 1.0f - F);
    kd = rtm_scale(kd, 1.0f - 0.5f);
    const rtm_f3 diffuse = rtm_div(rtm_mul(kd, color), 3.14f);
    return rtm_v3(diffuse.x + spec, diffuse.y + spec, diffuse.z + spec);
}

struct Mat {
    int type;
    rtm_f3 color;
    float rough;
};

// Device material rows are padded to kMatF = 8 floats (rt_internal.h DevScene::mat): two vector loads.
__device__ __forceinline__ Mat load_mat(const float* __restrict__ m, int idx) {
    const float4 a = reinterpret_cast<const float4*>(m)[2 * idx];
    const float rough = m[kMatF * idx + 4];
    Mat r;
    r.type = (int)a.x;
    r.color = rtm_v3(a.y, a.z, a.w);
    r.rough = rough;
    return r;
}

// Per-triangle hemisphere frame: the rotation rand_hemi_cosine / rand_hemi_uniform
// (MathLib.cl:325-336, 349-362) build from the hit normal, which only depends on
// the triangle.  Computed on the device with the same rtm_* arithmetic.
__global__ void prep_frames_kernel(const float4* __restrict__ tri_shade, const float* __restrict__ mat, int ntri,
                                   float4* __restrict__ frame) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntri) return;
    const float4 sh = tri_shade[t];
    const rtm_f3 n = xyz(sh);
    const int type = (int)mat[kMatF * __float_as_int(sh.w)];
    const rtm_f3 nn = dev_normalize(n);
    const float colinear = rtm_fabs(rtm_dot(nn, rtm_v3(0.0f, 0.0f, 1.0f)));
    rtm_rot R;
    R.q = rtm_v4(1, 0, 0, 0);
    R.qinv = R.q;
    if (colinear != 1.0f) {
        const float ang = rtm_acos(rtm_dot(n, rtm_v3(0, 0, 1)));
        if (type == 1) R = rtm_rot_prepare(ang, rtm_cross(rtm_v3(0, 0, 1), n));
        else if (type == 2) R = rtm_rot_prepare(ang, dev_normalize(rtm_cross(rtm_v3(0.0f, 0.0f, 1.0f), n)));
    }
    frame[3 * t + 0] = make_float4(R.q.x, R.q.y, R.q.z, R.q.w);
    frame[3 * t + 1] = make_float4(R.qinv.x, R.qinv.y, R.qinv.z, R.qinv.w);
    frame[3 * t + 2] = make_float4(nn.x, nn.y, nn.z, colinear == 1.0f ? 1.0f : 0.0f);
}

__device__ __forceinline__ void log_event(const FrameParams& F, float kind, int j, rtm_f3 o, rtm_f3 d, float k,
                                          int mat, rtm_f3 so) {
    const int n = *F.log_count;
    if (n >= F.log_cap) return;
    float* e = F.log_buf + 16 * n;
    e[0] = kind; e[1] = (float)j; e[2] = o.x; e[3] = o.y; e[4] = o.z; e[5] = d.x; e[6] = d.y; e[7] = d.z;
    e[8] = k; e[9] = (float)mat; e[10] = so.x; e[11] = so.y; e[12] = so.z; e[13] = 0; e[14] = 0; e[15] = 0;
    *F.log_count = n + 1;
}

// Mean + clamp of one pixel (Raytracing.cl:211-220).
__device__ __forceinline__ void store_pixel(float* __restrict__ out, int p, rtm_f3 acc, int spp) {
    const rtm_f3 o = rtm_div(acc, (float)spp);
    float* dst = out + 3 * (int64_t)p;
    dst[0] = rtm_fmax(rtm_fmin(o.x, 1.0f), 0.0f);
    dst[1] = rtm_fmax(rtm_fmin(o.y, 1.0f), 0.0f);
    dst[2] = rtm_fmax(rtm_fmin(o.z, 1.0f), 0.0f);
}

enum Phase { FETCH = 0, PRIMARY = 1, PREP = 2, BOUNCE = 3, SUN = 4, DONE = 5 };
// a job of sample slice k > 0 waiting for slice k - 1 of its pixel (FrameParams::slices)
constexpr int WAIT_SLICE = 7;
// words other workgroups read or write within a launch: global address space, agent-scope accesses
typedef unsigned __attribute__((address_space(1))) gu32;
typedef unsigned long long __attribute__((address_space(1))) gu64;

// ---- pixel hand-out ----
// Tile pixels are dealt in chunks of 2^kChunkShift consecutive pixels: chunk c belongs to group
// c % kGroups.  A block of group g = blockIdx.x % kGroups (under the round-robin dispatch of blocks
// over the 8 XCDs, the blocks of one XCD) takes pixels from group g's counter, one device-scope
// atomic per wave refill, so every 128-byte line of the frame is written through one XCD's L2 (a
// line written from several L2s leaves each of them as a partial write).  A group whose pixels are
// exhausted steals from the next groups in turn; `dry` remembers (per wave) which are exhausted.
// Correctness does not depend on the placement: every pixel is taken exactly once whatever XCD a
// block runs on.
struct PixelQueue {
    unsigned dry = 0;   // bit g: group g's counter is exhausted
    // FrameParams::handout = 1: group g owns the contiguous pixels [g per, (g + 1) per) of the tile instead
    // of every kGroups-th chunk, so one XCD's rays in flight come from one region of the image (the tree's
    // lines they need are fewer: the L2 of an XCD holds more of them).  0: interleaved chunks.
    unsigned per = 0;
};

// group g's j-th pixel (chunks g, g + kGroups, g + 2 kGroups, ...: increasing in j; or the j-th of its block)
__device__ __forceinline__ unsigned group_pixel(unsigned g, unsigned j, unsigned per) {
    if (per) return g * per + j;
    constexpr unsigned m = (1u << kChunkShift) - 1u;
    return (((j >> kChunkShift) * (unsigned)kGroups + g) << kChunkShift) | (j & m);
}

// pixels of group g in a tile of nloc pixels (wave-uniform)
__device__ __forceinline__ unsigned group_pixels(unsigned g, unsigned nloc, unsigned per) {
    if (per) return g * per >= nloc ? 0u : min(per, nloc - g * per);
    const unsigned chunks = nloc >> kChunkShift, rem = nloc & ((1u << kChunkShift) - 1u);
    const unsigned full = chunks > g ? (chunks - 1u - g) / (unsigned)kGroups + 1u : 0u;
    return (full << kChunkShift) + (chunks % (unsigned)kGroups == g ? rem : 0u);
}

// need: wave-uniform mask of the requesting lanes (team leaders); lane0: the calling lane's team
// leader.  Returns the calling lane's tile pixel index (>= nloc: none left in the tile).  Called
// with the whole wave active; all control flow is wave-uniform, and the requests are served in
// rank order (group by group), so a lane only needs its rank.
// slices > 1 (FrameParams::slices): a group hands out `slices` passes over its pixels, slice-major --
// the job after its pixels' slice k is their slice k + 1 -- and the return value is the job
// k * nloc + pixel (>= slices * nloc: none left).
__device__ __forceinline__ unsigned take_pixel(PixelQueue& Q, unsigned long long need, int lane0,
                                               unsigned* __restrict__ counters, unsigned nloc, int lane,
                                               unsigned slices = 1) {
    const bool mine = (need >> lane0) & 1ull;
    const unsigned rank = (unsigned)__popcll(need & ((1ull << lane0) - 1ull));
    const unsigned total = (unsigned)__popcll(need);
    const int leader = __ffsll((long long)need) - 1;
    unsigned q = nloc * slices;
    unsigned base = 0;   // requests served so far
    unsigned g = blockIdx.x % (unsigned)kGroups;
    for (int t = 0; t < kGroups && base < total; ++t, g = (g + 1u) % (unsigned)kGroups) {
        if ((Q.dry >> g) & 1u) continue;
        const unsigned k = total - base;
        unsigned got = 0;
        if (lane == leader) got = atomicAdd(counters + g * (unsigned)(kCounterStride / 4), k);
        const unsigned j0 = (unsigned)__builtin_amdgcn_readfirstlane((int)__shfl(got, leader, 64));
        const unsigned px = group_pixels(g, nloc, Q.per);
        const unsigned have = px * slices;
        const unsigned nok = j0 < have ? min(have - j0, k) : 0u;
        if (mine && rank >= base && rank < base + nok) {
            const unsigned jj = j0 + (rank - base);
            q = slices == 1 ? group_pixel(g, jj, Q.per) : (jj / px) * nloc + group_pixel(g, jj % px, Q.per);
        }
        if (nok < k) Q.dry |= 1u << g;   // the group's sequence has run past the tile
        base += nok;
    }
    return q;
}

// ---- resumable FAST traversal (option "resume_min") ----
// On deep scenes a wave's traversal loop runs until its slowest ray is done
// (SIMD efficiency 13 % on C3/C4).  Here each lane keeps its traversal state in
// registers across render-loop iterations: the wave runs traversal rounds only
// until at least F.resume_min lanes have no ray in flight, then those lanes shade
// and start their next ray while the others continue where they stopped.
struct FastRay {
    rtm_f3 o, d;
    float ix, iy, iz;
    int item;
    unsigned soff;    // stack top, bytes
    float bk;         // best distance
    int bt;           // best triangle's reference index (BVH2 walks; 48 x it on the 4-wide walk), -1 = none
    int brank;        // its rank in the reference DFS order
    bool any;         // any hit ends the ray (a shadow ray whose hit only matters as hit / miss)
};

// Returns true when the ray is already finished (no triangles / root box missed).
template <bool COUNT>
__device__ __forceinline__ bool fast_init(const DevScene& S, FastRay& R, rtm_f3 o, rtm_f3 d, Cnt& c) {
    if (COUNT) c.rays++;
    R.o = o;
    R.d = d;
    R.bk = 1000.0f;
    R.bt = -1;
    R.brank = -1;
    R.soff = 0;
    if (S.ntri <= 0) return true;
    R.ix = dev_recip(d.x);
    R.iy = dev_recip(d.y);
    R.iz = dev_recip(d.z);
    float tmin, tmax;
    slab(S.root_box[0], S.root_box[3], S.root_box[1], S.root_box[4], S.root_box[2], S.root_box[5], o, R.ix, R.iy, R.iz,
         tmin, tmax);
    if (!(tmax >= tmin && tmax >= 0.0f)) return true;
    R.item = S.root_ref;
    return false;
}

// One round of trace_fast's loop: descend nearest children until a leaf is
// tested or nothing is hit, then pop the next live stack entry.  Same
// arithmetic and order as trace_fast.  Returns true when the ray is finished.
template <bool COUNT, bool SOA, bool OVF>
__device__ __forceinline__ bool fast_round(const DevScene& S, FastRay& R, const char* nb, const char* tb,
                                           const LaneStack& st, unsigned kstride, Cnt& c) {
    const unsigned sstride = st.stride;
    while (R.item >= 0) {
        if (COUNT) { count_wave(c.wave_trav); c.nodes++; c.boxes += 2; }
        const char* np = nb + (SOA ? 16u : 16u * kNodeF4) * (unsigned)R.item;
        R.item = node_step<OVF>(np, kstride, R.o, R.ix, R.iy, R.iz, R.bk * CULL_MARGIN, st, R.soff);
    }
    if (R.item != INT_MIN) {      // a leaf: one triangle test
        if (COUNT) { count_wave(c.wave_trav); c.tris++; }
        float k;
        int rank;
        const unsigned toff = ~(unsigned)R.item;
        int index;
        if (mt_flat(tb, toff, R.o, R.d, &k, &rank, &index) && k > 0.0001f &&
            (k < R.bk || (k == R.bk && rank < R.brank))) {
            R.bk = k;
            R.bt = index;
            R.brank = rank;
            if (R.any) return true;
        }
    }
    while (R.soff > 0) {   // pop the next item still in front of the best hit
        R.soff -= sstride;
        const int2 en = st.template get<OVF>(R.soff);
        if (__int_as_float(en.y) <= R.bk * CULL_MARGIN) {
            R.item = en.x;
            return false;
        }
    }
    return true;
}

// The fourth load of an item step reads a node's child refs, and for a leaf the last 8 bytes of its
// record (e2.z and the pad), whose e2.z the leaf test takes from it: both kinds of lanes then use the
// load, so the compiler issues it with the other three before the node / leaf branch instead of
// sinking it into the node branch, where a wave holding both kinds waited for it after the leaf code
// (a second memory round trip per step).
constexpr unsigned kLeafTail = 40u;
__device__ __forceinline__ float4 leaf_e2(float4 g2, int2 tail) {
    return make_float4(g2.x, g2.y, __int_as_float(tail.x), g2.w);
}

// One item of trace_fast's loop per call: an internal node or a leaf, then a pop when the item
// yields no next item.  The per-lane sequence of node steps, leaf tests and pops is trace_fast's, so
// the hit is the same.  Every tracing lane fetches its item with the SAME four vector loads, whether
// it is a node (64 B: both child boxes + refs) or a triangle (48 B: a.p | rank, e1, e2; the fourth
// load re-reads its first bytes), so a wave issues 4 load instructions per step with all its
// tracing lanes active.  On C3 the texture address unit was 89 % busy with the descend-until-leaf
// rounds of fast_round, whose loads ran with few lanes active.  Returns true when the ray is finished.
template <bool COUNT, bool SOA, bool OVF>
__device__ __forceinline__ bool fast_step(const DevScene& S, FastRay& R, const char* nb, const char* tb,
                                          const LaneStack& st, unsigned kstride, Cnt& c) {
    const bool node = R.item >= 0;
    const char* p = node ? nb + (SOA ? 16u : 16u * kNodeF4) * (unsigned)R.item : tb + ~(unsigned)R.item;
    const unsigned ks = node ? kstride : 16u;
    const float4 g0 = *reinterpret_cast<const float4*>(p);
    const float4 g1 = *reinterpret_cast<const float4*>(p + ks);
    const float4 g2 = *reinterpret_cast<const float4*>(p + 2 * ks);
    const int2 e = *reinterpret_cast<const int2*>(p + (node ? 3 * ks : kLeafTail));
    if (COUNT) count_wave(c.wave_trav);
    // Both tests on every lane's item, outcomes by selects: a wave's step almost always holds node
    // and leaf lanes together (C3: ~20 % of the items are leaves, ~40 lanes trace), so both codes run
    // anyway; in one basic block the compiler can sink no load into one kind's branch.  The node
    // arithmetic on a leaf record and the Moller-Trumbore arithmetic on a node record are discarded.
    const float cull = R.bk * CULL_MARGIN;
    float t0n, t0x, t1n, t1x;
    slab(g0.x, g0.y, g0.z, g0.w, g2.x, g2.y, R.o, R.ix, R.iy, R.iz, t0n, t0x);
    slab(g1.x, g1.y, g1.z, g1.w, g2.z, g2.w, R.o, R.ix, R.iy, R.iz, t1n, t1x);
    const bool h0 = node && box_hit(t0n, t0x, cull), h1 = node && box_hit(t1n, t1x, cull);
    float k;
    int rank;
    const bool mt = mt_vals(g0, g1, leaf_e2(g2, e), R.o, R.d, &k, &rank);
    // bitwise, not short-circuit: the compiler keeps && / || here as nested exec-mask branches (~14 SALU
    // per step on the wave's own issue slots)
    const bool take = (!node) & mt & (k > 0.0001f) & ((k < R.bk) | ((k == R.bk) & (rank < R.brank)));
    if (COUNT) {
        if (node) { c.nodes++; c.boxes += 2; }
        else c.tris++;
    }
    R.bk = take ? k : R.bk;
    R.bt = take ? __float_as_int(g1.w) : R.bt;   // e1.w: the triangle's reference index
    R.brank = take ? rank : R.brank;
    const bool first0 = t0n <= t1n;
    if (h0 && h1) {   // the farther child waits on the stack
        st.template put<OVF>(R.soff, make_int2(first0 ? e.y : e.x, __float_as_int(first0 ? t1n : t0n)));
        R.soff += st.stride;
    }
    const int next = (h0 && h1) ? (first0 ? e.x : e.y) : h0 ? e.x : h1 ? e.y : INT_MIN;
    if (take && R.any) return true;
    if (next != INT_MIN) {
        R.item = next;
        return false;
    }
    while (R.soff > 0) {   // pop the next item still in front of the best hit
        R.soff -= st.stride;
        const int2 en = st.template get<OVF>(R.soff);
        if (__int_as_float(en.y) <= R.bk * CULL_MARGIN) {
            R.item = en.x;
            return false;
        }
    }
    return true;
}

// ---- software-pipelined item step (render_resume_kernel's BVH2 walk with one lane per ray) ----
// fast_step with the next item's four loads issued before this item's leaf test: the node test and
// the pop (culled against the best hit as it was before this step's leaf test -- a conservative cull:
// an entry the new best would cull is fetched and its children culled one step later) decide the next
// item, its loads go out, and the Moller-Trumbore arithmetic of the current item runs while they are
// in flight.  The accepted triangles are fast_step's (the acceptance test is unchanged), so the hit is.
struct ItemData {
    float4 g0, g1, g2;
    int2 e;
};
template <bool SOA>
__device__ __forceinline__ ItemData item_fetch(int item, const char* nb, const char* tb, unsigned kstride) {
    const bool node = item >= 0;
    const char* p = node ? nb + (SOA ? 16u : 16u * kNodeF4) * (unsigned)item : tb + ~(unsigned)item;
    const unsigned ks = node ? kstride : 16u;
    ItemData D;
    D.g0 = *reinterpret_cast<const float4*>(p);
    D.g1 = *reinterpret_cast<const float4*>(p + ks);
    D.g2 = *reinterpret_cast<const float4*>(p + 2 * ks);
    D.e = *reinterpret_cast<const int2*>(p + (node ? 3 * ks : kLeafTail));
    return D;
}
template <bool COUNT, bool SOA, bool OVF>
__device__ __forceinline__ bool fast_step_pipe(FastRay& R, ItemData& D, const char* nb, const char* tb,
                                               const LaneStack& st, unsigned kstride, Cnt& c) {
    const bool node = R.item >= 0;
    const float4 g0 = D.g0, g1 = D.g1, g2 = D.g2;
    const int2 e = D.e;
    if (COUNT) count_wave(c.wave_trav);
    const float cull = R.bk * CULL_MARGIN;
    float t0n, t0x, t1n, t1x;
    slab(g0.x, g0.y, g0.z, g0.w, g2.x, g2.y, R.o, R.ix, R.iy, R.iz, t0n, t0x);
    slab(g1.x, g1.y, g1.z, g1.w, g2.z, g2.w, R.o, R.ix, R.iy, R.iz, t1n, t1x);
    const bool h0 = node && box_hit(t0n, t0x, cull), h1 = node && box_hit(t1n, t1x, cull);
    const bool first0 = t0n <= t1n;
    if (h0 && h1) {
        st.template put<OVF>(R.soff, make_int2(first0 ? e.y : e.x, __float_as_int(first0 ? t1n : t0n)));
        R.soff += st.stride;
    }
    int next = (h0 && h1) ? (first0 ? e.x : e.y) : h0 ? e.x : h1 ? e.y : INT_MIN;
    while (next == INT_MIN && R.soff > 0) {
        R.soff -= st.stride;
        const int2 en = st.template get<OVF>(R.soff);
        if (__int_as_float(en.y) <= cull) next = en.x;
    }
    const bool done = next == INT_MIN;
    if (!done) D = item_fetch<SOA>(next, nb, tb, kstride);
    float k;
    int rank;
    const bool mt = mt_vals(g0, g1, leaf_e2(g2, e), R.o, R.d, &k, &rank);
    const bool take = (!node) & mt & (k > 0.0001f) & ((k < R.bk) | ((k == R.bk) & (rank < R.brank)));
    if (COUNT) {
        if (node) { c.nodes++; c.boxes += 2; }
        else c.tris++;
    }
    R.bk = take ? k : R.bk;
    R.bt = take ? __float_as_int(g1.w) : R.bt;
    R.brank = take ? rank : R.brank;
    R.item = done ? R.item : next;
    return done | (take & R.any);
}

// ---- top levels of the BVH2 tree from scalar loads (RT_TOP_LEVELS = 1: the root; 2: and its children) ----
// The first node steps of a ray that has just started at the root run here for every such lane of
// the wave at once, with the node read through scalar loads (one record per wave, SGPR operands,
// no vector memory instruction): the root, then (RT_TOP_LEVELS = 2) each of its two internal
// children for the lanes whose walk continues into it.  The arithmetic, push order and cull are
// fast_step_pipe's node part, so the walk that follows is the one the item steps would have made.
// Returns false when the ray is finished (every box missed).  r06 (profiles/r06_ab_top_levels_ta.json):
// the root alone C3 107.4 / 107.3 -> 107.1 / 106.6 ms, C4 272.2 / 269.6 -> 270.1 / 267.4 ms (kept); with
// its children vector-memory reads -5.4 % (C3) / -1.8 % (C4) but C3 108.8-109.1 ms, C4 270.8-273.4 ms.
#ifndef RT_TOP_LEVELS
#define RT_TOP_LEVELS 1
#endif
template <bool COUNT, bool OVF>
__device__ __forceinline__ void top_node_step(const const_f* n, bool on, FastRay& R, const LaneStack& st,
                                              int& next, Cnt& c) {
    const float4 g0 = sgpr4(make_float4(n[0], n[1], n[2], n[3]));
    const float4 g1 = sgpr4(make_float4(n[4], n[5], n[6], n[7]));
    const float4 g2 = sgpr4(make_float4(n[8], n[9], n[10], n[11]));
    const int ex = __builtin_amdgcn_readfirstlane(__float_as_int(n[12]));
    const int ey = __builtin_amdgcn_readfirstlane(__float_as_int(n[13]));
    if (!on) return;
    if (COUNT) { count_wave(c.wave_trav); c.nodes++; c.boxes += 2; }
    const float cull = R.bk * CULL_MARGIN;
    float t0n, t0x, t1n, t1x;
    slab(g0.x, g0.y, g0.z, g0.w, g2.x, g2.y, R.o, R.ix, R.iy, R.iz, t0n, t0x);
    slab(g1.x, g1.y, g1.z, g1.w, g2.z, g2.w, R.o, R.ix, R.iy, R.iz, t1n, t1x);
    const bool h0 = box_hit(t0n, t0x, cull), h1 = box_hit(t1n, t1x, cull);
    const bool first0 = t0n <= t1n;
    if (h0 && h1) {
        st.template put<OVF>(R.soff, make_int2(first0 ? ey : ex, __float_as_int(first0 ? t1n : t0n)));
        R.soff += st.stride;
    }
    next = (h0 && h1) ? (first0 ? ex : ey) : h0 ? ex : h1 ? ey : INT_MIN;
    if (next == INT_MIN) {   // the pop of fast_step_pipe (cull as of this step)
        while (R.soff > 0) {
            R.soff -= st.stride;
            const int2 en = st.template get<OVF>(R.soff);
            if (__int_as_float(en.y) <= cull) { next = en.x; break; }
        }
    }
}
// nb: the AoS node array (global memory); fresh: this lane's ray starts at the root this round
template <bool COUNT, bool OVF>
__device__ __forceinline__ bool top_levels(const DevScene& S, FastRay& R, bool fresh, const char* nb,
                                           const LaneStack& st, Cnt& c) {
    const int root = S.root_ref;
    int next = R.item;
    const const_f* cn = (const const_f*)(const float*)nb;
    top_node_step<COUNT, OVF>(cn + 16 * root, fresh, R, st, next, c);
    // the root's two children, each for the lanes whose walk went on into it
    const int ex = __builtin_amdgcn_readfirstlane(__float_as_int(cn[16 * root + 12]));
    const int ey = __builtin_amdgcn_readfirstlane(__float_as_int(cn[16 * root + 13]));
    const bool on_x = fresh && ex >= 0 && next == ex, on_y = fresh && ey >= 0 && next == ey;
    if (RT_TOP_LEVELS >= 2) {
        if (ex >= 0 && __ballot(on_x)) top_node_step<COUNT, OVF>(cn + 16 * ex, on_x, R, st, next, c);
        if (ey >= 0 && __ballot(on_y)) top_node_step<COUNT, OVF>(cn + 16 * ey, on_y, R, st, next, c);
    }
    if (!fresh) return true;
    R.item = next;
    return next != INT_MIN;
}

// ---- team traversal: TS lanes walk one ray (tiles with about one pixel per lane, option "walk_team") ----
// When a tile has no more pixels than the device has lanes, a frame lasts as long as its slowest
// pixel's chain of samples, and a chain advances one dependent node fetch per step.
// Here TS consecutive lanes (a team, TS = 2, 4 or 8, aligned) carry the same pixel with
// identical shading arithmetic and split each ray's tree walk: every lane runs trace_fast's
// closest-first descent on its own LDS stack, and a lane whose stack runs dry steals the BOTTOM
// entry (the shallowest: the largest untested subtree) of a teammate's stack.  A lane's stack top
// evolves exactly as in a one-lane walk started at the subtree it took, so it never holds more than
// DevScene::depth entries; steals only remove entries from the bottom.  The team's best hit (k, rank,
// triangle) is reduced across the team (DPP within the quad) in every step where a lane improved it,
// so culling uses the team's best (DPP: quad xors, then the half-row mirror for 8).  The hit is the minimum (k, rank) over accepted triangles, which
// no traversal order changes (every ancestor box is a union of leaf boxes): the frame is the one-lane
// walk's, bit for bit.
constexpr int NO_ITEM = INT_MIN;

// One DPP move: M = 1 / 2: lane ^ M within the quad; M = 4: row_half_mirror (lane i <-> 7 - i within
// 8 lanes), which pairs every lane with one of the other quad of its 8-lane team
template <int M>
__device__ __forceinline__ int quad_xor(int x) {
    return __builtin_amdgcn_update_dpp(0, x, M == 1 ? 0xB1 : M == 2 ? 0x4E : 0x141, 0xF, 0xF, false);
}

// the r-th set bit (r < popcount) of a team mask (shifted to bit 0)
__device__ __forceinline__ int nth_bit4(unsigned m, unsigned r) {
    for (unsigned k = 0; k < r; ++k) m &= m - 1u;
    return __builtin_ctz(m);
}

// One step of a team's walk over the BVH2 item layout (fast_step's loads and arithmetic).  R.item is
// the lane's own item (NO_ITEM: none), R.soff its stack top and boff its stack bottom (bytes).  ts:
// lanes per team (2, 4, 8; wave-uniform).  Returns true (for every lane of the team) when the team's
// ray is finished.
template <bool COUNT, bool SOA, bool OVF>
__device__ __forceinline__ bool team_step(int ts, FastRay& R, unsigned& boff, const char* nb, const char* tb,
                                          const LaneStack& st, unsigned kstride, Cnt& c) {
    const unsigned lane = threadIdx.x & 63u;
    const unsigned tbase = lane & ~(unsigned)(ts - 1);
    const unsigned sub = lane - tbase;
    const unsigned tm = (1u << ts) - 1u;
    // 1. a lane without an item pops its own stack (entries behind the team's best are discarded)
    if (R.item == NO_ITEM) {
        while (R.soff > boff) {
            R.soff -= st.stride;
            const int2 en = st.template get<OVF>(R.soff);
            if (__int_as_float(en.y) <= R.bk * CULL_MARGIN) {
                R.item = en.x;
                break;
            }
        }
        if (R.soff == boff) R.soff = boff = 0u;   // drained: the next subtree starts a fresh stack
    }
    // 2. lanes still without an item steal the bottom entry of teammates with a non-empty stack
    const unsigned idle = (unsigned)(__ballot(R.item == NO_ITEM) >> tbase) & tm;
    const unsigned vict = (unsigned)(__ballot(R.soff > boff) >> tbase) & tm;
    if (idle && vict) {
        const unsigned nth = (unsigned)__popc(idle), nv = (unsigned)__popc(vict);
        const unsigned below = (1u << sub) - 1u;
        const bool thief = ((idle >> sub) & 1u) && (unsigned)__popc(idle & below) < nv;
        const bool robbed = ((vict >> sub) & 1u) && (unsigned)__popc(vict & below) < nth;
        const int v = thief ? (int)tbase + nth_bit4(vict, (unsigned)__popc(idle & below)) : (int)lane;
        const unsigned vb = (unsigned)__shfl((int)boff, v, 64);
        if (thief) {
            const int2 en = st.template get_lane<OVF>(vb, v - (int)lane);
            if (__int_as_float(en.y) <= R.bk * CULL_MARGIN) R.item = en.x;
        }
        if (robbed) boff += st.stride;
    }
    // 3. every lane with an item processes it (fast_step)
    bool improved = false;
    if (R.item != NO_ITEM) {
        const bool node = R.item >= 0;
        const char* p = node ? nb + (SOA ? 16u : 16u * kNodeF4) * (unsigned)R.item : tb + ~(unsigned)R.item;
        const unsigned ks = node ? kstride : 16u;
        const float4 g0 = *reinterpret_cast<const float4*>(p);
        const float4 g1 = *reinterpret_cast<const float4*>(p + ks);
        const float4 g2 = *reinterpret_cast<const float4*>(p + 2 * ks);
        const int2 e = *reinterpret_cast<const int2*>(p + (node ? 3 * ks : kLeafTail));
        // both tests, outcomes by selects (fast_step)
        const float cull = R.bk * CULL_MARGIN;
        float t0n, t0x, t1n, t1x;
        slab(g0.x, g0.y, g0.z, g0.w, g2.x, g2.y, R.o, R.ix, R.iy, R.iz, t0n, t0x);
        slab(g1.x, g1.y, g1.z, g1.w, g2.z, g2.w, R.o, R.ix, R.iy, R.iz, t1n, t1x);
        const bool h0 = node && box_hit(t0n, t0x, cull), h1 = node && box_hit(t1n, t1x, cull);
        float k;
        int rank;
        const bool mt = mt_vals(g0, g1, leaf_e2(g2, e), R.o, R.d, &k, &rank);
        improved = (!node) & mt & (k > 0.0001f) & ((k < R.bk) | ((k == R.bk) & (rank < R.brank)));
        if (COUNT) {
            if (node) { c.nodes++; c.boxes += 2; }
            else c.tris++;
        }
        R.bk = improved ? k : R.bk;
        R.bt = improved ? __float_as_int(g1.w) : R.bt;
        R.brank = improved ? rank : R.brank;
        const bool first0 = t0n <= t1n;
        if (h0 && h1) {
            st.template put<OVF>(R.soff, make_int2(first0 ? e.y : e.x, __float_as_int(first0 ? t1n : t0n)));
            R.soff += st.stride;
        }
        R.item = (h0 && h1) ? (first0 ? e.x : e.y) : h0 ? e.x : h1 ? e.y : NO_ITEM;
    }
    if (COUNT) count_wave(c.wave_trav);
    // 4. the team's best: lowest (k, rank) over the team, in every lane
    if (__ballot(improved)) {
        auto fold = [&](float ok, int orank, int obt) __attribute__((always_inline)) {
            if (ok < R.bk || (ok == R.bk && orank < R.brank)) {
                R.bk = ok;
                R.brank = orank;
                R.bt = obt;
            }
        };
        fold(__int_as_float(quad_xor<1>(__float_as_int(R.bk))), quad_xor<1>(R.brank), quad_xor<1>(R.bt));
        if (ts >= 4) fold(__int_as_float(quad_xor<2>(__float_as_int(R.bk))), quad_xor<2>(R.brank), quad_xor<2>(R.bt));
        if (ts >= 8) fold(__int_as_float(quad_xor<4>(__float_as_int(R.bk))), quad_xor<4>(R.brank), quad_xor<4>(R.bt));
        if (R.any && R.bt >= 0) return true;   // a shadow ray's hit only matters as hit / miss
    }
    // 5. finished when no lane of the team holds an item or a stack entry
    const unsigned busy = (unsigned)(__ballot(R.item != NO_ITEM || R.soff > boff) >> tbase) & tm;
    return busy == 0u;
}

// One item of the walk over the 4-wide quantised layout (DevScene::wnodes, rt_api.hip emit_wide):
// an internal node -- its up to 4 child boxes dequantised (p + q * 2^e per bound) and tested, the
// hit children sorted by entry distance, the nearest continued and the others pushed farthest first
// -- or a leaf: its exact box tested again (the quantised box is a superset) and its triangle
// intersected.  Nodes and leaves are both 64 bytes, fetched with the same four 16-byte loads, like
// fast_step.  The accepted triangles are the binary walk's (own exact leaf box passes, MT hit,
// k > 1e-4, lowest (k, rank)), so the hit is the same.  Returns true when the ray is finished.
// The wide node on its loaded data: the hit children sorted by entry distance, the others pushed
// farthest first.  Returns the nearest hit child, or INT_MIN (pop next).
// PRE0: child 0's entry distance and box test were computed by the caller (tn0, hit0: wide_step's shared
// slab), the loop tests children 1..3
template <bool COUNT, bool OVF, bool PRE0 = false, bool DQ = false>
__device__ __forceinline__ int wide_node(float4 g0, float4 g1, float4 g2, float4 g3, FastRay& R, const LaneStack& st,
                                         Cnt& c, bool on = true, float tn0 = 0.0f, bool hit0 = false) {   // on = false: no child is hit
    const float cull = R.bk * CULL_MARGIN;
    const unsigned meta = __float_as_uint(g0.w);
    const float sx = __uint_as_float((meta & 255u) << 23);
    const float sy = __uint_as_float(((meta >> 8) & 255u) << 23);
    const float sz = __uint_as_float(((meta >> 16) & 255u) << 23);
    const unsigned qlx = __float_as_uint(g2.x), qly = __float_as_uint(g2.y), qlz = __float_as_uint(g2.z);
    const unsigned qhx = __float_as_uint(g2.w), qhy = __float_as_uint(g3.x), qhz = __float_as_uint(g3.y);
    int r[4] = {__float_as_int(g1.x), __float_as_int(g1.y), __float_as_int(g1.z), __float_as_int(g1.w)};
    float t[4];
    if (PRE0) t[0] = (on && r[0] != INT_MIN && hit0) ? tn0 : INFINITY;
    // DQ (origin-folded): p - o once per node and axis, then each bound as fma(q, s, p - o) -- one
    // subtract per bound fewer.  It rounds differently from (p + q s) - o, so it is conservative only
    // because the builder keeps every bound with q > 0 at least 2^-17 P outside its child's exact
    // bound (rt_api.hip emit_wide), which exceeds the rounding of the two forms, 2^-24 (|p - o| +
    // |p + q s - o| + |b - o|) for a leaf bound b below, for every ray origin up to DevScene::wdq_omax
    // (~20 P): a child box never rejects what a leaf below it accepts; q = 0 is fl(p - o) in both
    // forms.  launch_fast picks DQ per frame (hit points are within P; the camera is checked).
    const float px = g0.x - R.o.x, py = g0.y - R.o.y, pz = g0.z - R.o.z;
#pragma unroll
    for (int i = PRE0 ? 1 : 0; i < 4; ++i) {
        // p + q * s with q * s exact (s a power of two, q < 256): one correctly rounded fma gives the
        // builder's p + (q * s) bit for bit
        auto dq = [&](float pp, unsigned w, float sc) { return fmaf((float)((w >> (8 * i)) & 255u), sc, pp); };
        float tn, tx;
        if (DQ) {
            const float x0 = dq(px, qlx, sx) * R.ix, x1 = dq(px, qhx, sx) * R.ix;
            const float y0 = dq(py, qly, sy) * R.iy, y1 = dq(py, qhy, sy) * R.iy;
            const float z0 = dq(pz, qlz, sz) * R.iz, z1 = dq(pz, qhz, sz) * R.iz;
            tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
            tx = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
        } else {
            slab(dq(g0.x, qlx, sx), dq(g0.x, qhx, sx), dq(g0.y, qly, sy), dq(g0.y, qhy, sy), dq(g0.z, qlz, sz),
                 dq(g0.z, qhz, sz), R.o, R.ix, R.iy, R.iz, tn, tx);
        }
        t[i] = (on && r[i] != INT_MIN && box_hit(tn, tx, cull)) ? tn : INFINITY;   // misses sort last
    }
    if (COUNT && on) {
        c.nodes++;
        c.boxes += (r[0] != INT_MIN) + (r[1] != INT_MIN) + (r[2] != INT_MIN) + (r[3] != INT_MIN);
    }
    auto ce = [&](int a, int b) __attribute__((always_inline)) {
        const bool sw = t[b] < t[a];
        const float ta = t[a], tb = t[b];
        const int ra = r[a], rb = r[b];
        t[a] = sw ? tb : ta; t[b] = sw ? ta : tb;
        r[a] = sw ? rb : ra; r[b] = sw ? ra : rb;
    };
    // the nearest child first (continued), the other three pushed in tournament order, not fully sorted:
    // the order only steers the walk (r04, VALU-bound: C5 4,764 / 4,762 -> 4,726 / 4,730 ms with 2 of the
    // 5 compare-exchanges dropped; r03, before the walk was issue-bound, it was -0.2 %)
    ce(0, 1); ce(2, 3); ce(0, 2);
#pragma unroll
    for (int i = 3; i >= 1; --i) {
        if (t[i] < INFINITY) {
            st.template put<OVF>(R.soff, make_int2(r[i], __float_as_int(t[i])));
            R.soff += st.stride;
        }
    }
    return t[0] < INFINITY ? r[0] : INT_MIN;
}

// The wide leaf on its loaded record: the exact leaf box, then Moller-Trumbore.  Returns true when
// an any-hit ray is finished.
// PRE: the exact leaf box test was done by the caller (bh0: wide_step's shared slab)
template <bool COUNT, bool PRE = false>
__device__ __forceinline__ bool wide_leaf(float4 g0, float4 g1, float4 g2, float4 g3, FastRay& R, Cnt& c,
                                          bool on = true, bool bh0 = false) {   // on = false: no triangle is accepted
    if (COUNT && on) { c.tris++; c.boxes++; }
    bool bh = bh0;
    if (!PRE) {
        float tn, tx;
        slab(g0.x, g0.w, g0.y, g1.x, g0.z, g1.y, R.o, R.ix, R.iy, R.iz, tn, tx);
        bh = box_hit(tn, tx, R.bk * CULL_MARGIN);
    }
    float k;
    const int rank = (int)((~(unsigned)R.item) >> 6);
    const bool mt =
        mt_core(rtm_v3(g1.z, g1.w, g2.x), rtm_v3(g2.y, g2.z, g2.w), rtm_v3(g3.x, g3.y, g3.z), R.o, R.d, &k);
    const bool take = on & bh & mt & (k > 0.0001f) & ((k < R.bk) | ((k == R.bk) & (rank < R.brank)));
    R.bk = take ? k : R.bk;
    // the 4-wide walk keeps 48 x the index (its consumer divides): the plain index changed the register
    // allocation of its 72-VGPR kernel for the worse (51 instead of 36 spilled, one scratch access in the loop)
    R.bt = take ? 48 * __float_as_int(g3.w) : R.bt;
    R.brank = take ? rank : R.brank;
    return take && R.any;
}

// One item of the walk over the 4-wide quantised layout (DevScene::wnodes, rt_api.hip emit_wide):
// an internal node -- its up to 4 child boxes dequantised (p + q * 2^e per bound) and tested, the
// hit children sorted by entry distance, the nearest continued and the others pushed farthest first
// -- or a leaf: its exact box tested again (the quantised box is a superset) and its triangle
// intersected.  Nodes and leaves are both 64 bytes, fetched with the same four 16-byte loads, like
// fast_step.  The accepted triangles are the binary walk's (own exact leaf box passes, MT hit,
// k > 1e-4, lowest (k, rank)), so the hit is the same.  Returns true when the ray is finished.
template <bool COUNT, bool OVF, bool DQ = false>
__device__ __forceinline__ bool wide_step(FastRay& R, const char* nb, const char* lb, const LaneStack& st, Cnt& c) {
    const bool node = R.item >= 0;
    const char* p = node ? nb + 64u * (unsigned)R.item : lb + ~(unsigned)R.item;
    const float4 g0 = *reinterpret_cast<const float4*>(p);
    const float4 g1 = *reinterpret_cast<const float4*>(p + 16);
    const float4 g2 = *reinterpret_cast<const float4*>(p + 32);
    const float4 g3 = *reinterpret_cast<const float4*>(p + 48);
    if (COUNT) count_wave(c.wave_trav);
    // both codes on every lane (a step almost always holds node and leaf lanes), predicated
    // one slab test serves a node lane's child 0 (its dequantised box) and a leaf lane's exact leaf box:
    // the bounds are selected per lane, the arithmetic is the same slab either way (r04: C5 4,893 ->
    // 4,767 ms per frame; the walk is VALU-issue-bound, 12 of its ~490 instructions per step fewer)
    const unsigned meta = __float_as_uint(g0.w);
    auto dq0 = [&](float pp, float w, unsigned sh) {
        return fmaf((float)(__float_as_uint(w) & 255u), __uint_as_float(((meta >> sh) & 255u) << 23), pp);
    };
    float tn0, tx0;
    slab(node ? dq0(g0.x, g2.x, 0) : g0.x, node ? dq0(g0.x, g2.w, 0) : g0.w, node ? dq0(g0.y, g2.y, 8) : g0.y,
         node ? dq0(g0.y, g3.x, 8) : g1.x, node ? dq0(g0.z, g2.z, 16) : g0.z, node ? dq0(g0.z, g3.y, 16) : g1.y, R.o,
         R.ix, R.iy, R.iz, tn0, tx0);
    const bool h0 = box_hit(tn0, tx0, R.bk * CULL_MARGIN);
    const int nx = wide_node<COUNT, OVF, true, DQ>(g0, g1, g2, g3, R, st, c, node, tn0, h0);
    if (wide_leaf<COUNT, true>(g0, g1, g2, g3, R, c, !node, h0)) return true;
    if (nx != INT_MIN) {
        R.item = nx;
        return false;
    }
    while (R.soff > 0) {   // pop the next item still in front of the best hit
        R.soff -= st.stride;
        const int2 en = st.template get<OVF>(R.soff);
        if (__int_as_float(en.y) <= R.bk * CULL_MARGIN) {
            R.item = en.x;
            return false;
        }
    }
    return true;
}

// One round of the wide walk (the counterpart of fast_round): descend nearest children until a
// leaf is reached or nothing is hit, test the leaf, then pop the next live entry.
template <bool COUNT, bool OVF>
__device__ __forceinline__ bool wide_round(FastRay& R, const char* nb, const char* lb, const LaneStack& st, Cnt& c) {
    while (R.item >= 0) {
        if (COUNT) count_wave(c.wave_trav);
        const char* p = nb + 64u * (unsigned)R.item;
        R.item = wide_node<COUNT, OVF>(*reinterpret_cast<const float4*>(p), *reinterpret_cast<const float4*>(p + 16),
                                       *reinterpret_cast<const float4*>(p + 32),
                                       *reinterpret_cast<const float4*>(p + 48), R, st, c);
    }
    if (R.item != INT_MIN) {
        if (COUNT) count_wave(c.wave_trav);
        const char* p = lb + ~(unsigned)R.item;
        if (wide_leaf<COUNT>(*reinterpret_cast<const float4*>(p), *reinterpret_cast<const float4*>(p + 16),
                             *reinterpret_cast<const float4*>(p + 32), *reinterpret_cast<const float4*>(p + 48), R, c))
            return true;
    }
    while (R.soff > 0) {
        R.soff -= st.stride;
        const int2 en = st.template get<OVF>(R.soff);
        if (__int_as_float(en.y) <= R.bk * CULL_MARGIN) {
            R.item = en.x;
            return false;
        }
    }
    return true;
}

}  // namespace

}  // namespace rt
