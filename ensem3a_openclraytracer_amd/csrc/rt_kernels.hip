// HIP kernels of the MI355X path tracer (gfx950 / CDNA4).
//
// One work-item per pixel, like the reference kernel (Raytracing.cl:161-221),
// but the per-pixel work is restructured for a 64-wide wavefront:
//
//  * the nested spp x bounce loops of Raytracing.cl:191-209 / naiveGI
//    (Raytracing.cl:46-151) become ONE flat loop whose every iteration traces
//    exactly one ray per lane (bounce ray or sun ray).  A lane whose path ends
//    starts its next sample in the same iteration, so lanes never wait for the
//    longest path of the wave; only the per-ray traversal length diverges.
//    The RNG stream of a pixel is consumed in exactly the reference order, so
//    results are unchanged.
//  * BVH traversal (MathLib.cl:234-288) has two implementations:
//      REF  - the reference's pre-order DFS over its own 9-float AoS nodes,
//             true divisions in the slab test, 20-slot stack with silent drop.
//             Bit-identical to the CPU oracle.
//      FAST - a BVH2 whose nodes carry both child boxes (64 B, four float4
//             loads), reciprocal-direction slab tests, closest-child-first
//             descent, t-culling against the best hit, and a tie break on the
//             leaf's rank in the reference DFS order, so the closest hit is
//             the one the reference selects (first found among equal k).
//    Both keep the per-ray stack in LDS, one column per work-item
//    ([depth][blockDim] ints: lane-consecutive, bank-conflict free).
//
// Numerics: every OpenCL builtin of the reference is taken from rtm.h and the
// file is compiled with -ffp-contract=off (see rtm.h).
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
constexpr int REF_STACK = 20;  // stack.cl:4, Raytracing capacity 20

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
                if (top == REF_STACK - 1) { if (COUNT) c.dropped++; }
                else stk[(++top) * B] = L;
            }
            const int R = (int)nd[1];
            if (R != -1) {
                if (top == REF_STACK - 1) { if (COUNT) c.dropped++; }
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
// Moller-Trumbore on a triangle given as (a.p, e1, e2): MathLib.cl:117-160's arithmetic.
__device__ __forceinline__ bool mt_core(rtm_f3 p0, rtm_f3 e1, rtm_f3 e2, rtm_f3 o, rtm_f3 d, float* kout) {
    const rtm_f3 h = rtm_cross(d, e2);
    const float a = rtm_dot(e1, h);
    const float f = 1.0f / a;
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
#ifndef RT_STACK_AS
#define RT_STACK_AS 1
#endif
#if RT_STACK_AS
// The LDS part is addressed through an LDS-qualified pointer: the compiler then cannot merge the
// LDS and overflow branches of put/get into one generic (flat) access, which waits on both the
// vector-memory and the LDS counters
typedef char __attribute__((address_space(3))) lds_char;
typedef unsigned long long __attribute__((address_space(3))) lds_u64;
#else
typedef char lds_char;
typedef unsigned long long lds_u64;
#endif
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
    // entry `off` of the stack of the lane dl lanes away in the same wave (team walk steals)
    template <bool OVF>
    __device__ __forceinline__ int2 get_lane(unsigned off, int dl) const {
        int2 e;
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
    const float ix = 1.0f / d.x, iy = 1.0f / d.y, iz = 1.0f / d.z;
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
constexpr int BRUTE_WAVE_LDS = 64 * 6 * 4 + 64 * 8 + 256 * 4;   // ray table | best keys | pair ring

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
    unsigned* ring = reinterpret_cast<unsigned*>(wl + 64 * 6 * 4 + 64 * 8);   // owner << 16 | triangle
    ray[0 * 64 + lane] = o.x; ray[1 * 64 + lane] = o.y; ray[2 * 64 + lane] = o.z;
    ray[3 * 64 + lane] = d.x; ray[4 * 64 + lane] = d.y; ray[5 * 64 + lane] = d.z;
    const unsigned long long nokey = ((unsigned long long)__float_as_uint(1000.0f) << 32) | 0xffffffffull;
    bestk[lane] = nokey;
    wave_lds_sync();
    const float ix = 1.0f / d.x, iy = 1.0f / d.y, iz = 1.0f / d.z;
    float bk = 1000.0f;
    unsigned head = 0, tail = 0;   // wave-uniform ring positions
    auto run_batch = [&](int n) __attribute__((always_inline)) {
        if (myrank < n) {
            const unsigned e = ring[(head + myrank) & 255];
            const unsigned ow = e >> 16, q = e & 0xffffu;
            const rtm_f3 ro = rtm_v3(ray[ow], ray[64 + ow], ray[128 + ow]);
            const rtm_f3 rd = rtm_v3(ray[192 + ow], ray[256 + ow], ray[320 + ow]);
            // record q's last three float4 (hi.yz a.xy | a.z e1.xyz | e2.xyz tri): LDS copy or global
            const float4* rq = mtrec + mtstride * q;
            const float4 r1 = rq[0], r2 = rq[1], r3 = rq[2];
            const rtm_f3 a = rtm_v3(r1.z, r1.w, r2.x), e1 = rtm_v3(r2.y, r2.z, r2.w), e2 = rtm_v3(r3.x, r3.y, r3.z);
            const rtm_f3 h = rtm_cross(rd, e2);
            const float det = rtm_dot(e1, h);
            const float f = 1.0f / det;
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
        if (pass) {
            if (COUNT) c.tris += qb >= 0 ? 2 : 1;
            const unsigned r = lane_prefix(m, tail);
            ring[r & 255] = (tl << 16) | qa;
            if (qb >= 0) ring[(r + n) & 255] = (tl << 16) | (unsigned)qb;
        }
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
                if (g0 + j >= S.nbox) break;   // padding (never hit; skipped so the counters stay exact)
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

__device__ __forceinline__ LaunchConst make_const(const FrameParams& F) {  // evaluated once per launch
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
    rtm_f3 d = rtm_normalize(rtm_sub(rtm_add(C.position, pc), C.focal));
    d = rtm_rot_apply(C.cam_rx, d);
    d = rtm_rot_apply(C.cam_ry, d);
    return rtm_rot_apply(C.cam_rz, d);
}

// ---- IBL, MathLib.cl:72-90 (integer coords through a linear sampler) ----
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
    const int x0 = min(max(x > -2147483647 ? x - 1 : x, 0), W - 1), x1 = min(max(x, 0), W - 1);
    const int y0 = min(max(y > -2147483647 ? y - 1 : y, 0), H - 1), y1 = min(max(y, 0), H - 1);
    const uchar4 t00 = S.ibl[(int64_t)y0 * W + x0];
    const uchar4 t10 = S.ibl[(int64_t)y0 * W + x1];
    const uchar4 t01 = S.ibl[(int64_t)y1 * W + x0];
    const uchar4 t11 = S.ibl[(int64_t)y1 * W + x1];
    const float sr = (float)((int)t00.x + (int)t10.x + (int)t01.x + (int)t11.x);
    const float sg = (float)((int)t00.y + (int)t10.y + (int)t01.y + (int)t11.y);
    const float sb = (float)((int)t00.z + (int)t10.z + (int)t01.z + (int)t11.z);
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
    const float r = sqrtf(u);
    float st, ct;
    rtm_sincos(theta, &st, &ct);
    const rtm_f3 localV = rtm_v3(r * ct, r * st, sqrtf(rtm_fmax(0.0f, 1.0f - u)));
    rtm_f3 l;
    if (f2.w != 0.0f) {
        l = rtm_scale(localV, n.z);
    } else {
        rtm_rot R;
        R.q = rtm_v4(f0.x, f0.y, f0.z, f0.w);
        R.qinv = rtm_v4(f1.x, f1.y, f1.z, f1.w);
        l = rtm_normalize(rtm_rot_apply(R, localV));
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
        A = sqrtf(ra);
        Z = sqrtf(rtm_fmax(0.0f, 1.0f - ra));
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
        if (cosine) l = rtm_normalize(l);
    }
    *invPdf = cosine ? 3.14f / (rtm_fmax(rtm_dot(l, n), 0.0f)) : 2.0f * 3.14f;
    return l;
}

// ---- BRDF_GGX, MathLib.cl:461-500 ----
__device__ __forceinline__ rtm_f3 brdf_ggx(rtm_f3 color, float rough, rtm_f3 v, rtm_f3 l, rtm_f3 n) {
    const rtm_f3 h = rtm_normalize(rtm_add(l, v));
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
        (1.0f / rtm_fmax(4.0f * rtm_fmax(rtm_dot(v, n), 0.0f) * rtm_fmax(rtm_dot(l, n), 0.0f), 0.001f));
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
    const rtm_f3 nn = rtm_normalize(n);
    const float colinear = rtm_fabs(rtm_dot(nn, rtm_v3(0.0f, 0.0f, 1.0f)));
    rtm_rot R;
    R.q = rtm_v4(1, 0, 0, 0);
    R.qinv = R.q;
    if (colinear != 1.0f) {
        const float ang = rtm_acos(rtm_dot(n, rtm_v3(0, 0, 1)));
        if (type == 1) R = rtm_rot_prepare(ang, rtm_cross(rtm_v3(0, 0, 1), n));
        else if (type == 2) R = rtm_rot_prepare(ang, rtm_normalize(rtm_cross(rtm_v3(0.0f, 0.0f, 1.0f), n)));
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
};

// group g's j-th pixel (chunks g, g + kGroups, g + 2 kGroups, ...: increasing in j)
__device__ __forceinline__ unsigned group_pixel(unsigned g, unsigned j) {
    constexpr unsigned m = (1u << kChunkShift) - 1u;
    return (((j >> kChunkShift) * (unsigned)kGroups + g) << kChunkShift) | (j & m);
}

// pixels of group g in a tile of nloc pixels (wave-uniform)
__device__ __forceinline__ unsigned group_pixels(unsigned g, unsigned nloc) {
    const unsigned chunks = nloc >> kChunkShift, rem = nloc & ((1u << kChunkShift) - 1u);
    const unsigned full = chunks > g ? (chunks - 1u - g) / (unsigned)kGroups + 1u : 0u;
    return (full << kChunkShift) + (chunks % (unsigned)kGroups == g ? rem : 0u);
}

// need: wave-uniform mask of the requesting lanes (team leaders); lane0: the calling lane's team
// leader.  Returns the calling lane's tile pixel index (>= nloc: none left in the tile).  Called
// with the whole wave active; all control flow is wave-uniform, and the requests are served in
// rank order (group by group), so a lane only needs its rank.
__device__ __forceinline__ unsigned take_pixel(PixelQueue& Q, unsigned long long need, int lane0,
                                               unsigned* __restrict__ counters, unsigned nloc, int lane) {
    const bool mine = (need >> lane0) & 1ull;
    const unsigned rank = (unsigned)__popcll(need & ((1ull << lane0) - 1ull));
    const unsigned total = (unsigned)__popcll(need);
    const int leader = __ffsll((long long)need) - 1;
    unsigned q = nloc;
    unsigned base = 0;   // requests served so far
    unsigned g = blockIdx.x % (unsigned)kGroups;
    for (int t = 0; t < kGroups && base < total; ++t, g = (g + 1u) % (unsigned)kGroups) {
        if ((Q.dry >> g) & 1u) continue;
        const unsigned k = total - base;
        unsigned got = 0;
        if (lane == leader) got = atomicAdd(counters + g * (unsigned)(kCounterStride / 4), k);
        const unsigned j0 = (unsigned)__builtin_amdgcn_readfirstlane((int)__shfl(got, leader, 64));
        const unsigned have = group_pixels(g, nloc);
        const unsigned nok = j0 < have ? min(have - j0, k) : 0u;
        if (mine && rank >= base && rank < base + nok) q = group_pixel(g, j0 + (rank - base));
        if (nok < k) Q.dry |= 1u << g;   // the group's sequence has run past the tile
        base += nok;
    }
    return q;
}

// One persistent lane = one pixel at a time.  Lanes that finish their pixel
// take the next pixel index from a global counter: the wave ballots the lanes
// that need work, one lane adds the count to the counter, and each lane takes
// base + (its rank among the requesting lanes) -- so no lane idles while the
// rest of its wave finishes a slower pixel.  Per loop iteration every busy
// lane traces exactly one ray (primary, bounce or sun ray).
template <int TRAV, bool COUNT, bool LOG = false, bool SMEM = false, bool OVF = false, int BRUTE = 0>
// amdgpu_waves_per_eu(5): the register allocator keeps the kernel at 96 VGPRs, i.e. 5 waves per SIMD
// (one register more costs a wave per SIMD and ~10 % on C2); the product instantiations fit without
// spills, the instrumented (COUNT) ones spill a few registers to scratch.
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) render_kernel(DevScene S, FrameParams F, float* __restrict__ out,
                                               unsigned long long* __restrict__ counts,
                                               unsigned int* __restrict__ work_counter,
                                               const LaunchConst* __restrict__ lconst) {
    extern __shared__ int lds_stack[];
    const int B = blockDim.x;
    int* stk = lds_stack + threadIdx.x;
    const LaneStack lst = lane_stack(S, lds_stack);
    Cnt c{};
    // BRUTE (small scenes, brute-force traversal): the MT batches' triangle records and all shading
    // tables (hit records, hemisphere frames, materials) are staged in LDS behind the per-wave regions
    const float4* mtrec = nullptr;
    const float4* boxrec = nullptr;
    const float4* tshade = S.tri_shade;
    const float4* tframe = S.tri_frame;
    const float* tmat = S.mat;
    if (BRUTE) {
        float4* lr = reinterpret_cast<float4*>(reinterpret_cast<char*>(lds_stack) + (B / 64) * BRUTE_WAVE_LDS);
        float4* lb = lr + 3 * S.nbrute;                  // the distinct leaf boxes (team box tests)
        if (BRUTE == 2) {
            for (int q = threadIdx.x; q < 2 * S.nbox; q += B) lb[q] = S.brute_box[q];
            boxrec = lb;
        }
        float4* ls = lb + 2 * S.nbox;
        float4* lf = ls + S.ntri;
        float* lm = reinterpret_cast<float*>(lf + 3 * S.ntri);
        for (int q = threadIdx.x; q < 3 * S.nbrute; q += B) lr[q] = S.brute[4 * (q / 3) + 1 + q % 3];
        for (int q = threadIdx.x; q < S.ntri; q += B) ls[q] = S.tri_shade[q];
        for (int q = threadIdx.x; q < 3 * S.ntri; q += B) lf[q] = S.tri_frame[q];
        for (int q = threadIdx.x; q < kMatF * S.nmat; q += B) lm[q] = S.mat[q];
        __syncthreads();
        mtrec = lr;
        tshade = ls;
        tframe = lf;
        tmat = lm;
    }
    const LaunchConst& C = *lconst;   // uniform: scalar loads, no VGPRs
    // SMEM: the whole BVH2 node array and triangle array of a small scene are
    // staged in LDS behind the stacks, once per (persistent) block.
    const float4* nodes = S.nodes;
    const float4* tris = S.tri_fast;
    if (SMEM) {
        float4* ln = reinterpret_cast<float4*>(lds_stack + 2 * S.stack_lds * B);
        float4* lt = ln + kNodeF4 * S.nnodes;
        for (int q = threadIdx.x; q < kNodeF4 * S.nnodes; q += B)
            ln[(q % kNodeF4) * S.nnodes + q / kNodeF4] = S.nodes[q];
        for (int q = threadIdx.x; q < 3 * S.ntri; q += B) lt[q] = S.tri_fast[q];
        __syncthreads();
        nodes = ln;
        tris = lt;
    }
    const int W = F.width;
    const int imgSize = (int)F.npix;
    const float e3 = F.env[3], e4 = F.env[4];
    const int spp = F.spp, maxB = F.max_bounce;
    const unsigned int nloc = (unsigned int)F.nloc;
    const int lane = threadIdx.x & 63;
    const int ts = BRUTE == 2 ? F.team : 1;                      // lanes per pixel (1, 2, 4, 8)
    const int team_lane0 = lane & ~(ts - 1);
    const bool team_leader = lane == team_lane0;
    const unsigned long long team_leaders = ts == 1 ? ~0ull : ts == 2 ? 0x5555555555555555ull
                                             : ts == 4 ? 0x1111111111111111ull : 0x0101010101010101ull;

    int phase = FETCH;
    PixelQueue pq;
    int p = 0, i = 0;
    bool logme = false;
    uint32_t seed0 = 0, seed1 = 0;
    rtm_f3 cd = rtm_v3(0, 0, 0);              // camera ray direction (origin = C.position)
    float kc = 1000.0f;                       // cached primary hit
    int tc = -1;
    // the ray being shaded is not kept: at bounce 0 it is the camera ray (C.position, cd, hit kc),
    // later the bounce ray just traced (Bo, Bd, hit k) -- fewer registers live across the trace
    rtm_f3 so = rtm_v3(1, 1, 1);
    float k = 1000.0f;
    int tri = -1, j = 0;
    rtm_f3 Bo = rtm_v3(0, 0, 0), Bd = rtm_v3(0, 0, 0);
    rtm_f3 acc = rtm_v3(0, 0, 0);
    int s = 0;
    int cost = 0;   // pass 1: rays this pixel traced (pilot_cost)
    int sun0 = -2;  // the first bounce's shadow-ray hit (-1 = miss; -2 = not traced yet)

    // pass 1 (FrameParams::pass): after the pilot samples, save the pixel's state for pass 2; the
    // pixel is written (and its cost set to 0) when all its samples are done
    auto save_pilot = [&]() __attribute__((always_inline)) {
        F.pilot_state[2 * (int64_t)p] = make_float4(acc.x, acc.y, acc.z, kc);
        F.pilot_state[2 * (int64_t)p + 1] =
            make_float4(__uint_as_float(seed0), __uint_as_float(seed1), __int_as_float(tc), __int_as_float(s));
        F.pilot_cost[p] = s >= spp ? 0u : (unsigned)cost;
    };

    while (true) {
        // -- refill: ballot the lanes that need a pixel, one atomic per wave --
        // teams (BRUTE, F.team lanes per pixel): one bit per team, the team's lanes take the same pixel
        const unsigned long long need = __ballot(phase == FETCH) & team_leaders;
        if (need) {
            const unsigned int q = take_pixel(pq, need, team_lane0, work_counter, nloc, lane);
            if (phase == FETCH) {
                bool ok = q < nloc;
                if (ok) {
                    p = F.pass == 2 ? (int)F.pilot_order[q] : (int)q;
                    const int krow = p / W;
                    const int col = p - krow * W;
                    const int64_t i64 = ((int64_t)F.row0 + (int64_t)krow * F.row_step) * W + col;
                    ok = i64 < F.npix;
                    i = (int)i64;
                }
                if (ok) {
                    seed0 = (uint32_t)(i % imgSize);
                    seed1 = (uint32_t)(i / imgSize);
                    cd = camera_dir(C, W, i);
                    acc = rtm_v3(0, 0, 0);
                    s = 0;
                    cost = 0;
                    sun0 = -2;
                    phase = PRIMARY;
                    logme = LOG && i == F.log_pixel;
                    if (F.pass == 2) {   // continue from the pilot state: camera hit cached, sample s next
                        const float4 a = F.pilot_state[2 * (int64_t)p], b = F.pilot_state[2 * (int64_t)p + 1];
                        acc = rtm_v3(a.x, a.y, a.z);
                        kc = a.w;
                        seed0 = __float_as_uint(b.x);
                        seed1 = __float_as_uint(b.y);
                        tc = __float_as_int(b.z);
                        s = __float_as_int(b.w);
                        tri = tc; j = 0;
                        so = rtm_v3(1, 1, 1);
                        phase = s >= spp ? FETCH : PREP;   // finished in pass 1: already written
                    }
                } else {
                    // past the tile, or (pass 2, pixels in cost order) a padding pixel past the frame
                    phase = (F.pass == 2 && q < nloc) ? FETCH : DONE;
                }
            }
        }
        if (__all(phase == DONE)) break;
        if (COUNT && lane == 0) c.wave_outer++;
        if (phase == DONE || phase == FETCH) continue;   // FETCH: a pass-2 pixel finished in pass 1

        if (phase == PREP) {
            // naiveGI loop head for bounce j (Raytracing.cl:46-79); may complete samples without tracing
            bool done = true;
            const bool cam = j == 0;
            const rtm_f3 Ro = cam ? C.position : Bo, Rd = cam ? cd : Bd;
            const float kh = cam ? kc : k;
            if (j > maxB) {
                // naiveGI's loop never entered (maxBounce < 0): the sample stays 1
            } else if (tri < 0) {
                so = rtm_scale(rtm_mul(so, sample_ibl_if<COUNT>(S, C, Rd, e4, c)), e4);
            } else {
                const float4 sh = tshade[tri];
                const rtm_f3 n = xyz(sh);
                const Mat cm = load_mat(tmat, __float_as_int(sh.w));
                if (cm.type == 0) {
                    so = rtm_scale(so, cm.rough);
                } else {
                    const float4 f2 = tframe[3 * tri + 2];
                    const rtm_f3 nn = xyz(f2);
                    float invPdf = 0.0f;
                    rtm_f3 brdf = rtm_v3(0, 0, 0);
                    if (COUNT) count_event(c, cm.type);
                    if (cm.type == 1) {
                        Bd = hemi_cosine(n, tframe[3 * tri], tframe[3 * tri + 1], f2, &seed1, &seed0,
                                         &invPdf);
                        brdf = rtm_scale(cm.color, 1.0f / 3.14f);
                    } else if (cm.type == 2) {
                        Bd = hemi_uniform(n, tframe[3 * tri], tframe[3 * tri + 1], f2, &seed1, &seed0,
                                          &invPdf);
                        brdf = brdf_ggx(cm.color, cm.rough, rtm_scale(Rd, -1.0f), Bd, n);
                    } else {
                        Bd = Rd;
                        brdf = cm.color;
                        invPdf = 1.0f / rtm_fabs(rtm_dot(Bd, nn));
                    }
                    const rtm_f3 nd = rtm_normalize(Rd);
                    Bo = rtm_v3(fmaf(nd.x, kh, Ro.x), fmaf(nd.y, kh, Ro.y), fmaf(nd.z, kh, Ro.z));
                    // attenuation depends only on pre-trace values (Raytracing.cl:86-87): apply now
                    const float att = invPdf * rtm_fabs(rtm_dot(Bd, nn));
                    so = rtm_scale(rtm_mul(so, brdf), att);
                    phase = BOUNCE;
                    done = false;
                }
            }
            if (done) {
                if (LOG && logme) log_event(F, 3.0f, s + 1, rtm_v3(0, 0, 0), rtm_v3(0, 0, 0), 0.0f, 0, so);
                acc = rtm_add(acc, so);
                if (COUNT) c.samples++;
                ++s;
                // A sample that ends at its first loop head (j == 0: no bounce sampled) drew no random
                // numbers, so the RNG state is unchanged and every later sample of the pixel is this
                // sample again (same cached camera hit, same state): their colours are added in order,
                // bit for bit the reference's sum (FrameParams::fixed_point).
                if (TRAV == TRAV_FAST && F.fixed_point && j == 0 && !(LOG && logme)) {
                    if (COUNT) c.samples += (unsigned long long)max(spp - s, 0);
                    for (; s < spp; ++s) acc = rtm_add(acc, so);
                }
                if (s >= spp) {
                    phase = FETCH;
                    if (team_leader) store_pixel(out, p, acc, spp);
                    if (F.pass == 1) save_pilot();
                } else if (F.pass == 1 && s >= F.pilot) {
                    save_pilot();
                    phase = FETCH;
                } else {
                    tri = tc; j = 0;
                    so = rtm_v3(1, 1, 1);
                }
                continue;
            }
        }

        // -- one ray per busy lane --
        const rtm_f3 to = (phase == PRIMARY) ? C.position : Bo;
        const rtm_f3 td = (phase == PRIMARY) ? cd : ((phase == BOUNCE) ? Bd : C.sun);
        const Hit h = trace<TRAV, COUNT, SMEM, OVF, BRUTE != 0>(S, nodes, tris, to, td, stk, B, lst, c, mtrec, ts, boxrec);
        ++cost;
        bool finish = false;
        if (phase == PRIMARY) {
            tc = h.tri;
            kc = h.k;
            tri = tc; j = 0;
            so = rtm_v3(1, 1, 1);
            phase = PREP;
            if (spp <= 0) {   // reference: output = 0/0 -> NaN -> clamp gives 1
                if (team_leader) store_pixel(out, p, acc, spp);
                phase = FETCH;
            }
            continue;
        }
        if (LOG && logme) {
            const int hm = h.tri >= 0 ? __float_as_int(tshade[h.tri].w) : 0;
            log_event(F, phase == BOUNCE ? 1.0f : 2.0f, j, Bo, td, h.tri >= 0 ? h.k : -1.0f, hm, so);
        }
        int sun_hit = -2;   // the shadow ray's hit for the sun term below (-1 = miss; -2 = no sun term now)
        // the first bounce leaves from the cached camera hit in every sample of the pixel, so its shadow
        // ray towards the sun is the same ray each time: traced once per pixel (FrameParams::fixed_point)
        const bool sun_first = TRAV == TRAV_FAST && F.sun_cache && j == 0 && !(LOG && logme);
        if (phase == BOUNCE) {
            if (h.tri >= 0) {
                tri = h.tri; k = h.k;
                const Mat bm = load_mat(tmat, __float_as_int(tshade[h.tri].w));
                if (bm.type != 0) {
                    if (j == maxB) {
                        so = rtm_v3(0, 0, 0);
                        finish = true;
                    } else {
                        ++j;
                        phase = PREP;
                    }
                } else {
                    so = rtm_scale(so, bm.rough);
                    finish = true;
                }
            } else if (TRAV == TRAV_FAST && F.sun_skip) {
                sun_hit = -1;   // unlit sun: the shadow ray cannot change the sample (FrameParams::sun_skip)
            } else if (sun_first && sun0 != -2) {
                sun_hit = sun0;   // the first bounce's shadow ray, traced in an earlier sample of the pixel
            } else {
                phase = SUN;
            }
        } else {
            sun_hit = h.tri;
            if (sun_first) sun0 = h.tri;
        }
        if (sun_hit != -2) {  // SUN (Raytracing.cl:115-137)
            rtm_f3 sunLight = rtm_v3(0, 0, 0);
            if (COUNT) c.sun++;
            const Mat cm = load_mat(tmat, __float_as_int(tshade[tri].w));
            if (sun_hit < 0 && cm.type != 3) sunLight = rtm_v3(e3, e3, e3);
            if (sun_hit >= 0) {
                const Mat sm = load_mat(tmat, __float_as_int(tshade[sun_hit].w));
                if (sm.type == 3) sunLight = rtm_scale(sm.color, e3);
            }
            const rtm_f3 envLight = rtm_scale(sample_ibl_if<COUNT>(S, C, Bd, e4, c), e4);
            so = rtm_mul(so, rtm_add(sunLight, envLight));
            finish = true;
        }
        if (finish) {
            if (LOG && logme) log_event(F, 3.0f, s + 1, rtm_v3(0, 0, 0), rtm_v3(0, 0, 0), 0.0f, 0, so);
            acc = rtm_add(acc, so);
            if (COUNT) c.samples++;
            ++s;
            if (s >= spp) {
                if (team_leader) store_pixel(out, p, acc, spp);
                if (F.pass == 1) save_pilot();
                phase = FETCH;
            } else if (F.pass == 1 && s >= F.pilot) {
                save_pilot();
                phase = FETCH;
            } else {
                tri = tc; j = 0;
                so = rtm_v3(1, 1, 1);
                phase = PREP;
            }
        }
    }
    if (COUNT) {
        if (!team_leader) {   // a team's lanes repeat its pixel's shading: counted once
            c.env = 0; c.diffuse = 0; c.glossy = 0; c.glass = 0; c.sun = 0; c.samples = 0;
        }
        unsigned long long v[NCOUNTS] = {c.nodes, c.tris, c.rays, c.env, c.dropped, c.wave_trav, c.wave_outer,
                                          c.cyc_shade, c.cyc_trav, c.boxes, c.diffuse, c.glossy, c.glass,
                                          c.sun, c.samples};
#pragma unroll
        for (int q = 0; q < NCOUNTS; ++q) {
            unsigned long long x = v[q];
            for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
            if (lane == 0 && x) atomicAdd(&counts[q], x);
        }
    }
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
    int bt;           // best triangle's byte offset (48 t), -1 = none
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
    R.ix = 1.0f / d.x;
    R.iy = 1.0f / d.y;
    R.iz = 1.0f / d.z;
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
            R.bt = 48 * index;
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
#ifndef RT_FLAT_STEP
#define RT_FLAT_STEP 1
#endif
#ifndef RT_FLAT_TEAM
#define RT_FLAT_TEAM RT_FLAT_STEP
#endif
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
#if RT_FLAT_STEP
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
    const bool take = !node && mt && k > 0.0001f && (k < R.bk || (k == R.bk && rank < R.brank));
    if (COUNT) {
        if (node) { c.nodes++; c.boxes += 2; }
        else c.tris++;
    }
    R.bk = take ? k : R.bk;
    R.bt = take ? 48 * __float_as_int(g1.w) : R.bt;   // e1.w: the triangle's reference index
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
#else
    if (node) {
        if (COUNT) { c.nodes++; c.boxes += 2; }
        R.item = node_pick<OVF>(g0, g1, g2, e, R.o, R.ix, R.iy, R.iz, R.bk * CULL_MARGIN, st, R.soff);
        if (R.item != INT_MIN) return false;
    } else {
        if (COUNT) c.tris++;
        float k;
        int rank;
        if (mt_vals(g0, g1, leaf_e2(g2, e), R.o, R.d, &k, &rank) && k > 0.0001f && (k < R.bk || (k == R.bk && rank < R.brank))) {
            R.bk = k;
            R.bt = 48 * __float_as_int(g1.w);   // e1.w: the triangle's reference index
            R.brank = rank;
            if (R.any) return true;
        }
    }
#endif
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
#if RT_FLAT_TEAM
        // both tests, outcomes by selects (fast_step)
        const float cull = R.bk * CULL_MARGIN;
        float t0n, t0x, t1n, t1x;
        slab(g0.x, g0.y, g0.z, g0.w, g2.x, g2.y, R.o, R.ix, R.iy, R.iz, t0n, t0x);
        slab(g1.x, g1.y, g1.z, g1.w, g2.z, g2.w, R.o, R.ix, R.iy, R.iz, t1n, t1x);
        const bool h0 = node && box_hit(t0n, t0x, cull), h1 = node && box_hit(t1n, t1x, cull);
        float k;
        int rank;
        const bool mt = mt_vals(g0, g1, leaf_e2(g2, e), R.o, R.d, &k, &rank);
        improved = !node && mt && k > 0.0001f && (k < R.bk || (k == R.bk && rank < R.brank));
        if (COUNT) {
            if (node) { c.nodes++; c.boxes += 2; }
            else c.tris++;
        }
        R.bk = improved ? k : R.bk;
        R.bt = improved ? 48 * __float_as_int(g1.w) : R.bt;
        R.brank = improved ? rank : R.brank;
        const bool first0 = t0n <= t1n;
        if (h0 && h1) {
            st.template put<OVF>(R.soff, make_int2(first0 ? e.y : e.x, __float_as_int(first0 ? t1n : t0n)));
            R.soff += st.stride;
        }
        R.item = (h0 && h1) ? (first0 ? e.x : e.y) : h0 ? e.x : h1 ? e.y : NO_ITEM;
#else
        if (node) {
            if (COUNT) { c.nodes++; c.boxes += 2; }
            R.item = node_pick<OVF>(g0, g1, g2, e, R.o, R.ix, R.iy, R.iz, R.bk * CULL_MARGIN, st, R.soff);
        } else {
            if (COUNT) c.tris++;
            float k;
            int rank;
            if (mt_vals(g0, g1, leaf_e2(g2, e), R.o, R.d, &k, &rank) && k > 0.0001f &&
                (k < R.bk || (k == R.bk && rank < R.brank))) {
                R.bk = k;
                R.bt = 48 * __float_as_int(g1.w);
                R.brank = rank;
                improved = true;
            }
            R.item = NO_ITEM;
        }
#endif
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
#ifndef RT_FLAT_WIDE
#define RT_FLAT_WIDE 1
#endif
#ifndef RT_WIDE_PK
#define RT_WIDE_PK 0
#endif
typedef float f2 __attribute__((ext_vector_type(2)));
template <bool COUNT, bool OVF>
__device__ __forceinline__ int wide_node(float4 g0, float4 g1, float4 g2, float4 g3, FastRay& R, const LaneStack& st,
                                         Cnt& c, bool on = true) {   // on = false: no child is hit
    const float cull = R.bk * CULL_MARGIN;
    const unsigned meta = __float_as_uint(g0.w);
    const float sx = __uint_as_float((meta & 255u) << 23);
    const float sy = __uint_as_float(((meta >> 8) & 255u) << 23);
    const float sz = __uint_as_float(((meta >> 16) & 255u) << 23);
    const unsigned qlx = __float_as_uint(g2.x), qly = __float_as_uint(g2.y), qlz = __float_as_uint(g2.z);
    const unsigned qhx = __float_as_uint(g2.w), qhy = __float_as_uint(g3.x), qhz = __float_as_uint(g3.y);
    int r[4] = {__float_as_int(g1.x), __float_as_int(g1.y), __float_as_int(g1.z), __float_as_int(g1.w)};
    float t[4];
#if RT_WIDE_PK
    // the (lo, hi) pair of each axis in one packed-FP32 lane pair: v_pk_fma / v_pk_add / v_pk_mul
    // round each element exactly like the scalar fma / sub / mul below
    const f2 px = {g0.x, g0.x}, py = {g0.y, g0.y}, pz = {g0.z, g0.z};
    const f2 sxx = {sx, sx}, syy = {sy, sy}, szz = {sz, sz};
    const f2 nox = {-R.o.x, -R.o.x}, noy = {-R.o.y, -R.o.y}, noz = {-R.o.z, -R.o.z};
    const f2 ixx = {R.ix, R.ix}, iyy = {R.iy, R.iy}, izz = {R.iz, R.iz};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        auto qq = [&](unsigned wl, unsigned wh) -> f2 {
            return f2{(float)((wl >> (8 * i)) & 255u), (float)((wh >> (8 * i)) & 255u)};
        };
        const f2 tx = (__builtin_elementwise_fma(qq(qlx, qhx), sxx, px) + nox) * ixx;
        const f2 ty = (__builtin_elementwise_fma(qq(qly, qhy), syy, py) + noy) * iyy;
        const f2 tz = (__builtin_elementwise_fma(qq(qlz, qhz), szz, pz) + noz) * izz;
        const float tn = fmaxf(fmaxf(fminf(tx.x, tx.y), fminf(ty.x, ty.y)), fminf(tz.x, tz.y));
        const float tm = fminf(fminf(fmaxf(tx.x, tx.y), fmaxf(ty.x, ty.y)), fmaxf(tz.x, tz.y));
        t[i] = (on && r[i] != INT_MIN && box_hit(tn, tm, cull)) ? tn : INFINITY;   // misses sort last
    }
#else
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        // p + q * s with q * s exact (s a power of two, q < 256): one correctly rounded fma gives the
        // builder's p + (q * s) bit for bit
        auto dq = [&](float pp, unsigned w, float sc) { return fmaf((float)((w >> (8 * i)) & 255u), sc, pp); };
        float tn, tx;
        slab(dq(g0.x, qlx, sx), dq(g0.x, qhx, sx), dq(g0.y, qly, sy), dq(g0.y, qhy, sy), dq(g0.z, qlz, sz),
             dq(g0.z, qhz, sz), R.o, R.ix, R.iy, R.iz, tn, tx);
        t[i] = (on && r[i] != INT_MIN && box_hit(tn, tx, cull)) ? tn : INFINITY;   // misses sort last
    }
#endif
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
    ce(0, 1); ce(2, 3); ce(0, 2); ce(1, 3); ce(1, 2);
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
template <bool COUNT>
__device__ __forceinline__ bool wide_leaf(float4 g0, float4 g1, float4 g2, float4 g3, FastRay& R, Cnt& c,
                                          bool on = true) {   // on = false: no triangle is accepted
    if (COUNT && on) { c.tris++; c.boxes++; }
    float tn, tx;
    slab(g0.x, g0.w, g0.y, g1.x, g0.z, g1.y, R.o, R.ix, R.iy, R.iz, tn, tx);
    float k;
    const int rank = (int)((~(unsigned)R.item) >> 6);
#if RT_FLAT_STEP
    const bool bh = box_hit(tn, tx, R.bk * CULL_MARGIN);
    const bool mt =
        mt_core(rtm_v3(g1.z, g1.w, g2.x), rtm_v3(g2.y, g2.z, g2.w), rtm_v3(g3.x, g3.y, g3.z), R.o, R.d, &k);
    const bool take = on & bh & mt & (k > 0.0001f) & ((k < R.bk) | ((k == R.bk) & (rank < R.brank)));
    R.bk = take ? k : R.bk;
    R.bt = take ? 48 * __float_as_int(g3.w) : R.bt;   // the triangle's reference index
    R.brank = take ? rank : R.brank;
    return take && R.any;
#else
    if (on && box_hit(tn, tx, R.bk * CULL_MARGIN) &&
        mt_core(rtm_v3(g1.z, g1.w, g2.x), rtm_v3(g2.y, g2.z, g2.w), rtm_v3(g3.x, g3.y, g3.z), R.o, R.d, &k) &&
        k > 0.0001f && (k < R.bk || (k == R.bk && rank < R.brank))) {
        R.bk = k;
        R.bt = 48 * __float_as_int(g3.w);   // the triangle's reference index
        R.brank = rank;
        return R.any;
    }
    return false;
#endif
}

// One item of the walk over the 4-wide quantised layout (DevScene::wnodes, rt_api.hip emit_wide):
// an internal node -- its up to 4 child boxes dequantised (p + q * 2^e per bound) and tested, the
// hit children sorted by entry distance, the nearest continued and the others pushed farthest first
// -- or a leaf: its exact box tested again (the quantised box is a superset) and its triangle
// intersected.  Nodes and leaves are both 64 bytes, fetched with the same four 16-byte loads, like
// fast_step.  The accepted triangles are the binary walk's (own exact leaf box passes, MT hit,
// k > 1e-4, lowest (k, rank)), so the hit is the same.  Returns true when the ray is finished.
template <bool COUNT, bool OVF>
__device__ __forceinline__ bool wide_step(FastRay& R, const char* nb, const char* lb, const LaneStack& st, Cnt& c) {
    const bool node = R.item >= 0;
    const char* p = node ? nb + 64u * (unsigned)R.item : lb + ~(unsigned)R.item;
    const float4 g0 = *reinterpret_cast<const float4*>(p);
    const float4 g1 = *reinterpret_cast<const float4*>(p + 16);
    const float4 g2 = *reinterpret_cast<const float4*>(p + 32);
    const float4 g3 = *reinterpret_cast<const float4*>(p + 48);
    if (COUNT) count_wave(c.wave_trav);
#if RT_FLAT_WIDE
    // both codes on every lane (a step almost always holds node and leaf lanes), predicated
    const int nx = wide_node<COUNT, OVF>(g0, g1, g2, g3, R, st, c, node);
    if (wide_leaf<COUNT>(g0, g1, g2, g3, R, c, !node)) return true;
    if (nx != INT_MIN) {
        R.item = nx;
        return false;
    }
#else
    if (node) {
        R.item = wide_node<COUNT, OVF>(g0, g1, g2, g3, R, st, c);
        if (R.item != INT_MIN) return false;
    } else if (wide_leaf<COUNT>(g0, g1, g2, g3, R, c)) {
        return true;
    }
#endif
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

// FrameParams::step = 0 (auto): one item per step (fast_step) when the node array is at most this
// many bytes (L2-resident scenes, bound by the texture-address unit), descend-until-leaf rounds
// (fast_round) above (C5's 64 MB: bound by the latency of L2 misses; fast_round 1000 vs fast_step
// 944 Msamples/s there)
constexpr size_t kStepMaxBytes = 16u << 20;

// Occupancy: the 4-wide walk (C5) is bound by the latency of dependent L2 misses, so it runs
// kWideWaves waves per SIMD -- the register allocator keeps it at 72 VGPRs with some spilled to
// scratch, and dev_scene keeps kStackLdsWide stack entries per lane in LDS so that the LDS admits
// them.  C5 ms per frame at 4 / 5 / 6 / 7 / 8 waves: 7,214 / 6,432 / 6,045 / 5,890 / 6,040.  The
// BVH2 walk (C3/C4) is bound by the vector memory pipeline and keeps 4 waves with its whole 20-entry
// stack in LDS (5 waves with a 14-entry spilling stack: C3 149 -> 157 ms, C4 475 -> 502 ms).
#ifndef RT_WIDE_WAVES
#define RT_WIDE_WAVES 7   // variant builds (tools/variants.py) override it for the spill A/B
#endif
constexpr int kWideWaves = RT_WIDE_WAVES;
// TS > 1: teams of TS lanes per pixel walk each ray together (team_step; BVH2 item steps only).
// F.walk_team_dev (pass 2 of a pilot launch): the team size was chosen on the device from the pixels
// pass 1 left unfinished (pilot_team_pick_kernel); the instantiations of the other sizes, launched
// beside this one, return at once.
template <bool COUNT, bool LOG, bool SMEM, bool OVF, bool STEP, bool WIDE, int TS = 1>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WIDE ? kWideWaves : 4))) render_resume_kernel(DevScene S, FrameParams F, float* __restrict__ out,
                                                      unsigned long long* __restrict__ counts,
                                                      unsigned int* __restrict__ work_counter,
                                                      const LaunchConst* __restrict__ lconst) {
    // pass 2 with the team size chosen on the device: only the instantiation of that size renders
    if (F.walk_team_dev && __builtin_amdgcn_readfirstlane(*F.walk_team_dev) != TS) return;
    extern __shared__ int lds_stack[];
    const int B = blockDim.x;
    Cnt c{};
    const LaunchConst& C = *lconst;
    const float4* nodes = S.nodes;
    const float4* tris = S.tri_fast;
    if (SMEM) {
        float4* ln = reinterpret_cast<float4*>(lds_stack + 2 * S.stack_lds * B);
        float4* lt = ln + kNodeF4 * S.nnodes;
        for (int q = threadIdx.x; q < kNodeF4 * S.nnodes; q += B)
            ln[(q % kNodeF4) * S.nnodes + q / kNodeF4] = S.nodes[q];
        for (int q = threadIdx.x; q < 3 * S.ntri; q += B) lt[q] = S.tri_fast[q];
        __syncthreads();
        nodes = ln;
        tris = lt;
    }
    const LaneStack lst = lane_stack(S, lds_stack);
    const char* const nb = reinterpret_cast<const char*>(nodes);
    const char* const tb = reinterpret_cast<const char*>(tris);
    const char* const wnb = reinterpret_cast<const char*>(S.wnodes);   // WIDE: 4-wide nodes / leaf records
    const char* const wlb = reinterpret_cast<const char*>(S.wleaves);
    const unsigned kstride = SMEM ? 16u * (unsigned)S.nnodes : 16u;
    const int W = F.width;
    const int imgSize = (int)F.npix;
    const float e3 = F.env[3], e4 = F.env[4];
    const int spp = F.spp, maxB = F.max_bounce;
    const unsigned int nloc = (unsigned int)F.nloc;
    const int lane = threadIdx.x & 63;
    static_assert(TS == 1 || ((TS == 2 || TS == 4 || TS == 8) && STEP && !WIDE), "team walk: BVH2 item steps");
    const int team_lane0 = lane & ~(TS - 1);
    const bool team_leader = lane == team_lane0;
    const unsigned long long team_leaders = TS == 1 ? ~0ull : TS == 2 ? 0x5555555555555555ull
                                            : TS == 4 ? 0x1111111111111111ull : 0x0101010101010101ull;
    unsigned boff = 0;   // team walk: bottom of this lane's stack (bytes; entries below were stolen)

    int phase = FETCH;
    bool tracing = false;
    PixelQueue pq;
    FastRay T;
    T.item = 0; T.soff = 0; T.bk = 1000.0f; T.bt = -1; T.brank = -1; T.any = false;
    T.o = rtm_v3(0, 0, 0); T.d = rtm_v3(0, 0, 1); T.ix = T.iy = T.iz = 0.0f;
    int p = 0, i = 0;
    bool logme = false;
    uint32_t seed0 = 0, seed1 = 0;
    rtm_f3 cd = rtm_v3(0, 0, 0);              // camera ray direction (origin = C.position)
    float kc = 1000.0f;                       // cached primary hit (Raytracing.cl:186-187)
    int tc = -1;
    // the ray being shaded is not kept: at bounce 0 it is the camera ray (C.position, cd, hit kc),
    // later the bounce ray just traced (T.o, T.d, hit T.bk) -- fewer registers live across traversal
    rtm_f3 so = rtm_v3(1, 1, 1);
    int tri = -1, j = 0;
    rtm_f3 Bd = rtm_v3(0, 0, 0);   // bounce direction (its origin is T.o while it and the sun ray are traced)
    rtm_f3 acc = rtm_v3(0, 0, 0);
    int s = 0;
    bool drew = false;   // the current sample has drawn random numbers (a diffuse or glossy bounce)
    int cost = 0;        // pass 1: rays this pixel traced (pilot_cost)
    // The deterministic prefix of the pixel's samples (FrameParams::fixed_point; BVH2 walk): a sample's
    // path up to its first diffuse or glossy bounce draws no random number -- it is the cached camera
    // hit followed by straight-through glass bounces (Raytracing.cl:72-77) -- so it is the same path in
    // every sample of the pixel.  The state at the first bounce that draws (bounce j, surface, sample
    // colour so far, and the ray that reached it) is kept once met, and every later sample of the
    // pixel starts there instead of re-tracing the glass chain: the same rays would give the same hits.
    constexpr bool PREFIX = !WIDE;
    bool pre = false;
    int pre_j = 0, pre_tri = -1;
    rtm_f3 pre_so = rtm_v3(1, 1, 1), pre_o = rtm_v3(0, 0, 0), pre_d = rtm_v3(0, 0, 1);
    float pre_k = 1000.0f;
    // The sample's first diffuse or glossy bounce leaves from the same point in every sample (the end of
    // the deterministic prefix), so when its bounce ray escapes, the shadow ray towards the sun
    // (Raytracing.cl:115-124) is the same ray in every sample: its hit is traced once per pixel and kept.
    constexpr bool SUNC = true;
    constexpr int SUN_UNKNOWN = -2;
    int sun_c = SUN_UNKNOWN;   // the first drawing bounce's shadow-ray hit (triangle, -1 for none)
    bool fdb = false;          // the bounce in flight is the sample's first drawing bounce

    auto write_pixel = [&]() __attribute__((always_inline)) {
        if (team_leader) store_pixel(out, p, acc, spp);
    };
    // pass 1 (FrameParams::pass): after the pilot samples, save the pixel's state for pass 2; the
    // pixel is written (and its cost set to 0) when all its samples are done
    auto save_pilot = [&]() __attribute__((always_inline)) {
        if (!team_leader) return;
        F.pilot_state[2 * (int64_t)p] = make_float4(acc.x, acc.y, acc.z, kc);
        F.pilot_state[2 * (int64_t)p + 1] =
            make_float4(__uint_as_float(seed0), __uint_as_float(seed1), __int_as_float(tc), __int_as_float(s));
        F.pilot_cost[p] = s >= spp ? 0u : (unsigned)cost;
    };
    auto finish_sample = [&]() __attribute__((always_inline)) {  // output += baseColor; next sample from the cached camera hit
        if (LOG && logme) log_event(F, 3.0f, s + 1, rtm_v3(0, 0, 0), rtm_v3(0, 0, 0), 0.0f, 0, so);
        acc = rtm_add(acc, so);
        if (COUNT) c.samples++;
        ++s;
        if (s >= spp) write_pixel();
        const bool stop = F.pass == 1 && (s >= spp || s >= F.pilot);
        if (stop) save_pilot();
        // the next sample restarts from the cached camera hit; written as selects so that no branch
        // ends in a store the compiler could merge with the pixel store (that would force the path
        // state into scratch memory through a generic pointer)
        phase = (s >= spp || stop) ? FETCH : PREP;
        tri = tc; j = 0;
        so = rtm_v3(1, 1, 1);
        drew = false;
        if (PREFIX && pre) {   // the next sample starts after the deterministic prefix
            tri = pre_tri; j = pre_j;
            so = pre_so;
            T.o = pre_o; T.d = pre_d; T.bk = pre_k;
        }
    };
    // A sample that drew no random numbers (camera ray escaped or on an emitter, or only glass
    // bounces): the RNG state is unchanged, so every later sample of the pixel is this sample again.
    // Their colours are added in order here (finish_sample adds the last), bit for bit the
    // reference's sum (FrameParams::fixed_point).
    auto repeat_fixed = [&]() __attribute__((always_inline)) {
        if (F.fixed_point && !drew && !(LOG && logme)) {
            if (COUNT) c.samples += (unsigned long long)max(spp - 1 - s, 0);
            for (; s + 1 < spp; ++s) acc = rtm_add(acc, so);
        }
    };
    auto start = [&](rtm_f3 o, rtm_f3 d) __attribute__((always_inline)) {
        ++cost;
        tracing = !fast_init<COUNT>(S, T, o, d, c);
        if (WIDE) T.item = S.wroot_ref;
        if (TS > 1) {   // the team's first lane takes the root; the others steal from it
            if (!team_leader) T.item = NO_ITEM;
            boff = 0;
        }
        T.any = false;
    };

    while (true) {
        const unsigned long long t_iter = COUNT ? clock64() : 0;
        // -- refill: ballot the lanes that need a pixel, one atomic per wave (one pixel per team) --
        const unsigned long long need = __ballot(phase == FETCH) & team_leaders;
        if (need) {
            const unsigned int q = take_pixel(pq, need, team_lane0, work_counter, nloc, lane);
            if (phase == FETCH) {
                bool ok = q < nloc;
                if (ok) {
                    p = F.pass == 2 ? (int)F.pilot_order[q] : (int)q;
                    const int krow = p / W;
                    const int col = p - krow * W;
                    const int64_t i64 = ((int64_t)F.row0 + (int64_t)krow * F.row_step) * W + col;
                    ok = i64 < F.npix;
                    i = (int)i64;
                }
                if (ok) {
                    seed0 = (uint32_t)(i % imgSize);
                    seed1 = (uint32_t)(i / imgSize);
                    cd = camera_dir(C, W, i);
                    acc = rtm_v3(0, 0, 0);
                    s = 0;
                    cost = 0;
                    pre = false;
                    sun_c = SUN_UNKNOWN;
                    phase = PRIMARY;
                    logme = LOG && i == F.log_pixel;
                    if (F.pass == 2) {   // continue from the pilot state: camera hit cached, sample s next
                        const float4 a = F.pilot_state[2 * (int64_t)p], b = F.pilot_state[2 * (int64_t)p + 1];
                        acc = rtm_v3(a.x, a.y, a.z);
                        kc = a.w;
                        seed0 = __float_as_uint(b.x);
                        seed1 = __float_as_uint(b.y);
                        tc = __float_as_int(b.z);
                        s = __float_as_int(b.w);
                        tri = tc; j = 0;
                        so = rtm_v3(1, 1, 1);
                        drew = false;
                        phase = s >= spp ? FETCH : PREP;   // finished in pass 1: already written
                    } else {
                        start(C.position, cd);
                    }
                } else {
                    // past the tile, or (pass 2, pixels in cost order) a padding pixel past the frame
                    phase = (F.pass == 2 && q < nloc) ? FETCH : DONE;
                }
            }
        }
        if (__all(phase == DONE)) break;
        if (COUNT && lane == 0) c.wave_outer++;

        // -- advance every lane without a ray in flight until it needs one --
        if (!tracing && phase != DONE && phase != FETCH) {
            Hit h{T.bk, T.bt >= 0 ? (int)((unsigned)T.bt / 48u) : -1};
            if (phase == PRIMARY) {
                tc = h.tri;
                kc = h.k;
                tri = tc; j = 0;
                so = rtm_v3(1, 1, 1);
                drew = false;
                phase = PREP;
                if (spp <= 0) {   // reference: output = 0/0 -> NaN -> clamp gives 1
                    write_pixel();
                    phase = FETCH;
                }
            } else if (phase == BOUNCE) {
                if (LOG && logme) {
                    const int hm = h.tri >= 0 ? __float_as_int(S.tri_shade[h.tri].w) : 0;
                    log_event(F, 1.0f, j, T.o, Bd, h.tri >= 0 ? h.k : -1.0f, hm, so);
                }
                if (h.tri >= 0) {
                    tri = h.tri;
                    const Mat bm = load_mat(S.mat, __float_as_int(S.tri_shade[h.tri].w));
                    if (bm.type != 0) {
                        if (j == maxB) {
                            so = rtm_v3(0, 0, 0);
                            repeat_fixed();
                            finish_sample();
                        } else {
                            ++j;
                            phase = PREP;
                        }
                    } else {
                        so = rtm_scale(so, bm.rough);
                        repeat_fixed();
                        finish_sample();
                    }
                } else {
                    phase = SUN;   // escaped: shadow ray towards the sun (Raytracing.cl:115-124)
                    // unlit sun (FrameParams::sun_skip): the shadow ray cannot change the sample; it is not
                    // traced and the sun term below runs now with h, the bounce ray's miss
                    if (F.sun_skip) {
                    } else if (SUNC && fdb && sun_c != SUN_UNKNOWN) {
                        h.tri = sun_c;   // the first drawing bounce's shadow ray, traced in an earlier sample
                    } else {
                        start(T.o, C.sun);
                        T.any = F.sun_any != 0;
                        if (!tracing) continue;  // unreachable in practice (root box always hit from inside)
                    }
                }
            }
            if (phase == SUN && !tracing) {  // Raytracing.cl:125-137
                if (LOG && logme) {
                    const int hm = h.tri >= 0 ? __float_as_int(S.tri_shade[h.tri].w) : 0;
                    log_event(F, 2.0f, j, T.o, C.sun, h.tri >= 0 ? h.k : -1.0f, hm, so);
                }
                rtm_f3 sunLight = rtm_v3(0, 0, 0);
                if (COUNT) c.sun++;
                if (SUNC && fdb) sun_c = h.tri;
                const Mat cm = load_mat(S.mat, __float_as_int(S.tri_shade[tri].w));
                if (h.tri < 0 && cm.type != 3) sunLight = rtm_v3(e3, e3, e3);
                if (h.tri >= 0) {
                    const Mat sm = load_mat(S.mat, __float_as_int(S.tri_shade[h.tri].w));
                    if (sm.type == 3) sunLight = rtm_scale(sm.color, e3);
                }
                const rtm_f3 envLight = rtm_scale(sample_ibl_if<COUNT>(S, C, Bd, e4, c), e4);
                so = rtm_mul(so, rtm_add(sunLight, envLight));
                repeat_fixed();
                finish_sample();
            }
            // naiveGI loop heads (Raytracing.cl:46-79) until a ray is needed or the pixel is done
            while (phase == PREP) {
                const bool cam = j == 0;
                const rtm_f3 Ro = cam ? C.position : T.o, Rd = cam ? cd : T.d;
                const float k = cam ? kc : T.bk;
                if (j > maxB) {
                    repeat_fixed();
                    finish_sample();   // naiveGI's loop never entered (maxBounce < 0): the sample stays 1
                } else if (tri < 0) {
                    so = rtm_scale(rtm_mul(so, sample_ibl_if<COUNT>(S, C, Rd, e4, c)), e4);
                    repeat_fixed();
                    finish_sample();
                } else {
                    const float4 sh = S.tri_shade[tri];
                    const rtm_f3 n = xyz(sh);
                    const Mat cm = load_mat(S.mat, __float_as_int(sh.w));
                    if (cm.type == 0) {
                        so = rtm_scale(so, cm.rough);
                        repeat_fixed();
                        finish_sample();
                    } else {
                        const float4 f2 = S.tri_frame[3 * tri + 2];
                        const rtm_f3 nn = xyz(f2);
                        float invPdf = 0.0f;
                        rtm_f3 brdf = rtm_v3(0, 0, 0);
                        if (COUNT) count_event(c, cm.type);
                        if (PREFIX && F.fixed_point && cm.type != 3 && !drew && j > 0 && !pre && !(LOG && logme)) {
                            pre = true;   // the first bounce of the sample that draws, reached through glass only
                            pre_j = j; pre_tri = tri;
                            pre_so = so;
                            pre_o = T.o; pre_d = T.d; pre_k = T.bk;
                        }
                        fdb = SUNC && F.sun_cache && cm.type != 3 && !drew && !F.sun_skip && !(LOG && logme);
                        drew = drew || cm.type != 3;
                        if (cm.type != 3) {   // diffuse (1) or glossy (2): one sampler stream for both
                            Bd = hemi_sample(cm.type == 1, n, S.tri_frame[3 * tri], S.tri_frame[3 * tri + 1], f2,
                                             &seed1, &seed0, &invPdf);
                            if (cm.type == 1) brdf = rtm_scale(cm.color, 1.0f / 3.14f);
                            else brdf = brdf_ggx(cm.color, cm.rough, rtm_scale(Rd, -1.0f), Bd, n);
                        } else {
                            Bd = Rd;
                            brdf = cm.color;
                            invPdf = 1.0f / rtm_fabs(rtm_dot(Bd, nn));
                        }
                        const rtm_f3 nd = rtm_normalize(Rd);
                        const rtm_f3 Bo = rtm_v3(fmaf(nd.x, k, Ro.x), fmaf(nd.y, k, Ro.y), fmaf(nd.z, k, Ro.z));
                        // attenuation depends only on pre-trace values (Raytracing.cl:86-87): apply now
                        const float att = invPdf * rtm_fabs(rtm_dot(Bd, nn));
                        so = rtm_scale(rtm_mul(so, brdf), att);
                        phase = BOUNCE;
                        start(Bo, Bd);
                    }
                }
            }
        }

        // -- traversal rounds until at least F.resume_min lanes have no ray in flight --
        unsigned long long t_mid = 0;
        if (COUNT) {
            t_mid = clock64();
            if (lane == 0) c.cyc_shade += t_mid - t_iter;
        }
        // lanes that finished their tile (DONE) take no part in the threshold: it is resume_min / 64
        // of the lanes still rendering (all 64 until the pixel counters run dry)
        const unsigned long long alive = __ballot(phase != DONE);
        const int rthr = F.resume_min * __popcll(alive);
        while (true) {
            if (tracing && (TS > 1 ? team_step<COUNT, SMEM, OVF>(TS, T, boff, nb, tb, lst, kstride, c)
                            : WIDE ? (STEP ? wide_step<COUNT, OVF>(T, wnb, wlb, lst, c)
                                           : wide_round<COUNT, OVF>(T, wnb, wlb, lst, c))
                            : STEP ? fast_step<COUNT, SMEM, OVF>(S, T, nb, tb, lst, kstride, c)
                                   : fast_round<COUNT, SMEM, OVF>(S, T, nb, tb, lst, kstride, c)))
                tracing = false;
            const unsigned long long tr = __ballot(tracing);
            if (tr == 0 || 64 * __popcll(alive & ~tr) >= rthr) break;
        }
        if (COUNT && lane == 0) c.cyc_trav += clock64() - t_mid;
    }
    if (COUNT) {
        if (!team_leader) {   // a team's lanes repeat its pixel's shading and rays: counted once
            c.rays = 0; c.env = 0; c.diffuse = 0; c.glossy = 0; c.glass = 0; c.sun = 0; c.samples = 0;
        }
        unsigned long long v[NCOUNTS] = {c.nodes, c.tris, c.rays, c.env, c.dropped, c.wave_trav, c.wave_outer,
                                          c.cyc_shade, c.cyc_trav, c.boxes, c.diffuse, c.glossy, c.glass,
                                          c.sun, c.samples};
#pragma unroll
        for (int q = 0; q < NCOUNTS; ++q) {
            unsigned long long x = v[q];
            for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
            if (lane == 0 && x) atomicAdd(&counts[q], x);
        }
    }
}

__global__ void gamma_kernel(const float* __restrict__ in, float* __restrict__ out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const float p = fminf(in[i], 1.0f);
        out[i] = powf(p, 2.2f);
    }
}

// Output stage (FileManager.py:334-336 saveImg: (data*255).astype('uint8'); with gamma first the
// ImgProcessing.cl:1-10 kernel, as gamma_kernel above).  Four elements per thread: float4 in,
// one 32-bit word of bytes out.  v*255 rounds in fp32 like numpy's float32 product; the
// conversion truncates toward zero like numpy's cast for every v*255 in [0, 256) (rendered
// frames are clamped to [0, 1]); outside that range it saturates (NaN -> 0).
template <bool GAMMA>
__device__ __forceinline__ unsigned rgb8_byte(float v) {
    if (GAMMA) v = powf(fminf(v, 1.0f), 2.2f);
    const float x = v * 255.0f;
    return (unsigned)min(max((int)x, 0), 255);   // v_cvt_i32_f32 truncates, NaN -> 0
}

template <bool GAMMA>
__global__ void rgb8_kernel(const float* __restrict__ in, uint8_t* __restrict__ out, int64_t n) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // group of 4 elements
    const int64_t i = 4 * q;
    if (i + 4 <= n) {
        const float4 v = *reinterpret_cast<const float4*>(in + i);
        const unsigned w = rgb8_byte<GAMMA>(v.x) | (rgb8_byte<GAMMA>(v.y) << 8) | (rgb8_byte<GAMMA>(v.z) << 16) |
                           (rgb8_byte<GAMMA>(v.w) << 24);
        *reinterpret_cast<unsigned*>(out + i) = w;
    } else {
        for (int64_t k = i; k < n; ++k) out[k] = (uint8_t)rgb8_byte<GAMMA>(in[k]);
    }
}

// FrameParams::walk_team = 0 (auto): lanes per pixel of the tree walk.  Host rule (one-pass tiles,
// and pass 1 of a pilot launch) from the tile's pixels per resident lane: teams of 4 at <= 1 pixel
// per lane (measured on row tiles, profiles/r03_tile_scaling.json: C3 1/8 tile 83 -> 63 ms, C4 1/8
// tile 355 -> 167 ms, C4 1/4 tile 330 -> 206 ms; at 4-8 pixels per lane teams cost 1.3-2.1x).
inline int auto_walk_team(int64_t nloc, int64_t lanes) { return nloc <= lanes ? 4 : 1; }

// Device rule (pass 2 of a pilot launch): pass 1 finished every pixel whose samples draw nothing
// (fixed_point: sky pixels), so the pixels left, u per resident lane, are what pass 2 has to spread:
// teams of 4 at u <= 1/2, of 2 at u <= 1, else one lane per pixel (r03: C4 1/2 tile u = 0.9, teams
// of 2 323 vs 348 / 372 ms with 1 / 4 lanes; C3 1/2 tile u = 1.9, one lane 87 vs 106 ms).
__global__ void pilot_team_count_kernel(const uint32_t* __restrict__ cost, int64_t n, unsigned* __restrict__ left) {
    unsigned k = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        k += cost[i] != 0u;
    for (int off = 32; off > 0; off >>= 1) k += __shfl_down(k, off, 64);
    if ((threadIdx.x & 63) == 0 && k) atomicAdd(left, k);
}

__global__ void pilot_team_pick_kernel(const unsigned* __restrict__ left, int64_t lanes, int* __restrict__ ts) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const int64_t u2 = 2 * (int64_t)*left;   // 2 u lanes
        *ts = u2 <= lanes ? 4 : u2 <= 2 * lanes ? 2 : 1;
    }
}

template <int TRAV, bool COUNT, bool LOG, bool SMEM = false, bool RESUME = false, bool OVF = false,
          bool BRUTE = false, bool STEP = true, bool WIDE = false>
hipError_t launch_t(const DevScene& sc, const FrameParams& fp, int block, float* d_out, unsigned long long* d_counts,
                    unsigned int* d_work, hipStream_t stream) {
    // FAST: int2 entries; the brute-force path of small scenes needs no stack
    const int depth = (TRAV == TRAV_REF) ? REF_STACK : (sc.nbrute > 0 ? 1 : 2 * (sc.stack_lds > 0 ? sc.stack_lds : 1));
    size_t lds = (size_t)depth * block * sizeof(int);
    if (TRAV == TRAV_FAST && sc.nbrute > 0) lds = std::max(lds, (size_t)(block / 64) * BRUTE_WAVE_LDS);
    if (BRUTE)
        lds = (size_t)(block / 64) * BRUTE_WAVE_LDS + (size_t)sc.nbrute * 48 + (size_t)sc.nbox * 32 +
              (size_t)sc.ntri * 64 + (size_t)sc.nmat * (4 * kMatF);
    if (SMEM) lds += (size_t)(kNodeF4 * sc.nnodes + 3 * sc.ntri) * sizeof(float4);
    if (fp.nloc <= 0) return hipSuccess;
    // persistent grid: as many blocks as the device keeps resident (pixels are handed out by d_work)
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const void* kfn = RESUME ? (const void*)render_resume_kernel<COUNT, LOG, SMEM, OVF, STEP, WIDE>
                             : (const void*)render_kernel<TRAV, COUNT, LOG, SMEM, OVF, BRUTE ? 1 : 0>;
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, block, lds);
    if (e != hipSuccess) return e;
    // blocks per CU for at most max_waves waves per SIMD (4 SIMDs per CU)
    const int cap_cu = fp.max_waves > 0 ? std::max(1, fp.max_waves * 4 * 64 / block) : INT_MAX;
    const int64_t resident = (int64_t)std::max(1, cus) * std::max(1, std::min(per_cu, cap_cu));
    // team walk (render_resume_kernel TEAM): BVH2 item steps only.  walk_team_dev: the team size is
    // chosen on the device (pass 2 of a pilot launch); otherwise walk_team, 0 = auto (auto_walk_team)
    constexpr bool kTeamable = RESUME && STEP && !WIDE && !LOG;
    int wteam = 1;
    const bool dev_team = kTeamable && fp.walk_team_dev != nullptr;
    if (kTeamable && !dev_team) {
        wteam = fp.walk_team;
        if (wteam == 0) wteam = auto_walk_team(fp.nloc, resident * block);
        if (wteam != 2 && wteam != 4 && wteam != 8) wteam = 1;
    }

    // brute-force teams: a tile with fewer pixels than the device has lanes (a row slice of a
    // multi-GPU frame) gives each pixel 4 lanes that split its box tests when it fills at most a quarter of them
    FrameParams f = fp;
    f.team = 1;
    if (BRUTE) {
        f.team = fp.team;
        if (f.team == 0) {
            // measured on C2 tiles (one MI355X, 96-VGPR kernel: 327,680 resident lanes): a 1/8 tile
            // (131k pixels) is fastest with single lanes (2.23 vs 2.29 ms with pairs), a 1/16 tile with
            // teams of 4 (1.67 vs 1.88 with pairs, 2.28 single)
            const int64_t lanes = resident * block;
            f.team = fp.nloc * 4 <= lanes ? 4 : 1;
        }
    }
    f.walk_team = wteam;
    if (!dev_team) f.walk_team_dev = nullptr;
    const int64_t need = (fp.nloc * f.team * wteam + block - 1) / block;
    int64_t grid = std::min(need, resident);
    // the team instantiations (TS = 2, 4, 8) and their own occupancy
    auto team_fn = [&](int ts) -> const void* {
        if (!kTeamable) return nullptr;
        return ts == 2 ? (const void*)render_resume_kernel<COUNT, LOG, SMEM, OVF, STEP, WIDE, kTeamable ? 2 : 1>
             : ts == 4 ? (const void*)render_resume_kernel<COUNT, LOG, SMEM, OVF, STEP, WIDE, kTeamable ? 4 : 1>
                       : (const void*)render_resume_kernel<COUNT, LOG, SMEM, OVF, STEP, WIDE, kTeamable ? 8 : 1>;
    };
    auto team_grid = [&](int ts, int64_t* g) -> hipError_t {
        int per_cu_w = 0;
        hipError_t er = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_w, team_fn(ts), block, lds);
        *g = std::min((fp.nloc * ts + block - 1) / block,
                      (int64_t)std::max(1, cus) * std::max(1, std::min(per_cu_w, cap_cu)));
        return er;
    };
    if (kTeamable && wteam > 1 && !dev_team) {
        e = team_grid(wteam, &grid);
        if (e != hipSuccess) return e;
    }
    // teams run their own instantiation (the ts = 1 kernel keeps the scalar box loop)
    const void* tfn = (const void*)render_kernel<TRAV, COUNT, LOG, SMEM, OVF, BRUTE ? 2 : 0>;
    if (BRUTE && f.team > 1) {
        int per_cu_t = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_t, tfn, block, lds);
        if (e != hipSuccess) return e;
        grid = std::min(need, (int64_t)std::max(1, cus) * std::max(1, std::min(per_cu_t, cap_cu)));
    }
    e = hipMemsetAsync(d_work, 0, (size_t)kGroups * kCounterStride, stream);
    if (e != hipSuccess) return e;
    // the per-launch constants live after the counters in the same scratch block
    static_assert(kConstOffset >= kGroups * kCounterStride && kConstOffset + sizeof(LaunchConst) <= kWorkBytes,
                  "work block layout");
    LaunchConst* lc = reinterpret_cast<LaunchConst*>(reinterpret_cast<char*>(d_work) + kConstOffset);
    hipLaunchKernelGGL(make_const_kernel, dim3(1), dim3(64), 0, stream, f, lc);
    if (kTeamable && dev_team) {
        // the device picks 1, 2 or 4 (pilot_team_pick_kernel): all three are launched in order, and the
        // two whose size was not picked return at once
        int64_t g2 = 0, g4 = 0;
        e = team_grid(2, &g2);
        if (e == hipSuccess) e = team_grid(4, &g4);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((render_resume_kernel<COUNT, LOG, SMEM, OVF, STEP, WIDE, 1>), dim3((unsigned)grid),
                           dim3(block), lds, stream, sc, f, d_out, d_counts, d_work, (const LaunchConst*)lc);
        hipLaunchKernelGGL((render_resume_kernel<COUNT, LOG, SMEM, OVF, STEP, WIDE, kTeamable ? 2 : 1>),
                           dim3((unsigned)g2), dim3(block), lds, stream, sc, f, d_out, d_counts, d_work,
                           (const LaunchConst*)lc);
        hipLaunchKernelGGL((render_resume_kernel<COUNT, LOG, SMEM, OVF, STEP, WIDE, kTeamable ? 4 : 1>),
                           dim3((unsigned)g4), dim3(block), lds, stream, sc, f, d_out, d_counts, d_work,
                           (const LaunchConst*)lc);
    } else if (kTeamable && wteam == 2)
        hipLaunchKernelGGL((render_resume_kernel<COUNT, LOG, SMEM, OVF, STEP, WIDE, kTeamable ? 2 : 1>),
                           dim3((unsigned)grid), dim3(block), lds, stream, sc, f, d_out, d_counts, d_work,
                           (const LaunchConst*)lc);
    else if (kTeamable && wteam == 4)
        hipLaunchKernelGGL((render_resume_kernel<COUNT, LOG, SMEM, OVF, STEP, WIDE, kTeamable ? 4 : 1>),
                           dim3((unsigned)grid), dim3(block), lds, stream, sc, f, d_out, d_counts, d_work,
                           (const LaunchConst*)lc);
    else if (kTeamable && wteam == 8)
        hipLaunchKernelGGL((render_resume_kernel<COUNT, LOG, SMEM, OVF, STEP, WIDE, kTeamable ? 8 : 1>),
                           dim3((unsigned)grid), dim3(block), lds, stream, sc, f, d_out, d_counts, d_work,
                           (const LaunchConst*)lc);
    else if (RESUME)
        hipLaunchKernelGGL((render_resume_kernel<COUNT, LOG, SMEM, OVF, STEP, WIDE>), dim3((unsigned)grid), dim3(block), lds, stream,
                           sc, f, d_out, d_counts, d_work, (const LaunchConst*)lc);
    else if (BRUTE && f.team > 1)
        hipLaunchKernelGGL((render_kernel<TRAV, COUNT, LOG, SMEM, OVF, BRUTE ? 2 : 0>), dim3((unsigned)grid),
                           dim3(block), lds, stream, sc, f, d_out, d_counts, d_work, (const LaunchConst*)lc);
    else
        hipLaunchKernelGGL((render_kernel<TRAV, COUNT, LOG, SMEM, OVF, BRUTE ? 1 : 0>), dim3((unsigned)grid),
                           dim3(block), lds, stream, sc, f, d_out, d_counts, d_work, (const LaunchConst*)lc);
    return hipGetLastError();
}

// ---- test hooks (rt_debug.h): device evaluation of the numerics contract and of
// single rays through either traversal ----
__global__ void debug_math_kernel(int fn, const float* __restrict__ x, const float* __restrict__ y,
                                  float* __restrict__ out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float r = 0.0f;
    switch (fn) {
        case 0: r = rtm_sin(x[i]); break;
        case 1: r = rtm_cos(x[i]); break;
        case 2: r = rtm_tan(x[i]); break;
        case 3: r = rtm_asin(x[i]); break;
        case 4: r = rtm_acos(x[i]); break;
        case 5: r = rtm_atan2(x[i], y[i]); break;
        case 6: r = sqrtf(x[i]); break;
        case 7: r = x[i] / y[i]; break;
        default: break;
    }
    out[i] = r;
}

template <int TRAV>
__global__ void __launch_bounds__(256) debug_trace_kernel(DevScene S, const float* __restrict__ rays,
                                                          float* __restrict__ out, int64_t n) {
    extern __shared__ int lds_stack[];
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    Cnt c{};
    const float* r = rays + 6 * t;
    const Hit h = trace<TRAV, false>(S, S.nodes, S.tri_fast, rtm_v3(r[3], r[4], r[5]), rtm_v3(r[0], r[1], r[2]),
                                     lds_stack + threadIdx.x, blockDim.x, lane_stack(S, lds_stack), c);
    out[2 * t + 0] = h.k;
    out[2 * t + 1] = (float)h.tri;
}

}  // namespace

hipError_t launch_debug_math(int fn, const float* x, const float* y, float* out, int64_t n, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(debug_math_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, fn, x, y, out, n);
    return hipGetLastError();
}

hipError_t launch_debug_log(const DevScene& sc, const FrameParams& fp, int traversal, float* d_out,
                            unsigned int* d_work, hipStream_t stream) {
    if (traversal == TRAV_REF) return launch_t<TRAV_REF, false, true>(sc, fp, 64, d_out, nullptr, d_work, stream);
    if (sc.nbrute == 0 && sc.stack_lds < sc.depth)
        return launch_t<TRAV_FAST, false, true, false, false, true>(sc, fp, 64, d_out, nullptr, d_work, stream);
    return launch_t<TRAV_FAST, false, true>(sc, fp, 64, d_out, nullptr, d_work, stream);
}

hipError_t launch_prep_frames(const DevScene& sc, float4* frame, hipStream_t stream) {
    if (sc.ntri <= 0) return hipSuccess;
    hipLaunchKernelGGL(prep_frames_kernel, dim3((unsigned)((sc.ntri + 255) / 256)), dim3(256), 0, stream, sc.tri_shade,
                       sc.mat, sc.ntri, frame);
    return hipGetLastError();
}

hipError_t launch_debug_trace(const DevScene& sc, int traversal, const float* rays, float* out, int64_t n,
                              hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const int block = 128;
    // not a persistent grid: the whole FAST stack lives in LDS (no overflow buffer sized for this grid)
    DevScene s2 = sc;
    s2.stack_lds = sc.depth > 0 ? sc.depth : 1;
    s2.stack_ovf = nullptr;
    const int depth = traversal == TRAV_REF ? REF_STACK : 2 * s2.stack_lds;
    size_t lds = (size_t)depth * block * sizeof(int);
    if (traversal != TRAV_REF && sc.nbrute > 0) lds = std::max(lds, (size_t)(block / 64) * BRUTE_WAVE_LDS);
    if (traversal == TRAV_REF)
        hipLaunchKernelGGL(debug_trace_kernel<TRAV_REF>, dim3((unsigned)((n + block - 1) / block)), dim3(block), lds,
                           stream, s2, rays, out, n);
    else
        hipLaunchKernelGGL(debug_trace_kernel<TRAV_FAST>, dim3((unsigned)((n + block - 1) / block)), dim3(block), lds,
                           stream, s2, rays, out, n);
    return hipGetLastError();
}

template <bool COUNT, bool STEP>
hipError_t launch_resume(const DevScene& sc, const FrameParams& fp, int block, float* d_out,
                         unsigned long long* d_counts, unsigned int* d_work, hipStream_t stream, bool smem, bool ovf) {
    if (smem)
        return launch_t<TRAV_FAST, COUNT, false, true, true, false, false, STEP>(sc, fp, block, d_out, d_counts,
                                                                                 d_work, stream);
    if (ovf)
        return launch_t<TRAV_FAST, COUNT, false, false, true, true, false, STEP>(sc, fp, block, d_out, d_counts,
                                                                                 d_work, stream);
    return launch_t<TRAV_FAST, COUNT, false, false, true, false, false, STEP>(sc, fp, block, d_out, d_counts, d_work,
                                                                              stream);
}

template <bool COUNT>
hipError_t launch_fast(const DevScene& sc, const FrameParams& fp, int block, float* d_out,
                       unsigned long long* d_counts, unsigned int* d_work, hipStream_t stream) {
    const size_t scene_bytes = (size_t)(kNodeF4 * sc.nnodes + 3 * sc.ntri) * sizeof(float4);
    const bool smem = sc.ntri > 0 && sc.nbrute == 0 && scene_bytes <= kLdsSceneMax;
    const bool ovf = sc.nbrute == 0 && sc.stack_lds < sc.depth;
    const bool resume = sc.ntri > 0 && sc.nbrute == 0 && fp.resume_min > 0;
    const bool step = fp.step == 1 || (fp.step == 0 && (size_t)sc.nnodes * kNodeF4 * 16 <= kStepMaxBytes);
    if (resume && fp.wide && sc.wnodes && !smem) {
        // the wide walk takes item steps unless rounds are asked for (C5: 1,181 vs 1,035 Msamples/s)
        const bool step = fp.step != 2;
        if (ovf)
            return step ? launch_t<TRAV_FAST, COUNT, false, false, true, true, false, true, true>(
                              sc, fp, block, d_out, d_counts, d_work, stream)
                        : launch_t<TRAV_FAST, COUNT, false, false, true, true, false, false, true>(
                              sc, fp, block, d_out, d_counts, d_work, stream);
        return step ? launch_t<TRAV_FAST, COUNT, false, false, true, false, false, true, true>(
                          sc, fp, block, d_out, d_counts, d_work, stream)
                    : launch_t<TRAV_FAST, COUNT, false, false, true, false, false, false, true>(
                          sc, fp, block, d_out, d_counts, d_work, stream);
    }
    if (resume) {
        return step ? launch_resume<COUNT, true>(sc, fp, block, d_out, d_counts, d_work, stream, smem, ovf)
                    : launch_resume<COUNT, false>(sc, fp, block, d_out, d_counts, d_work, stream, smem, ovf);
    }
    // BRUTE stages the scene in LDS: only while two blocks still fit a CU
    const size_t brute_lds = (size_t)(block / 64) * BRUTE_WAVE_LDS + (size_t)sc.nbrute * 48 +
                             (size_t)sc.nbox * 32 + (size_t)sc.ntri * 64 + (size_t)sc.nmat * (4 * kMatF);
    if (sc.ntri > 0 && sc.nbrute > 0 && brute_lds <= 80 * 1024)
        return launch_t<TRAV_FAST, COUNT, false, false, false, false, true>(sc, fp, block, d_out, d_counts, d_work,
                                                                            stream);
    if (smem) return launch_t<TRAV_FAST, COUNT, false, true>(sc, fp, block, d_out, d_counts, d_work, stream);
    if (ovf)
        return launch_t<TRAV_FAST, COUNT, false, false, false, true>(sc, fp, block, d_out, d_counts, d_work, stream);
    return launch_t<TRAV_FAST, COUNT, false>(sc, fp, block, d_out, d_counts, d_work, stream);
}

// ---- two-pass ordering (FrameParams::pass): pilot costs -> pixel order, most expensive first ----
// Pixels are ordered in chunks of `chunk` consecutive tile pixels: the chunks by their summed pilot
// cost, the pixels of a chunk in tile order.  The tree walk orders single pixels (its lanes diverge
// anyway); the brute-force path would need chunks of a wave (64) to keep neighbouring lanes on
// neighbouring pixels -- its box loop and shading branches pay per wave -- and then gains nothing,
// so it runs one pass unless asked.
constexpr int kCostBins = 256;

__global__ void pilot_chunk_kernel(const uint32_t* __restrict__ cost, int64_t nfull, int chunk,
                                   uint32_t* __restrict__ ccost) {
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nfull; c += (int64_t)gridDim.x * blockDim.x) {
        uint32_t t = 0;
        for (int k = 0; k < chunk; ++k) t += cost[c * chunk + k];
        ccost[c] = t;
    }
}

__device__ __forceinline__ uint32_t cost_bin(uint32_t v, uint32_t scale, uint32_t maxbin) {
    return min(maxbin, (uint32_t)(((uint64_t)v * scale) >> 16));
}

// Stable counting sort of the chunks by cost bin (descending bins, tile order within a bin, so the
// pixels of one bin keep their raster order and a wave's lanes stay on nearby pixels), over segments
// of kSortSeg chunks: per-segment histograms (bin-major), their per-bin exclusive scan, the bin
// offsets, then each chunk's place = bin offset + segment offset + its rank among the segment's
// chunks of the same bin.
constexpr int kSortSeg = kCostBins;

__global__ void pilot_seg_hist_kernel(const uint32_t* __restrict__ ccost, int64_t n, int64_t nseg, uint32_t scale,
                                      uint32_t maxbin, uint32_t* __restrict__ seghist) {
    __shared__ uint32_t h[kCostBins];
    const int64_t seg = blockIdx.x;
    h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t q = seg * kSortSeg + threadIdx.x;
    if (q < n) atomicAdd(&h[cost_bin(ccost[q], scale, maxbin)], 1u);
    __syncthreads();
    seghist[threadIdx.x * nseg + seg] = h[threadIdx.x];
}

// one block per bin: exclusive scan of the bin's row of seghist in place, the row total to total[bin]
__global__ void pilot_seg_scan_kernel(uint32_t* __restrict__ seghist, int64_t nseg, uint32_t* __restrict__ total) {
    __shared__ uint32_t t[kCostBins];
    uint32_t* row = seghist + (int64_t)blockIdx.x * nseg;
    const int i0 = threadIdx.x;
    uint32_t carry = 0;
    for (int64_t base = 0; base < nseg; base += kCostBins) {
        const int64_t i = base + i0;
        const uint32_t v = i < nseg ? row[i] : 0u;
        t[i0] = v;
        __syncthreads();
        for (int off = 1; off < kCostBins; off <<= 1) {
            const uint32_t a = i0 >= off ? t[i0 - off] : 0u;
            __syncthreads();
            t[i0] += a;
            __syncthreads();
        }
        if (i < nseg) row[i] = carry + t[i0] - v;
        carry += t[kCostBins - 1];
        __syncthreads();
    }
    if (i0 == 0) total[blockIdx.x] = carry;
}

// offs[b] = number of chunks in bins above b (descending cost order); one block of kCostBins threads
__global__ void pilot_scan_kernel(const uint32_t* __restrict__ hist, uint32_t* __restrict__ offs) {
    __shared__ uint32_t t[kCostBins];
    const int b = threadIdx.x;
    t[b] = hist[b];
    __syncthreads();
    uint32_t above = 0;
    for (int c = b + 1; c < kCostBins; ++c) above += t[c];
    offs[b] = above;
}

__global__ void pilot_seg_scatter_kernel(const uint32_t* __restrict__ ccost, int64_t n, int64_t nseg, uint32_t scale,
                                         uint32_t maxbin, const uint32_t* __restrict__ seghist,
                                         const uint32_t* __restrict__ offs, uint32_t* __restrict__ corder) {
    __shared__ uint32_t bins[kSortSeg];
    const int64_t seg = blockIdx.x;
    const int64_t q = seg * kSortSeg + threadIdx.x;
    const uint32_t b = q < n ? cost_bin(ccost[q], scale, maxbin) : 0xffffffffu;
    bins[threadIdx.x] = b;
    __syncthreads();
    if (q >= n) return;
    uint32_t rank = 0;
    for (int j = 0; j < (int)threadIdx.x; ++j) rank += bins[j] == b ? 1u : 0u;
    corder[offs[b] + seghist[(int64_t)b * nseg + seg] + rank] = (uint32_t)q;
}

// pixel order: the full chunks in cost order, then the last partial chunk (if any) in place
__global__ void pilot_expand_kernel(const uint32_t* __restrict__ corder, int64_t nfull, int chunk, int64_t nloc,
                                    uint32_t* __restrict__ order) {
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nloc; q += (int64_t)gridDim.x * blockDim.x)
        order[q] = q < nfull * chunk ? corder[q / chunk] * (uint32_t)chunk + (uint32_t)(q % chunk) : (uint32_t)q;
}

hipError_t launch_render_pass(const DevScene& sc, const FrameParams& fp, int traversal, int block, float* d_out,
                              unsigned long long* d_counts, unsigned int* d_work, hipStream_t stream);

// Two passes (fp.pilot > 0, product launches only): the first fp.pilot samples of every pixel,
// then the rest of each pixel in descending order of the rays its (chunk's) pilot samples traced.  The
// frame ends when its last-started pixels finish; started last, the cheapest pixels make that tail
// short.  Every pixel's samples run in the same order as in one pass, so the frame is bit-identical.
hipError_t launch_render(const DevScene& sc, const FrameParams& fp, int traversal, int block, float* d_out,
                         unsigned long long* d_counts, unsigned int* d_work, hipStream_t stream) {
    if (fp.pilot <= 0 || fp.pass != 0 || d_counts || fp.spp <= fp.pilot || fp.nloc <= 0 || !fp.pilot_state)
        return launch_render_pass(sc, fp, traversal, block, d_out, d_counts, d_work, stream);
    FrameParams a = fp;
    a.pass = 1;
    hipError_t e = launch_render_pass(sc, a, traversal, block, d_out, nullptr, d_work, stream);
    if (e != hipSuccess) return e;
    // scratch after the pixel order (rt_api.hip setup_pilot): bin totals | offs | chunk costs |
    // chunk order | segment histograms
    uint32_t* order = const_cast<uint32_t*>(fp.pilot_order);
    uint32_t* total = order + fp.nloc;
    uint32_t* offs = total + kCostBins;
    const int chunk = std::max(fp.pilot_chunk, 1);
    const int64_t nfull = fp.nloc / chunk;
    const int64_t nseg = (nfull + kSortSeg - 1) / kSortSeg;
    uint32_t* ccost = offs + kCostBins;
    uint32_t* corder = ccost + nfull;
    uint32_t* seghist = corder + nfull;
    // `levels` cost bins over a chunk's rays up to 2 (maxBounce + 1) rays per pilot sample per pixel
    const int levels = std::min(std::max(fp.pilot_levels, 2), kCostBins);
    const uint64_t top = (uint64_t)chunk * fp.pilot * 2u * (uint64_t)(std::max(fp.max_bounce, 0) + 1);
    const uint32_t scale = (uint32_t)std::max<uint64_t>(1, ((uint64_t)levels << 16) / std::max<uint64_t>(top, 1));
    const uint32_t maxbin = (uint32_t)levels - 1;
    const unsigned gc = (unsigned)std::max<int64_t>(1, std::min<int64_t>((nfull + 255) / 256, 2048));
    const unsigned gp = (unsigned)std::min<int64_t>((fp.nloc + 255) / 256, 2048);
    if (nfull > 0) {
        hipLaunchKernelGGL(pilot_chunk_kernel, dim3(gc), dim3(256), 0, stream, fp.pilot_cost, nfull, chunk, ccost);
        hipLaunchKernelGGL(pilot_seg_hist_kernel, dim3((unsigned)nseg), dim3(kSortSeg), 0, stream, ccost, nfull, nseg,
                           scale, maxbin, seghist);
        hipLaunchKernelGGL(pilot_seg_scan_kernel, dim3(kCostBins), dim3(kCostBins), 0, stream, seghist, nseg, total);
        hipLaunchKernelGGL(pilot_scan_kernel, dim3(1), dim3(kCostBins), 0, stream, total, offs);
        hipLaunchKernelGGL(pilot_seg_scatter_kernel, dim3((unsigned)nseg), dim3(kSortSeg), 0, stream, ccost, nfull,
                           nseg, scale, maxbin, seghist, offs, corder);
    }
    hipLaunchKernelGGL(pilot_expand_kernel, dim3(gp), dim3(256), 0, stream, corder, nfull, chunk, fp.nloc, order);
    FrameParams b = fp;
    b.pass = 2;
    if (fp.walk_team == 0 && traversal == TRAV_FAST) {
        // pass 2's team size from the pixels pass 1 left unfinished (pilot_team_pick_kernel)
        static_assert(kTeamOffset >= kGroups * kCounterStride && kTeamOffset + 8 <= kConstOffset, "work block layout");
        unsigned* left = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(d_work) + kTeamOffset);
        int* ts = reinterpret_cast<int*>(left + 1);
        int dev = 0, cus = 0;
        e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e == hipSuccess) e = hipMemsetAsync(left, 0, sizeof(unsigned), stream);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(pilot_team_count_kernel, dim3(gp), dim3(256), 0, stream, fp.pilot_cost, fp.nloc, left);
        // resident lanes of the one-lane BVH2 walk: 4 waves per SIMD
        hipLaunchKernelGGL(pilot_team_pick_kernel, dim3(1), dim3(64), 0, stream, left,
                           (int64_t)std::max(cus, 1) * 4 * 4 * 64, ts);
        b.walk_team_dev = ts;
    }
    return launch_render_pass(sc, b, traversal, block, d_out, nullptr, d_work, stream);
}

hipError_t launch_render_pass(const DevScene& sc, const FrameParams& fp, int traversal, int block, float* d_out,
                         unsigned long long* d_counts, unsigned int* d_work, hipStream_t stream) {
    if (traversal == TRAV_REF) {
        return d_counts ? launch_t<TRAV_REF, true, false>(sc, fp, block, d_out, d_counts, d_work, stream)
                        : launch_t<TRAV_REF, false, false>(sc, fp, block, d_out, d_counts, d_work, stream);
    }
    return d_counts ? launch_fast<true>(sc, fp, block, d_out, d_counts, d_work, stream)
                    : launch_fast<false>(sc, fp, block, d_out, d_counts, d_work, stream);
}

hipError_t launch_rgb8(const float* d_in, uint8_t* d_out, int64_t n, bool gamma, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    // float4 loads and 32-bit stores need 16- and 4-byte alignment (torch / hipMalloc buffers have it)
    if (((uintptr_t)d_in & 15) || ((uintptr_t)d_out & 3)) return hipErrorInvalidValue;
    const int block = 256;
    const int64_t grid = ((n + 3) / 4 + block - 1) / block;
    if (gamma)
        hipLaunchKernelGGL(rgb8_kernel<true>, dim3((unsigned)grid), dim3(block), 0, stream, d_in, d_out, n);
    else
        hipLaunchKernelGGL(rgb8_kernel<false>, dim3((unsigned)grid), dim3(block), 0, stream, d_in, d_out, n);
    return hipGetLastError();
}

hipError_t launch_gamma(const float* d_in, float* d_out, int64_t n, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const int block = 256;
    const int64_t grid = (n + block - 1) / block;
    hipLaunchKernelGGL(gamma_kernel, dim3((unsigned)grid), dim3(block), 0, stream, d_in, d_out, n);
    return hipGetLastError();
}

}  // namespace rt
