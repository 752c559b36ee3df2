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
#include "rt_internal.h"
#include "rtm.h"

namespace rt {

namespace {

constexpr int TRAV_FAST = 0;
constexpr int TRAV_REF = 1;
constexpr int REF_STACK = 20;  // stack.cl:4, Raytracing capacity 20

struct Hit {
    float k;
    int tri;  // < 0: miss
};

struct Cnt {
    unsigned long long nodes, tris, rays, env, dropped;
};

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
        const int curr = stk[top * B];
        --top;
        if (COUNT) c.nodes++;
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
__device__ __forceinline__ void slab(float lo_x, float hi_x, float lo_y, float hi_y, float lo_z, float hi_z,
                                     float ox, float oy, float oz, float ix, float iy, float iz,
                                     float& tmin, float& tmax) {
    const float x0 = (lo_x - ox) * ix, x1 = (hi_x - ox) * ix;
    const float y0 = (lo_y - oy) * iy, y1 = (hi_y - oy) * iy;
    const float z0 = (lo_z - oz) * iz, z1 = (hi_z - oz) * iz;
    tmin = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
    tmax = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
}

constexpr float CULL_MARGIN = 1.0f + 0x1p-12f;

template <bool COUNT>
__device__ __forceinline__ void fast_leaf(const DevScene& S, int t, rtm_f3 o, rtm_f3 d, Hit& best, int& best_rank,
                                          Cnt& c) {
    if (COUNT) c.tris++;
    float k;
    int rank;
    if (mt_test(S.tri_geo, t, o, d, &k, &rank) && k > 0.0001f &&
        (k < best.k || (k == best.k && rank < best_rank))) {
        best.k = k;
        best.tri = t;
        best_rank = rank;
    }
}

template <bool COUNT>
__device__ Hit trace_fast(const DevScene& S, rtm_f3 o, rtm_f3 d, int* __restrict__ stk, int B, Cnt& c) {
    Hit best{1000.0f, -1};
    int best_rank = -1;
    if (COUNT) c.rays++;
    if (S.ntri <= 0) return best;
    const float ix = 1.0f / d.x, iy = 1.0f / d.y, iz = 1.0f / d.z;
    float tmin, tmax;
    slab(S.root_box[0], S.root_box[3], S.root_box[1], S.root_box[4], S.root_box[2], S.root_box[5], o.x, o.y, o.z,
         ix, iy, iz, tmin, tmax);
    if (!(tmax >= tmin && tmax >= 0.0f)) return best;
    if (S.root_ref < 0) {
        fast_leaf<COUNT>(S, ~S.root_ref, o, d, best, best_rank, c);
        return best;
    }
    int node = S.root_ref;
    int sp = 0;
    const float4* __restrict__ nodes = S.nodes;
    while (true) {
        if (COUNT) c.nodes++;
        const float4 a = nodes[4 * node + 0];
        const float4 b = nodes[4 * node + 1];
        const float4 z = nodes[4 * node + 2];
        const float4 e = nodes[4 * node + 3];
        float t0n, t0x, t1n, t1x;
        slab(a.x, a.y, a.z, a.w, z.x, z.y, o.x, o.y, o.z, ix, iy, iz, t0n, t0x);
        slab(b.x, b.y, b.z, b.w, z.z, z.w, o.x, o.y, o.z, ix, iy, iz, t1n, t1x);
        const int r0 = __float_as_int(e.x), r1 = __float_as_int(e.y);
        const float cull = best.k * CULL_MARGIN;
        const bool h0 = t0x >= t0n && t0x >= 0.0f && t0n <= cull;
        const bool h1 = t1x >= t1n && t1x >= 0.0f && t1n <= cull;
        if (h0 && r0 < 0) fast_leaf<COUNT>(S, ~r0, o, d, best, best_rank, c);
        if (h1 && r1 < 0) fast_leaf<COUNT>(S, ~r1, o, d, best, best_rank, c);
        const bool i0 = h0 && r0 >= 0, i1 = h1 && r1 >= 0;
        if (i0 && i1) {
            const bool first0 = t0n <= t1n;
            stk[sp * B] = first0 ? r1 : r0;
            ++sp;
            node = first0 ? r0 : r1;
        } else if (i0) {
            node = r0;
        } else if (i1) {
            node = r1;
        } else {
            if (sp == 0) break;
            --sp;
            node = stk[sp * B];
        }
    }
    return best;
}

template <int TRAV, bool COUNT>
__device__ __forceinline__ Hit trace(const DevScene& S, rtm_f3 o, rtm_f3 d, int* stk, int B, Cnt& c) {
    if (TRAV == TRAV_REF) return trace_ref<COUNT>(S, o, d, stk, B, c);
    return trace_fast<COUNT>(S, o, d, stk, B, c);
}

// ---- camera, Raytracing.cl:18-37 ----
__device__ __forceinline__ void gen_camera_ray(const float* cam, int i, rtm_f3& o, rtm_f3& d) {
    const int W = (int)cam[6];
    const int pixelY = (i + 1) % W;
    const int pixelX = (i - pixelY) / W;
    const rtm_f3 focal = rtm_v3(cam[0], cam[1] - (1.0f / (2.0f * rtm_tan(cam[9] / 2.0f))), cam[2]);
    const rtm_f3 position = rtm_v3(cam[0], cam[1], cam[2]);
    const float pas = 1.0f / cam[6];
    const rtm_f3 pc = rtm_v3(fmaf((float)pixelY, pas, -0.5f), 0.0f, fmaf(-(float)pixelX, pas, 0.5f));
    o = position;
    d = rtm_normalize(rtm_sub(rtm_add(position, pc), focal));
    d = rtm_rotate(cam[3] * (3.14f / 180.0f), rtm_v3(1, 0, 0), d);
    d = rtm_rotate(cam[4] * (3.14f / 180.0f), rtm_v3(0, 1, 0), d);
    d = rtm_rotate(cam[5] * (3.14f / 180.0f), rtm_v3(0, 0, 1), d);
}

// ---- IBL, MathLib.cl:72-90 (integer coords through a linear sampler) ----
template <bool COUNT>
__device__ rtm_f3 sample_ibl(const DevScene& S, rtm_f3 dir, Cnt& c) {
    if (COUNT) c.env++;
    dir = rtm_rotate(90.0f * (3.14f / 180.0f), rtm_v3(1, 0, 0), dir);
    dir = rtm_rotate(90.0f * (3.14f / 180.0f), rtm_v3(0, 1, 0), dir);
    float u = rtm_atan2(dir.z, dir.x), v = rtm_asin(dir.y);
    u = u * 0.1591f;
    v = v * 0.3183f;
    u = u + 0.5f;
    v = v + 0.5f;
    const int W = S.ibl_w, H = S.ibl_h;
    const int x = (int)(u * (float)W);
    const int y = (int)(v * (float)H);
    const int x0 = min(max(x - 1, 0), W - 1), x1 = min(max(x, 0), W - 1);
    const int y0 = min(max(y - 1, 0), H - 1), y1 = min(max(y, 0), H - 1);
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

// ---- samplers, MathLib.cl:313-366 ----
__device__ __forceinline__ rtm_f3 hemi_cosine(rtm_f3 dir, uint32_t* s0, uint32_t* s1, float* invPdf) {
    const float u = rtm_rand(s0, s1);
    const float theta = rtm_rand(s0, s1) * 2.0f * 3.14f;
    const float r = sqrtf(u);
    float st, ct;
    rtm_sincos(theta, &st, &ct);
    const rtm_f3 localV = rtm_v3(r * ct, r * st, sqrtf(rtm_fmax(0.0f, 1.0f - u)));
    rtm_f3 l;
    const float colinear = rtm_fabs(rtm_dot(rtm_normalize(dir), rtm_v3(0.0f, 0.0f, 1.0f)));
    if (colinear == 1.0f) {
        l = rtm_scale(localV, dir.z);
    } else {
        const rtm_f3 axis = rtm_cross(rtm_v3(0, 0, 1), dir);
        const float ang = rtm_acos(rtm_dot(dir, rtm_v3(0, 0, 1)));
        l = rtm_normalize(rtm_rotate(ang, axis, localV));
    }
    *invPdf = 3.14f / (rtm_fmax(rtm_dot(l, dir), 0.0f));
    return l;
}

__device__ __forceinline__ rtm_f3 hemi_uniform(rtm_f3 dir, uint32_t* s0, uint32_t* s1, float* invPdf) {
    const float phi = 2.0f * 3.14f * (rtm_rand(s0, s1));
    const float theta = rtm_acos(1.0f - (rtm_rand(s0, s1)));
    float sp, cp, sth, cth;
    rtm_sincos(phi, &sp, &cp);
    rtm_sincos(theta, &sth, &cth);
    const rtm_f3 localV = rtm_v3(cp * sth, sth * sp, cth);
    rtm_f3 w;
    const float colinear = rtm_fabs(rtm_dot(rtm_normalize(dir), rtm_v3(0.0f, 0.0f, 1.0f)));
    if (colinear == 1.0f) {
        w = rtm_scale(localV, dir.z);
    } else {
        const rtm_f3 axis = rtm_normalize(rtm_cross(rtm_v3(0.0f, 0.0f, 1.0f), dir));
        const float ang = rtm_acos(rtm_dot(dir, rtm_v3(0, 0, 1.0f)));
        w = rtm_rotate(ang, axis, localV);
    }
    *invPdf = 2.0f * 3.14f;
    return w;
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

__device__ __forceinline__ Mat load_mat(const float* __restrict__ m, int idx) {
    const float* p = m + 6 * idx;
    Mat r;
    r.type = (int)p[0];
    r.color = rtm_v3(p[1], p[2], p[3]);
    r.rough = p[4];
    return r;
}

enum Phase { PREP = 0, BOUNCE = 1, SUN = 2 };

__device__ __forceinline__ void log_event(const FrameParams& F, float kind, int j, rtm_f3 o, rtm_f3 d, float k,
                                          int mat, rtm_f3 so) {
    const int n = *F.log_count;
    if (n >= F.log_cap) return;
    float* e = F.log_buf + 16 * n;
    e[0] = kind; e[1] = (float)j; e[2] = o.x; e[3] = o.y; e[4] = o.z; e[5] = d.x; e[6] = d.y; e[7] = d.z;
    e[8] = k; e[9] = (float)mat; e[10] = so.x; e[11] = so.y; e[12] = so.z; e[13] = 0; e[14] = 0; e[15] = 0;
    *F.log_count = n + 1;
}

template <int TRAV, bool COUNT, bool LOG = false>
__global__ void __launch_bounds__(256) render_kernel(DevScene S, FrameParams F, float* __restrict__ out,
                                                     unsigned long long* __restrict__ counts) {
    extern __shared__ int lds_stack[];
    const int B = blockDim.x;
    int* stk = lds_stack + threadIdx.x;
    Cnt c{0, 0, 0, 0, 0};
    const int64_t p = (int64_t)blockIdx.x * B + threadIdx.x;
    bool active = p < F.nloc;
    int i = 0;
    if (active) {
        const int64_t krow = p / F.width;
        const int64_t col = p - krow * F.width;
        const int64_t i64 = ((int64_t)F.row0 + krow * F.row_step) * F.width + col;
        active = i64 < F.npix;
        i = (int)i64;
    }
    const bool logme = LOG && active && i == F.log_pixel;
    if (active) {
        const int imgSize = (int)F.npix;
        uint32_t seed0 = (uint32_t)(i % imgSize);
        uint32_t seed1 = (uint32_t)(i / imgSize);
        const float e3 = F.env[3], e4 = F.env[4];

        rtm_f3 co, cd;
        gen_camera_ray(F.cam, i, co, cd);
        const Hit hc = trace<TRAV, COUNT>(S, co, cd, stk, B, c);
        const bool hitc = hc.tri >= 0;
        rtm_f3 nc = rtm_v3(0, 0, 0);
        int mc = 0;
        if (hitc) {
            const float4 sh = S.tri_shade[hc.tri];
            nc = xyz(sh);
            mc = __float_as_int(sh.w);
        }
        // sun direction (Raytracing.cl:115-118), unnormalised
        rtm_f3 sun = rtm_v3(1, 1, 1);
        sun = rtm_rotate(F.env[0] * (3.14f / 180.0f), rtm_v3(1, 0, 0), sun);
        sun = rtm_rotate(F.env[1] * (3.14f / 180.0f), rtm_v3(0, 1, 0), sun);
        sun = rtm_rotate(F.env[2] * (3.14f / 180.0f), rtm_v3(0, 0, 1), sun);

        // path state: the reference's (R_cam, H_cam, camMat, j, sampleOut)
        rtm_f3 Ro = co, Rd = cd, n = nc, so = rtm_v3(1, 1, 1);
        bool hit = hitc;
        float k = hc.k;
        int mid = mc, j = 0;
        rtm_f3 Bo = rtm_v3(0, 0, 0), Bd = rtm_v3(0, 0, 0);  // pending bounce ray
        rtm_f3 acc = rtm_v3(0, 0, 0);
        int s = 0;
        int phase = PREP;
        const int spp = F.spp, maxB = F.max_bounce;

        while (s < spp) {
            if (phase == PREP) {
                bool done = true;
                if (j > maxB) {
                    // loop of naiveGI never entered (maxBounce < 0): sample stays 1
                } else if (!hit) {
                    so = rtm_scale(rtm_mul(so, sample_ibl<COUNT>(S, Rd, c)), e4);
                } else {
                    const Mat cm = load_mat(S.mat, mid);
                    if (cm.type == 0) {
                        so = rtm_scale(so, cm.rough);
                    } else {
                        float invPdf = 0.0f;
                        rtm_f3 brdf = rtm_v3(0, 0, 0);
                        if (cm.type == 1) {
                            Bd = hemi_cosine(n, &seed1, &seed0, &invPdf);
                            brdf = rtm_scale(cm.color, 1.0f / 3.14f);
                        } else if (cm.type == 2) {
                            Bd = hemi_uniform(n, &seed1, &seed0, &invPdf);
                            brdf = brdf_ggx(cm.color, cm.rough, rtm_scale(Rd, -1.0f), Bd, n);
                        } else {
                            Bd = Rd;
                            brdf = cm.color;
                            invPdf = 1.0f / rtm_fabs(rtm_dot(Bd, rtm_normalize(n)));
                        }
                        const rtm_f3 nd = rtm_normalize(Rd);
                        Bo = rtm_v3(fmaf(nd.x, k, Ro.x), fmaf(nd.y, k, Ro.y), fmaf(nd.z, k, Ro.z));
                        // attenuation only depends on pre-trace values: apply now
                        const float att = invPdf * rtm_fabs(rtm_dot(Bd, rtm_normalize(n)));
                        so = rtm_scale(rtm_mul(so, brdf), att);
                        phase = BOUNCE;
                        done = false;
                    }
                }
                if (done) {
                    if (LOG && logme) log_event(F, 3.0f, s + 1, rtm_v3(0, 0, 0), rtm_v3(0, 0, 0), 0.0f, 0, so);
                    acc = rtm_add(acc, so);
                    ++s;
                    Ro = co; Rd = cd; n = nc; hit = hitc; k = hc.k; mid = mc; j = 0;
                    so = rtm_v3(1, 1, 1);
                    continue;
                }
            }
            // one ray per lane per iteration
            const rtm_f3 td = (phase == BOUNCE) ? Bd : sun;
            const Hit h = trace<TRAV, COUNT>(S, Bo, td, stk, B, c);
            bool finish = false;
            if (LOG && logme) {
                const int hm = h.tri >= 0 ? __float_as_int(S.tri_shade[h.tri].w) : 0;
                log_event(F, phase == BOUNCE ? 1.0f : 2.0f, j, Bo, td, h.tri >= 0 ? h.k : -1.0f, hm, so);
            }
            if (phase == BOUNCE) {
                if (h.tri >= 0) {
                    const float4 sh = S.tri_shade[h.tri];
                    Ro = Bo; Rd = Bd; hit = true; k = h.k; n = xyz(sh); mid = __float_as_int(sh.w);
                    const Mat bm = load_mat(S.mat, mid);
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
                } else {
                    phase = SUN;
                }
            } else {
                rtm_f3 sunLight = rtm_v3(0, 0, 0);
                const Mat cm = load_mat(S.mat, mid);
                if (h.tri < 0 && cm.type != 3) sunLight = rtm_v3(e3, e3, e3);
                if (h.tri >= 0) {
                    const float4 sh = S.tri_shade[h.tri];
                    const Mat sm = load_mat(S.mat, __float_as_int(sh.w));
                    if (sm.type == 3) sunLight = rtm_scale(sm.color, e3);
                }
                const rtm_f3 envLight = rtm_scale(sample_ibl<COUNT>(S, Bd, c), e4);
                so = rtm_mul(so, rtm_add(sunLight, envLight));
                finish = true;
            }
            if (finish) {
                if (LOG && logme) log_event(F, 3.0f, s + 1, rtm_v3(0, 0, 0), rtm_v3(0, 0, 0), 0.0f, 0, so);
                acc = rtm_add(acc, so);
                ++s;
                Ro = co; Rd = cd; n = nc; hit = hitc; k = hc.k; mid = mc; j = 0;
                so = rtm_v3(1, 1, 1);
                phase = PREP;
            }
        }
        const rtm_f3 o = rtm_div(acc, (float)spp);
        float* dst = out + 3 * p;
        dst[0] = rtm_fmax(rtm_fmin(o.x, 1.0f), 0.0f);
        dst[1] = rtm_fmax(rtm_fmin(o.y, 1.0f), 0.0f);
        dst[2] = rtm_fmax(rtm_fmin(o.z, 1.0f), 0.0f);
    }
    if (COUNT) {
        unsigned long long v[5] = {c.nodes, c.tris, c.rays, c.env, c.dropped};
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            unsigned long long x = v[q];
            for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
            if ((threadIdx.x & 63) == 0 && x) atomicAdd(&counts[q], x);
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

template <int TRAV, bool COUNT>
hipError_t launch_t(const DevScene& sc, const FrameParams& fp, int block, float* d_out, unsigned long long* d_counts,
                    hipStream_t stream) {
    const int depth = (TRAV == TRAV_REF) ? REF_STACK : (sc.depth > 0 ? sc.depth : 1);
    const size_t lds = (size_t)depth * block * sizeof(int);
    const int64_t grid = (fp.nloc + block - 1) / block;
    if (grid <= 0) return hipSuccess;
    hipLaunchKernelGGL((render_kernel<TRAV, COUNT>), dim3((unsigned)grid), dim3(block), lds, stream, sc, fp, d_out,
                       d_counts);
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
    Cnt c{0, 0, 0, 0, 0};
    const float* r = rays + 6 * t;
    const Hit h = trace<TRAV, false>(S, rtm_v3(r[3], r[4], r[5]), rtm_v3(r[0], r[1], r[2]),
                                     lds_stack + threadIdx.x, blockDim.x, c);
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
                            hipStream_t stream) {
    const int block = 64;
    const int depth = traversal == TRAV_REF ? REF_STACK : (sc.depth > 0 ? sc.depth : 1);
    const size_t lds = (size_t)depth * block * sizeof(int);
    const int64_t grid = (fp.nloc + block - 1) / block;
    if (traversal == TRAV_REF)
        hipLaunchKernelGGL((render_kernel<TRAV_REF, false, true>), dim3((unsigned)grid), dim3(block), lds, stream, sc,
                           fp, d_out, nullptr);
    else
        hipLaunchKernelGGL((render_kernel<TRAV_FAST, false, true>), dim3((unsigned)grid), dim3(block), lds, stream,
                           sc, fp, d_out, nullptr);
    return hipGetLastError();
}

hipError_t launch_debug_trace(const DevScene& sc, int traversal, const float* rays, float* out, int64_t n,
                              hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const int block = 128;
    const int depth = traversal == TRAV_REF ? REF_STACK : (sc.depth > 0 ? sc.depth : 1);
    const size_t lds = (size_t)depth * block * sizeof(int);
    if (traversal == TRAV_REF)
        hipLaunchKernelGGL(debug_trace_kernel<TRAV_REF>, dim3((unsigned)((n + block - 1) / block)), dim3(block), lds,
                           stream, sc, rays, out, n);
    else
        hipLaunchKernelGGL(debug_trace_kernel<TRAV_FAST>, dim3((unsigned)((n + block - 1) / block)), dim3(block), lds,
                           stream, sc, rays, out, n);
    return hipGetLastError();
}

hipError_t launch_render(const DevScene& sc, const FrameParams& fp, int traversal, int block, float* d_out,
                         unsigned long long* d_counts, hipStream_t stream) {
    if (traversal == TRAV_REF) {
        return d_counts ? launch_t<TRAV_REF, true>(sc, fp, block, d_out, d_counts, stream)
                        : launch_t<TRAV_REF, false>(sc, fp, block, d_out, d_counts, stream);
    }
    return d_counts ? launch_t<TRAV_FAST, true>(sc, fp, block, d_out, d_counts, stream)
                    : launch_t<TRAV_FAST, false>(sc, fp, block, d_out, d_counts, stream);
}

hipError_t launch_gamma(const float* d_in, float* d_out, int64_t n, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const int block = 256;
    const int64_t grid = (n + block - 1) / block;
    hipLaunchKernelGGL(gamma_kernel, dim3((unsigned)grid), dim3(block), 0, stream, d_in, d_out, n);
    return hipGetLastError();
}

}  // namespace rt
