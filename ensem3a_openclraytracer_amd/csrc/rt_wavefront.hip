// Wavefront tree walk (option "wavefront"): the per-pixel path tracer of Raytracing.cl:39-221 with
// shading split from traversal, for the tree walks (BVH2 item steps and the 4-wide layout).
//
// The per-lane megakernel (rt_kernels.hip render_resume_kernel) keeps every lane's path state AND
// its ray's traversal state in registers.  Lanes shade while other lanes of the wave are mid-walk,
// so the traversal registers stay live across the shading code: the 4-wide walk (C5) holds 72 VGPRs
// at 7 waves per SIMD and spills ~40 of them around shading -- two thirds of its memory traffic
//  -- and lanes whose ray is done wait for the wave's next shading round
// (resume_min: a traversal step finds work for ~70 % of the lanes).
//
// Here each persistent wave owns 64 * K path slots (K = FrameParams::wf_slots) whose state lives in
// HBM, in the wave's own region (SoA planes, lane-consecutive: every access is one coalesced
// 256-byte row per plane), and alternates two phases:
//   shade  -- in sub-rounds of 64 paths, read each path's state and the hit of the ray it traced,
//             run naiveGI's logic (Raytracing.cl:46-151) until the path needs its next ray (bounce,
//             shadow or, for a new pixel, camera ray), take new pixels for finished ones (one atomic
//             per wave, rt_device.h take_pixel), and append every live path -- ballot + mbcnt prefix,
//             no atomics -- to the wave's compacted ray queue together with its state;
//   trace  -- walk the queue's rays: a lane whose ray is done takes the next queued ray at once
//             (ballot + prefix over the idle lanes), so every lane traces until the queue is empty;
//             each result (distance, triangle) is written beside its ray.
// Only traversal state is live in the trace phase and only path state in the shade phase, so the
// kernel runs 8 waves per SIMD without scratch.  Every path keeps exactly one ray in flight and the
// shading code is the megakernel's, in the same order per pixel: the RNG chain and the sample order
// are unchanged and frames are bit-identical to the megakernel's (and, through it, to the oracle).
// Paths are compacted in place (a live path moves to a queue position <= its old one), so the state
// rows of paths that did not move are rewritten only where they changed.
#include <cstddef>

#include "rt_device.h"

namespace rt {

namespace {

// state planes (one float / int per path each), the wave's region = planes | rays 0 | rays 1 | hits
enum WfPlane {
    WF_FL = 0,      // phase | drew << 3 | fdb << 4 | pre << 5 | j << 8
    WF_P,           // tile pixel index
    WF_S0, WF_S1,   // the pixel's RNG words (Raytracing.cl:171-172)
    WF_SM,          // samples done
    WF_TR,          // triangle of the current surface (naiveGI hitInfo)
    WF_SO,          // sample colour (3 planes)
    WF_KC = WF_SO + 3,   // cached camera hit distance / triangle (Raytracing.cl:184-187)
    WF_TC,
    WF_SC,          // the first drawing bounce's shadow-ray hit (sun_cache)
    WF_CORE,
    // BVH2 walk: the deterministic glass prefix of the pixel's samples (render_resume_kernel PREFIX)
    WF_PJ = WF_CORE, WF_PT, WF_PSO, WF_PO = WF_PSO + 3, WF_PD = WF_PO + 3, WF_PK = WF_PD + 3,
    WF_ALL
};
constexpr int wf_planes(bool prefix) { return prefix ? (int)WF_ALL : (int)WF_CORE; }
// per queue entry besides the planes: ray (o.xyz d.x | d.yz flags -) 32 B + hit (k, triangle) 8 B
constexpr int kWfEntryBytes = 40;
#ifndef RT_WF_WAVES
#define RT_WF_WAVES 8
#endif
constexpr int kWfWaves = RT_WF_WAVES;
// LDS stack entries per lane: the CU's 160 KB over its lanes (8 waves per SIMD x 4 SIMDs x 64 lanes x 10 x
// 8 B; 20 entries at 4 waves)
constexpr int kStackLdsWave = 80 / kWfWaves;
constexpr int SUN_UNKNOWN = -2;
// dirty bits: state rows rewritten in place only where they changed
constexpr unsigned D_P = 1, D_SEED = 2, D_SM = 4, D_KCTC = 8, D_SUNC = 16;

__device__ __forceinline__ int as_i(float f) { return __float_as_int(f); }
__device__ __forceinline__ float as_f(int i) { return __int_as_float(i); }

// Every load of a shade sub-round has returned before its first store: a path written to queue
// position pos may overwrite the row another lane of the wave read at q = pos in this sub-round.
__device__ __forceinline__ void wait_loads() { __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// The kernel's parameters (scene, frame, launch constants) as one struct, laid out as the kernel
// argument segment lays them out (each argument at its natural alignment, in order)
struct WfArgs {
    DevScene S;
    FrameParams F;
    LaunchConst C;
};
// the kernel argument segment puts each argument at the next offset of its alignment: the same offsets
// as WfArgs (checked against the code object's argument metadata by tests/test_native_abi.py)
constexpr size_t wf_align(size_t x, size_t a) { return (x + a - 1) / a * a; }
static_assert(offsetof(WfArgs, F) == wf_align(sizeof(DevScene), alignof(FrameParams)), "kernarg layout");
static_assert(offsetof(WfArgs, C) == wf_align(offsetof(WfArgs, F) + sizeof(FrameParams), alignof(LaunchConst)),
              "kernarg layout");

// RT_WF_OPAQUE: the parameters are re-read (scalar loads from the kernel argument segment, through a
// pointer the compiler cannot see through) at the start of every shade sub-round and trace phase, so
// that the values only one phase uses are not held in SGPRs across the other (SGPR spills into VGPR lanes)
#ifndef RT_WF_OPAQUE
#define RT_WF_OPAQUE 1
#endif
#if RT_WF_OPAQUE
typedef const char __attribute__((address_space(4))) kernarg_char;
#define WF_REFRESH_PARAMS                                                                         \
    kernarg_char* kap_ = (kernarg_char*)__builtin_amdgcn_kernarg_segment_ptr();                     \
    __asm__ volatile("" : "+s"(kap_));                                                             \
    const WfArgs& wa_ = *(const WfArgs*)kap_;                                                      \
    const DevScene& S = wa_.S;                                                                     \
    const FrameParams& F = wa_.F;                                                                  \
    const LaunchConst& C = wa_.C;                                                                  \
    (void)S; (void)F; (void)C;
#else
#define WF_REFRESH_PARAMS
#endif

template <bool COUNT, bool OVF, bool WIDE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kWfWaves)))
wave_kernel(DevScene S, FrameParams F, LaunchConst C, float* __restrict__ out, unsigned long long* __restrict__ counts,
            unsigned int* __restrict__ work_counter) {
    constexpr bool PREFIX = !WIDE;
    constexpr int NPL = wf_planes(PREFIX);
    extern __shared__ int lds_stack[];
    Cnt c{};
    const int lane = threadIdx.x & 63;
    const unsigned SW = 64u * (unsigned)F.wf_slots;   // paths of this wave
    // the wave's index, wave-uniform (readfirstlane: its region's pointers live in SGPRs)
    const unsigned wave = (unsigned)__builtin_amdgcn_readfirstlane((int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6));
    char* const region = reinterpret_cast<char*>(F.wf_buf) + (size_t)wave * SW * (4 * NPL + kWfEntryBytes);
    float* const pl = reinterpret_cast<float*>(region);
    float4* const rb0 = reinterpret_cast<float4*>(region + (size_t)SW * 4 * NPL);
    float4* const rb1 = rb0 + SW;
    float2* const hb = reinterpret_cast<float2*>(rb1 + SW);
    // state rows, ray records and hits: streamed once per phase, read back one phase later
    auto PL = [&](int f, unsigned q) -> float { return pl[(unsigned)f * SW + q]; };
    auto PS = [&](int f, unsigned q, float v) { pl[(unsigned)f * SW + q] = v; };

    PixelQueue pq;
    pq.per = (F.handout && F.pass != 2) ? (unsigned)((F.nloc + kGroups - 1) / kGroups) : 0u;   // pass 2: cost order, interleaved
    unsigned n = SW;     // queue entries (wave-uniform); the first shade phase: every slot takes a pixel
    bool first = true;
    while (true) {
        // ================= shade phase =================
        const unsigned long long t_shade = COUNT ? clock64() : 0;
        unsigned nout = 0;
        for (unsigned r0 = 0; r0 < n; r0 += 64) {
            WF_REFRESH_PARAMS
            const int W = F.width;
            const int imgSize = (int)F.npix;
            const float e3 = F.env[3], e4 = F.env[4];
            const int spp = F.spp, maxB = F.max_bounce;
            const unsigned nloc = (unsigned)F.nloc;
            auto global_pixel = [&](int p) -> int64_t {
                const int krow = p / W;
                return ((int64_t)F.row0 + (int64_t)krow * F.row_step) * W + (p - krow * W);
            };
            if (COUNT && lane == 0) c.wave_outer++;
            const unsigned q = r0 + (unsigned)lane;
            const bool valid = q < n;
            int phase = valid ? FETCH : DONE;
            unsigned dirty = 0;
            int p = 0, s = 0, tri = -1, j = 0, tc = -1, sun_c = SUN_UNKNOWN, ht = -1;
            uint32_t seed0 = 0, seed1 = 0;
            bool drew = false, fdb = false, pre = false;
            float kc = 1000.0f, hk = 1000.0f;
            rtm_f3 so = rtm_v3(1, 1, 1);
            rtm_f3 ro = rtm_v3(0, 0, 0), rd = rtm_v3(0, 0, 1);
            if (!first && valid) {
                const unsigned fl = (unsigned)as_i(PL(WF_FL, q));
                phase = (int)(fl & 7u);
                drew = (fl >> 3) & 1u;
                fdb = (fl >> 4) & 1u;
                pre = (fl >> 5) & 1u;
                j = (int)(fl >> 8);
                p = as_i(PL(WF_P, q));
                seed0 = (uint32_t)as_i(PL(WF_S0, q));
                seed1 = (uint32_t)as_i(PL(WF_S1, q));
                s = as_i(PL(WF_SM, q));
                tri = as_i(PL(WF_TR, q));
                so = rtm_v3(PL(WF_SO, q), PL(WF_SO + 1, q), PL(WF_SO + 2, q));
                kc = PL(WF_KC, q);
                tc = as_i(PL(WF_TC, q));
                sun_c = as_i(PL(WF_SC, q));
                const float4 a = rb0[q], b = rb1[q];
                ro = rtm_v3(a.x, a.y, a.z);
                rd = rtm_v3(a.w, b.x, b.y);   // a shadow ray keeps the bounce direction here (its own is C.sun)
                const float2 h = hb[q];
                hk = h.x;
                ht = as_i(h.y);
            }
            // The pixel's sum is kept in its output row (out[3 p .. 3 p + 2], zeroed when the pixel is taken):
            // the same float additions in the same order as the megakernel's register sum
            auto add_samples = [&](int reps) __attribute__((always_inline)) {
                float* const o3 = out + 3 * (int64_t)p;
                rtm_f3 acc = rtm_v3(o3[0], o3[1], o3[2]);
                for (int r = 0; r < reps; ++r) acc = rtm_add(acc, so);
                if (s + reps >= spp) acc = rtm_div(acc, (float)spp);   // the mean + clamp of store_pixel
                o3[0] = s + reps >= spp ? rtm_fmax(rtm_fmin(acc.x, 1.0f), 0.0f) : acc.x;
                o3[1] = s + reps >= spp ? rtm_fmax(rtm_fmin(acc.y, 1.0f), 0.0f) : acc.y;
                o3[2] = s + reps >= spp ? rtm_fmax(rtm_fmin(acc.z, 1.0f), 0.0f) : acc.z;
            };
            // output += baseColor; the next sample restarts from the cached camera hit (or after the
            // deterministic prefix, read back from the path's row): render_resume_kernel finish_sample.
            // reps > 1: the repeats of a sample that drew no random number (fixed_point) added with it
            auto finish_sample = [&](int reps) __attribute__((always_inline)) {
                add_samples(reps);
                if (COUNT) c.samples += (unsigned long long)reps;
                s += reps;
                dirty |= D_SM;
                phase = s >= spp ? FETCH : PREP;
                tri = tc; j = 0;
                so = rtm_v3(1, 1, 1);
                drew = false;
                if (PREFIX && pre) {
                    tri = as_i(PL(WF_PT, q)); j = as_i(PL(WF_PJ, q));
                    so = rtm_v3(PL(WF_PSO, q), PL(WF_PSO + 1, q), PL(WF_PSO + 2, q));
                    ro = rtm_v3(PL(WF_PO, q), PL(WF_PO + 1, q), PL(WF_PO + 2, q));
                    rd = rtm_v3(PL(WF_PD, q), PL(WF_PD + 1, q), PL(WF_PD + 2, q));
                    hk = PL(WF_PK, q);
                }
            };
            // a sample that drew no random number is every later sample of its pixel (fixed_point)
            auto end_sample = [&]() __attribute__((always_inline)) {
                finish_sample(F.fixed_point && !drew ? max(spp - s, 1) : 1);
            };

            // -- the traced ray's result (Raytracing.cl:184-187, 92-137) --
            bool sun_now = false;
            int hs = -1;
            if (phase == PRIMARY) {
                tc = ht;
                kc = hk;
                dirty |= D_KCTC;
                tri = tc; j = 0;
                so = rtm_v3(1, 1, 1);
                drew = false;
                phase = PREP;
            } else if (phase == BOUNCE) {
                if (ht >= 0) {
                    tri = ht;
                    const Mat bm = load_mat(S.mat, __float_as_int(S.tri_shade[ht].w));
                    if (bm.type != 0) {
                        if (j == maxB) {
                            so = rtm_v3(0, 0, 0);
                            end_sample();
                        } else {
                            ++j;
                            phase = PREP;
                        }
                    } else {
                        so = rtm_scale(so, bm.rough);
                        end_sample();
                    }
                } else if (F.sun_skip) {
                    sun_now = true;   // unlit sun: the term with the bounce ray's miss (FrameParams::sun_skip)
                } else if (fdb && sun_c != SUN_UNKNOWN) {
                    sun_now = true;   // the first drawing bounce's shadow ray, traced in an earlier sample
                    hs = sun_c;
                } else {
                    phase = SUN;      // shadow ray towards the sun from the bounce origin (Raytracing.cl:115-124)
                }
            } else if (phase == SUN) {
                sun_now = true;
                hs = ht;
            }
            if (sun_now) {   // Raytracing.cl:125-137
                rtm_f3 sunLight = rtm_v3(0, 0, 0);
                if (COUNT) c.sun++;
                if (fdb) {
                    sun_c = hs;
                    dirty |= D_SUNC;
                }
                const Mat cm = load_mat(S.mat, __float_as_int(S.tri_shade[tri].w));
                if (hs < 0 && cm.type != 3) sunLight = rtm_v3(e3, e3, e3);
                if (hs >= 0) {
                    const Mat sm = load_mat(S.mat, __float_as_int(S.tri_shade[hs].w));
                    if (sm.type == 3) sunLight = rtm_scale(sm.color, e3);
                }
                const rtm_f3 envLight = rtm_scale(sample_ibl_if<COUNT>(S, C, rd, e4, c), e4);
                so = rtm_mul(so, rtm_add(sunLight, envLight));
                end_sample();
            }
            // -- naiveGI loop heads (Raytracing.cl:46-79) until a ray is needed or the pixel is done --
            while (phase == PREP) {
                const bool cam = j == 0;
                const rtm_f3 Ro = cam ? C.position : ro;
                const rtm_f3 Rd = cam ? camera_dir(C, W, (int)global_pixel(p)) : rd;
                const float k = cam ? kc : hk;
                if (j > maxB) {
                    end_sample();   // naiveGI's loop never entered (maxBounce < 0): the sample stays 1
                } else if (tri < 0) {
                    so = rtm_scale(rtm_mul(so, sample_ibl_if<COUNT>(S, C, Rd, e4, c)), e4);
                    end_sample();
                } else {
                    const float4 sh = S.tri_shade[tri];
                    const rtm_f3 nrm = xyz(sh);
                    const Mat cm = load_mat(S.mat, __float_as_int(sh.w));
                    if (cm.type == 0) {
                        so = rtm_scale(so, cm.rough);
                        end_sample();
                    } else {
                        const float4 f2 = S.tri_frame[3 * tri + 2];
                        const rtm_f3 nn = xyz(f2);
                        float invPdf = 0.0f;
                        rtm_f3 brdf = rtm_v3(0, 0, 0);
                        if (COUNT) count_event(c, cm.type);
                        if (PREFIX && F.fixed_point && cm.type != 3 && !drew && j > 0 && !pre) {
                            // the first bounce of the sample that draws, reached through glass only: its
                            // state goes to the path's row now (read back at every later sample start)
                            pre = true;
                            PS(WF_PJ, q, as_f(j)); PS(WF_PT, q, as_f(tri));
                            PS(WF_PSO, q, so.x); PS(WF_PSO + 1, q, so.y); PS(WF_PSO + 2, q, so.z);
                            PS(WF_PO, q, ro.x); PS(WF_PO + 1, q, ro.y); PS(WF_PO + 2, q, ro.z);
                            PS(WF_PD, q, rd.x); PS(WF_PD + 1, q, rd.y); PS(WF_PD + 2, q, rd.z);
                            PS(WF_PK, q, hk);
                        }
                        fdb = F.sun_cache && cm.type != 3 && !drew && !F.sun_skip;
                        drew = drew || cm.type != 3;
                        rtm_f3 Bd;
                        if (cm.type != 3) {   // diffuse (1) or glossy (2): one sampler stream for both
                            dirty |= D_SEED;
                            Bd = hemi_sample(cm.type == 1, nrm, S.tri_frame[3 * tri], S.tri_frame[3 * tri + 1], f2,
                                             &seed1, &seed0, &invPdf);
                            if (cm.type == 1) brdf = rtm_scale(cm.color, 1.0f / 3.14f);
                            else brdf = brdf_ggx(cm.color, cm.rough, rtm_scale(Rd, -1.0f), Bd, nrm);
                        } else {
                            Bd = Rd;
                            brdf = cm.color;
                            invPdf = 1.0f / rtm_fabs(rtm_dot(Bd, nn));
                        }
                        const rtm_f3 nd = rtm_normalize(Rd);
                        ro = rtm_v3(fmaf(nd.x, k, Ro.x), fmaf(nd.y, k, Ro.y), fmaf(nd.z, k, Ro.z));
                        rd = Bd;
                        // attenuation depends only on pre-trace values (Raytracing.cl:86-87): apply now
                        const float att = invPdf * rtm_fabs(rtm_dot(Bd, nn));
                        so = rtm_scale(rtm_mul(so, brdf), att);
                        phase = BOUNCE;
                    }
                }
            }
            // -- new pixels for the paths that finished theirs (the whole wave takes part) --
            const unsigned long long need = __ballot(phase == FETCH);
            if (need) {
                const unsigned qq = take_pixel(pq, need, lane, work_counter, nloc, lane);
                if (phase == FETCH) {
                    phase = DONE;
                    if (qq < nloc) {
                        const int64_t i64 = global_pixel((int)qq);
                        if (i64 < F.npix) {
                            const int i = (int)i64;
                            p = (int)qq;
                            seed0 = (uint32_t)(i % imgSize);
                            seed1 = (uint32_t)(i / imgSize);
                            s = 0;
                            float* const o3 = out + 3 * (int64_t)p;
                            o3[0] = 0.0f; o3[1] = 0.0f; o3[2] = 0.0f;
                            pre = false;
                            sun_c = SUN_UNKNOWN;
                            ro = C.position;
                            rd = camera_dir(C, W, i);
                            phase = PRIMARY;
                            dirty |= D_P | D_SEED | D_SM | D_SUNC;
                        }
                    }
                }
            }
            // -- append the live paths to the queue (in place: pos <= q) --
            const bool live = phase == PRIMARY || phase == BOUNCE || phase == SUN;
            const unsigned long long m = __ballot(live);
            const unsigned pos = lane_prefix(m, nout);
            const bool moved = pos != q;
            const bool copy_pre = PREFIX && live && moved && pre;
            wait_loads();
            if (live) {
                const unsigned fl = (unsigned)phase | (drew ? 8u : 0u) | (fdb ? 16u : 0u) | (pre ? 32u : 0u) |
                                    ((unsigned)j << 8);
                rb0[pos] = make_float4(ro.x, ro.y, ro.z, rd.x);
                rb1[pos] = make_float4(rd.y, rd.z, as_f(phase == SUN ? 1 : 0), 0.0f);
                PS(WF_FL, pos, as_f((int)fl));
                PS(WF_TR, pos, as_f(tri));
                PS(WF_SO, pos, so.x); PS(WF_SO + 1, pos, so.y); PS(WF_SO + 2, pos, so.z);
                if (moved || (dirty & D_P)) PS(WF_P, pos, as_f(p));
                if (moved || (dirty & D_SEED)) {
                    PS(WF_S0, pos, as_f((int)seed0));
                    PS(WF_S1, pos, as_f((int)seed1));
                }
                if (moved || (dirty & D_SM)) PS(WF_SM, pos, as_f(s));
                if (moved || (dirty & D_KCTC)) {
                    PS(WF_KC, pos, kc);
                    PS(WF_TC, pos, as_f(tc));
                }
                if (moved || (dirty & D_SUNC)) PS(WF_SC, pos, as_f(sun_c));
            }
            // a moved path's glass prefix goes to its new row plane by plane: every lane's read of a plane
            // returns before any lane writes that plane (the other planes are not touched in between)
            if (copy_pre) {
                for (int f = 0; f < 12; ++f) {
                    const float v = PL(WF_PJ + f, q);
                    wait_loads();
                    PS(WF_PJ + f, pos, v);
                }
            }
            nout += (unsigned)__popcll(m);
        }
        first = false;
        n = nout;
        if (n == 0) break;

        // ================= trace phase =================
        WF_REFRESH_PARAMS
        const LaneStack lst = lane_stack(S, lds_stack);
        const char* const nb = reinterpret_cast<const char*>(WIDE ? S.wnodes : S.nodes);
        const char* const tb = reinterpret_cast<const char*>(WIDE ? S.wleaves : S.tri_fast);
        const unsigned long long t_trace = COUNT ? clock64() : 0;
        if (COUNT && lane == 0) c.cyc_shade += t_trace - t_shade;
        FastRay T;
        T.item = 0; T.soff = 0; T.bk = 1000.0f; T.bt = -1; T.brank = -1; T.any = false;
        T.o = rtm_v3(0, 0, 0); T.d = rtm_v3(0, 0, 1); T.ix = T.iy = T.iz = 0.0f;
        bool tracing = false;
        unsigned myq = 0;
        unsigned next = 0;   // queue entries handed out (wave-uniform)
        while (true) {
            // refill the idle lanes from the queue once at least F.wf_refill of them are idle (a refill costs
            // the wave a memory round trip for the rays before their first step), or when the queue's
            // rest fits them, or when no lane traces
            const unsigned long long idle = __ballot(!tracing);
            const unsigned ni = (unsigned)__popcll(idle);
            if (idle && next < n && (ni >= (unsigned)F.wf_refill || n - next <= ni || ni == 64u)) {
                const unsigned qq = lane_prefix(idle, next);
                if (!tracing && qq < n) {
                    myq = qq;
                    const float4 a = rb0[qq], b = rb1[qq];
                    const bool sun = as_i(b.z) != 0;
                    tracing = !fast_init<COUNT>(S, T, rtm_v3(a.x, a.y, a.z), sun ? C.sun : rtm_v3(a.w, b.x, b.y), c);
                    if (WIDE) T.item = S.wroot_ref;
                    T.any = sun && F.sun_any != 0;
                    if (!tracing) hb[qq] = make_float2(T.bk, as_f(-1));
                }
                next += (unsigned)__popcll(idle);
            }
            if (!__any(tracing)) {
                if (next >= n) break;
                continue;
            }
            if (tracing) {
                const bool done = WIDE ? wide_step<COUNT, OVF>(T, nb, tb, lst, c)
                                       : fast_step<COUNT, false, OVF>(S, T, nb, tb, lst, 16u, c);
                if (done) {
                    tracing = false;
                    hb[myq] = make_float2(T.bk, as_f(T.bt >= 0 ? (int)((unsigned)T.bt / 48u) : -1));
                }
            }
        }
        if (COUNT && lane == 0) c.cyc_trav += clock64() - t_trace;
    }
    if (COUNT) {
        unsigned long long v[NCOUNTS] = {c.nodes, c.tris, c.rays, c.env, c.dropped, c.wave_trav, c.wave_outer,
                                          c.cyc_shade, c.cyc_trav, c.boxes, c.diffuse, c.glossy, c.glass,
                                          c.sun, c.samples};
#pragma unroll
        for (int k = 0; k < NCOUNTS; ++k) {
            unsigned long long x = v[k];
            for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
            if (lane == 0 && x) atomicAdd(&counts[k], x);
        }
    }
}

template <bool COUNT, bool OVF, bool WIDE>
const void* wave_fn() {
    return (const void*)wave_kernel<COUNT, OVF, WIDE>;
}

bool wide_walk(const DevScene& sc, const FrameParams& fp) { return fp.wide && sc.wnodes; }

// Upper bound of the persistent grid (blocks): every CU at kWfWaves waves per SIMD, no more waves
// than the tile needs to give every path slot a pixel at the start
int64_t wf_grid_bound(const FrameParams& fp, int block, int cus) {
    const int64_t per_cu = std::max(1, kWfWaves * 4 * 64 / block);
    const int64_t slots_per_block = (int64_t)block * std::max(fp.wf_slots, 1);
    const int64_t need = (fp.nloc + slots_per_block - 1) / slots_per_block;
    return std::max<int64_t>(1, std::min<int64_t>((int64_t)std::max(cus, 1) * per_cu, need));
}

int device_cus() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 1;
    return std::max(cus, 1);
}

}  // namespace

bool wavefront_eligible(const DevScene& sc, const FrameParams& fp) {
    const size_t scene_bytes = (size_t)(kNodeF4 * sc.nnodes + 3 * sc.ntri) * sizeof(float4);
    return fp.wf_slots > 0 && fp.pass == 0 && fp.spp > 0 && fp.nloc > 0 && fp.log_cap == 0 && sc.ntri > 0 &&
           sc.nbrute == 0 && fp.resume_min > 0 && fp.walk_team <= 1 && scene_bytes > kLdsSceneMax &&
           fp.max_bounce <= 4096;
}

size_t wavefront_bytes(const DevScene& sc, const FrameParams& fp, int block) {
    const int npl = wf_planes(!wide_walk(sc, fp));
    const size_t waves = (size_t)wf_grid_bound(fp, block, device_cus()) * (size_t)(block / 64);
    return waves * 64u * (size_t)fp.wf_slots * (size_t)(4 * npl + kWfEntryBytes);
}

hipError_t launch_wavefront(const DevScene& sc, const FrameParams& fp, int block, float* d_out,
                            unsigned long long* d_counts, unsigned int* d_work, hipStream_t stream) {
    if (!wavefront_eligible(sc, fp) || !fp.wf_buf) return hipErrorInvalidValue;
    DevScene s2 = sc;
    s2.stack_lds = std::max(1, std::min(sc.stack_lds, kStackLdsWave));
    const bool ovf = s2.stack_lds < s2.depth;
    const bool wide = wide_walk(sc, fp);
    const bool count = d_counts != nullptr;
    const void* fn = count ? (ovf ? (wide ? wave_fn<true, true, true>() : wave_fn<true, true, false>())
                                  : (wide ? wave_fn<true, false, true>() : wave_fn<true, false, false>()))
                           : (ovf ? (wide ? wave_fn<false, true, true>() : wave_fn<false, true, false>())
                                  : (wide ? wave_fn<false, false, true>() : wave_fn<false, false, false>()));
    const size_t lds = (size_t)s2.stack_lds * 8u * (size_t)block;
    const int cus = device_cus();
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, block, lds);
    if (e != hipSuccess) return e;
    const int cap_cu = fp.max_waves > 0 ? std::max(1, fp.max_waves * 4 * 64 / block) : INT_MAX;
    // the buffer (wavefront_bytes) holds wf_grid_bound blocks' regions: never launch more
    const int64_t grid = std::min<int64_t>(wf_grid_bound(fp, block, cus),
                                           (int64_t)cus * std::max(1, std::min(per_cu, cap_cu)));
    e = hipMemsetAsync(d_work, 0, (size_t)kGroups * kCounterStride, stream);
    if (e != hipSuccess) return e;
    DevScene a0 = s2;
    FrameParams a1 = fp;
    LaunchConst a2 = make_const(fp);
    float* a3 = d_out;
    unsigned long long* a4 = d_counts;
    unsigned int* a5 = d_work;
    void* args[] = {&a0, &a1, &a2, &a3, &a4, &a5};
    e = hipLaunchKernel(fn, dim3((unsigned)grid), dim3(block), args, lds, stream);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

}  // namespace rt
