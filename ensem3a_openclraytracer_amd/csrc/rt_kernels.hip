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
#include "rt_device.h"

namespace rt {

namespace {

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
#ifndef RT_RENDER_WAVES
#define RT_RENDER_WAVES 5   // variant builds: another waves-per-SIMD target for render_kernel
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_RENDER_WAVES))) render_kernel(DevScene S, FrameParams F, float* __restrict__ out,
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
    pq.per = (F.handout && F.pass != 2) ? (unsigned)((F.nloc + kGroups - 1) / kGroups) : 0u;   // pass 2: cost order, interleaved
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
    unsigned long long t_prev = 0;   // COUNT: the wave clock at the previous loop head

    // pass 1 (FrameParams::pass): after the pilot samples, save the pixel's state for pass 2; the
    // pixel is written (and its cost set to 0) when all its samples are done
    auto save_pilot = [&]() __attribute__((always_inline)) {
        F.pilot_state[2 * (int64_t)p] = make_float4(acc.x, acc.y, acc.z, kc);
        F.pilot_state[2 * (int64_t)p + 1] =
            make_float4(__uint_as_float(seed0), __uint_as_float(seed1), __int_as_float(tc), __int_as_float(s));
        F.pilot_cost[p] = s >= spp ? 0u : (unsigned)cost;
    };

    while (true) {
        // instrumented build: wave cycles in the trace (cyc_trav) and in the rest of the loop (cyc_shade:
        // every iteration's time, the trace's subtracted below; unsigned wrap-around cancels)
        if (COUNT && lane == 0) {
            const unsigned long long now = clock64();
            if (t_prev) c.cyc_shade += now - t_prev;
            t_prev = now;
        }
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
                    // past the tile, or a padding pixel of a partial last row (its hand-out group, or pass 2's
                    // cost order, may still hold real pixels): the lane retires once the queue is dry
                    phase = q < nloc ? FETCH : DONE;
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
                    const rtm_f3 nd = dev_normalize(Rd);
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
        const unsigned long long t_tr = COUNT ? clock64() : 0;
        const Hit h = trace<TRAV, COUNT, SMEM, OVF, BRUTE != 0>(S, nodes, tris, to, td, stk, B, lst, c, mtrec, ts, boxrec);
        if (COUNT && lane == __ffsll((long long)__ballot(1)) - 1) {   // the first tracing lane, once per wave
            const unsigned long long dt = clock64() - t_tr;
            c.cyc_trav += dt;
            c.cyc_shade -= dt;
        }
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
// (kWideWaves: rt_internal.h)

// TS > 1: teams of TS lanes per pixel walk each ray together (team_step; BVH2 item steps only).
// WIDE: 0 = the BVH2 walk, 1 = the 4-wide walk, 2 = the 4-wide walk with origin-folded dequantisation
// (wide_node DQ; launch_fast picks it when the camera lies within DevScene::wdq_omax)
template <bool COUNT, bool LOG, bool SMEM, bool OVF, bool STEP, int WIDE, int TS = 1>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WIDE ? kWideWaves : 4))) render_resume_kernel(DevScene S, FrameParams F, float* __restrict__ out,
                                                      unsigned long long* __restrict__ counts,
                                                      unsigned int* __restrict__ work_counter,
                                                      const LaunchConst* __restrict__ lconst) {
    extern __shared__ int lds_stack[];
    const int B = blockDim.x;
    // two-pass launches are BVH2-only (the 4-wide walk's pilot measured slower, rt_api.hip setup_pilot):
    // the 4-wide instantiations are one-pass and carry none of the pass code
    const int pass = WIDE ? 0 : F.pass;
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
    pq.per = (F.handout && pass != 2) ? (unsigned)((F.nloc + kGroups - 1) / kGroups) : 0u;   // pass 2: cost order, interleaved
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
    int ndraw = 0;       // pass 1, BVH2 walk: random numbers the pixel drew (its RNG offset, pilot_draws)
    // sample slices (FrameParams::slices): the sample count this job stops at; while the job waits for the
    // slice before it (phase WAIT_SLICE), the job's slice index
    // (one-pass launches, and pass 2 of a pilot launch: the samples after the pilot's sb = F.pilot; slice k
    // of a pixel ends at sb + (k + 1) (spp - sb) / nsl)
    const unsigned nsl = (TS == 1 && F.slices > 1 && pass != 1) ? (unsigned)F.slices : 1u;
    const int sb = pass == 2 ? F.pilot : 0;
    auto slice_end = [&](unsigned k) { return sb + (int)((k + 1u) * (unsigned)(spp - sb) / nsl); };
    int lim = spp;
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
        if (!WIDE && F.pilot_draws) F.pilot_draws[p] = (uint32_t)ndraw;
    };
    // slices: the pixel's state after this job's slice, stored write-through (sc1) for the lane that runs the
    // next slice; then, once the wave's stores have completed, the samples done (the word that lane polls)
    auto save_slice = [&]() __attribute__((always_inline)) {
        if (!team_leader) return;
        gu64* st = (gu64*)(F.slice_state + 2 * (int64_t)p);
        auto pk = [](float a, float b) { return (unsigned long long)__float_as_uint(a) | ((unsigned long long)__float_as_uint(b) << 32); };
        __hip_atomic_store(st + 0, pk(acc.x, acc.y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(st + 1, pk(acc.z, kc), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(st + 2, (unsigned long long)seed0 | ((unsigned long long)seed1 << 32), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(st + 3, (unsigned long long)(unsigned)tc | ((unsigned long long)(unsigned)s << 32),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // The hand-off is built by hand, not as a release / acquire pair: at agent scope those compile on
        // gfx950 to an L2 write-back (buffer_wbl2 sc1) before every ready store and an L2 invalidate
        // (buffer_inv sc1) after every successful poll -- of the whole L2 the BVH lives in -- measured
        // C3 106.9 -> 152.8 ms, C4 272.8 -> 297.1, C5 4,485 -> 5,705 ms (r06).  Here the
        // state words and the count are sc1 (agent-scope) atomics, which write through to memory and
        // read past this CU's L1; s_waitcnt vmcnt(0) orders the state stores' completion before the
        // count store, and the reader's wavefront fence keeps its state loads after the poll.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store((gu32*)(F.slice_ready + p), (unsigned)s, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    };
    auto finish_sample = [&]() __attribute__((always_inline)) {  // output += baseColor; next sample from the cached camera hit
        if (LOG && logme) log_event(F, 3.0f, s + 1, rtm_v3(0, 0, 0), rtm_v3(0, 0, 0), 0.0f, 0, so);
        acc = rtm_add(acc, so);
        if (COUNT) c.samples++;
        ++s;
        if (s >= spp) write_pixel();
        const bool stop = (pass == 1 && (s >= spp || s >= F.pilot)) || (nsl > 1 && s >= lim);
        if (stop) {
            if (nsl > 1) save_slice();
            else save_pilot();
        }
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
            const unsigned int qj = take_pixel(pq, need, team_lane0, work_counter, nloc, lane, nsl);
            if (phase == FETCH) {
                const unsigned sl = qj / nloc;   // the job's slice (>= nsl: none left)
                const unsigned q = sl < nsl ? qj - sl * nloc : nloc;
                bool ok = q < nloc;
                if (ok) {
                    p = pass == 2 ? (int)F.pilot_order[q] : (int)q;
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
                    ndraw = 0;
                    pre = false;
                    sun_c = SUN_UNKNOWN;
                    phase = PRIMARY;
                    logme = LOG && i == F.log_pixel;
                    if (sl > 0) {
                        lim = (int)sl;   // continues the pixel once slice sl - 1 is done (below)
                        phase = WAIT_SLICE;
                    } else if (pass == 2) {   // continue from the pilot state: camera hit cached, sample s next
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
                        lim = slice_end(0);
                        phase = s >= spp ? FETCH : PREP;   // finished in pass 1: already written
                        if (nsl > 1 && s >= spp) save_slice();   // ... and its later slices have nothing to do
                    } else {
                        lim = slice_end(0);
                        start(C.position, cd);
                    }
                } else {
                    // past the tile, or a padding pixel of a partial last row: with sample slices (jobs handed
                    // out slice-major) or pixels in cost order (pass 2) later jobs of real pixels may still be
                    // queued, so the lane only retires once the queue itself has run dry (q == nloc)
                    phase = q < nloc ? FETCH : DONE;
                }
            }
        }
        if (nsl > 1 && phase == WAIT_SLICE) {
            // slices: the previous slice's samples done, published by the lane that ran it (save_slice); its
            // state is read with sc1 loads (past this CU's L1) once the count is there
            const unsigned need_s = (unsigned)slice_end((unsigned)lim - 1u);
            const unsigned done_s = __hip_atomic_load((gu32*)(F.slice_ready + p), __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
            if (done_s >= need_s) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // the state loads stay after the poll
                gu64* st = (gu64*)(F.slice_state + 2 * (int64_t)p);
                const unsigned long long a = __hip_atomic_load(st + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long b = __hip_atomic_load(st + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long d = __hip_atomic_load(st + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long e = __hip_atomic_load(st + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                acc = rtm_v3(__uint_as_float((unsigned)a), __uint_as_float((unsigned)(a >> 32)), __uint_as_float((unsigned)b));
                kc = __uint_as_float((unsigned)(b >> 32));
                seed0 = (uint32_t)d;
                seed1 = (uint32_t)(d >> 32);
                tc = (int)(unsigned)e;
                s = (int)(unsigned)(e >> 32);
                tri = tc; j = 0;
                so = rtm_v3(1, 1, 1);
                drew = false;
                lim = slice_end((unsigned)lim);
                phase = s >= spp ? FETCH : PREP;   // finished early (a sample that draws nothing): written
            }
        }
        if (__all(phase == DONE)) break;
        if (nsl > 1 && __all(phase == DONE || phase == WAIT_SLICE)) __builtin_amdgcn_s_sleep(8);
        if (COUNT && lane == 0) c.wave_outer++;

        // -- advance every lane without a ray in flight until it needs one --
        if (!tracing && phase != DONE && phase != FETCH) {
            Hit h{T.bk, WIDE && T.bt >= 0 ? (int)((unsigned)T.bt / 48u) : T.bt};
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
                            if (!WIDE) ndraw += 2;
                            Bd = hemi_sample(cm.type == 1, n, S.tri_frame[3 * tri], S.tri_frame[3 * tri + 1], f2,
                                             &seed1, &seed0, &invPdf);
                            if (cm.type == 1) brdf = rtm_scale(cm.color, 1.0f / 3.14f);
                            else brdf = brdf_ggx(cm.color, cm.rough, rtm_scale(Rd, -1.0f), Bd, n);
                        } else {
                            Bd = Rd;
                            brdf = cm.color;
                            invPdf = 1.0f / rtm_fabs(rtm_dot(Bd, nn));
                        }
                        const rtm_f3 nd = dev_normalize(Rd);
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
        // BVH2 item steps of single lanes are software-pipelined (fast_step_pipe: the next item's loads go
        // out before this item's leaf test; r05: C3 114.4 -> 110.5 ms, C4 282.7 -> 284.6 ms); the loads
        // for the first step of this round are issued here (a lane continuing its ray re-fetches its item)
        constexpr bool PIPE = STEP && !WIDE && TS == 1;
        ItemData D;
        if (RT_TOP_LEVELS && PIPE && !SMEM && S.root_ref >= 0) {
            // rays started this round (still at the root: a started ray steps at least once per round)
            const bool fresh = tracing && T.item == S.root_ref;
            if (__ballot(fresh) && !top_levels<COUNT, OVF>(S, T, fresh, nb, lst, c)) tracing = false;
        }
        if (PIPE && tracing) D = item_fetch<SMEM>(T.item, nb, tb, kstride);
        while (true) {
            if (tracing && (PIPE ? fast_step_pipe<COUNT, SMEM, OVF>(T, D, nb, tb, lst, kstride, c)
                            : TS > 1 ? team_step<COUNT, SMEM, OVF>(TS, T, boff, nb, tb, lst, kstride, c)
                            : WIDE ? (STEP ? wide_step<COUNT, OVF, WIDE == 2>(T, wnb, wlb, lst, c)
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

// spec: with speculation available (FrameParams::spec < 0, auto) the same thresholds pick trails instead of
// teams: 8 trails per pixel at u <= 1/4 per lane, 4 at u <= 1/2, 2 at u <= 1 (r04, 1/8 and 1/4 row tiles:
// C4 1/8 u ~ 0.23 per lane: 8 trails 82.1 ms, 4 trails 91.0 (85 on another box), teams 109, 2 trails 137;
// C3 1/8 u ~ 0.47: 2 / 4 / 8 trails 36.1 / 35.0 / 41.7 ms, teams 50.7; C3 1/4 u ~ 0.93: 2 trails 53.8,
// 4 trails 58.1-61.6, teams 66.8; whole frames (u ~ 1.8 C4, ~3.7 C3): 2 trails 302 / 151 vs one lane 300 /
// 125 ms), encoded kSpecPick + trails
__global__ void pilot_team_pick_kernel(const unsigned* __restrict__ left, int64_t lanes, int spec, int* __restrict__ ts) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const int64_t u4 = 4 * (int64_t)*left;   // 4 u lanes
        const int k = u4 <= 2 * lanes ? 4 : u4 <= 4 * lanes ? 2 : 1;
        *ts = (spec && k > 1) ? kSpecPick + (u4 <= lanes ? 8 : k) : k;
    }
}

template <int TRAV, bool COUNT, bool LOG, bool SMEM = false, bool RESUME = false, bool OVF = false,
          bool BRUTE = false, bool STEP = true, int WIDE = 0>
hipError_t launch_t(const DevScene& sc, const FrameParams& fp, int block, float* d_out, unsigned long long* d_counts,
                    unsigned int* d_work, hipStream_t stream) {
    // FAST: int2 entries; the brute-force path of small scenes needs no stack
    const int depth = (TRAV == TRAV_REF) ? sc.ref_stack : (sc.nbrute > 0 ? 1 : 2 * (sc.stack_lds > 0 ? sc.stack_lds : 1));
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
    // team walk (render_resume_kernel TEAM): BVH2 item steps only; walk_team, 0 = auto (auto_walk_team;
    // pass 2 of a pilot launch: the size pilot_team_pick_kernel chose, launch_render)
    constexpr bool kTeamable = RESUME && STEP && !WIDE && !LOG;
    int wteam = 1;
    if (kTeamable) {
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
    if (kTeamable && wteam > 1) {
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
    if (kTeamable && wteam == 2)
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
        case 8: r = mt_recip(x[i]); break;   // the Moller-Trumbore reciprocal of the FAST walks
        case 9: r = dev_sqrt(x[i]); break;   // the shading's sqrtf
        case 10: r = dev_inv_sqrt(x[i]); break;   // dev_normalize's scale, 1.0f / sqrtf
        case 11: r = dev_recip(x[i]); break;   // the kernels' 1.0f / x (ray inverses, GGX)
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

hipError_t launch_ibl_sum(const uchar4* rgba, int w, int h, uint32_t* sum, hipStream_t stream) {
    const int64_t n = (int64_t)(w + 1) * (h + 1);
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 65536);
    hipLaunchKernelGGL(ibl_sum_kernel, dim3(grid), dim3(256), 0, stream, rgba, w, h, sum);
    return hipGetLastError();
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
    const int depth = traversal == TRAV_REF ? s2.ref_stack : 2 * s2.stack_lds;
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
        // the wide walk takes item steps unless rounds are asked for (C5: 1,181 vs 1,035 Msamples/s);
        // the item steps dequantise origin-folded (WIDE 2) when every ray origin of the frame is within
        // the bound the builder's gap covers: hit points always are, the camera is checked here
        const bool step = fp.step != 2;
        const float cmax = std::max(std::fabs(fp.cam[0]), std::max(std::fabs(fp.cam[1]), std::fabs(fp.cam[2])));
        const bool dq = fp.wdq != 0 && sc.wdq_omax > 0.0f && cmax <= sc.wdq_omax;
        if (ovf)
            return !step ? launch_t<TRAV_FAST, COUNT, false, false, true, true, false, false, 1>(
                               sc, fp, block, d_out, d_counts, d_work, stream)
                   : dq  ? launch_t<TRAV_FAST, COUNT, false, false, true, true, false, true, 2>(
                               sc, fp, block, d_out, d_counts, d_work, stream)
                         : launch_t<TRAV_FAST, COUNT, false, false, true, true, false, true, 1>(
                               sc, fp, block, d_out, d_counts, d_work, stream);
        return !step ? launch_t<TRAV_FAST, COUNT, false, false, true, false, false, false, 1>(
                           sc, fp, block, d_out, d_counts, d_work, stream)
               : dq  ? launch_t<TRAV_FAST, COUNT, false, false, true, false, false, true, 2>(
                           sc, fp, block, d_out, d_counts, d_work, stream)
                     : launch_t<TRAV_FAST, COUNT, false, false, true, false, false, true, 1>(
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
                         unsigned long long* d_counts, unsigned int* d_work, hipStream_t stream, RenderPending* pend) {
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
    // small tiles of the BVH2 walk: each pixel's remaining samples as speculative trails (rt_spec.hip):
    // a set number of trails, or (spec < 0) chosen on the device with the team size
    const bool spec_ok = traversal == TRAV_FAST && fp.spec != 0 && fp.spec_log && fp.pilot_draws && spec_walk(sc, fp);
    if (spec_ok && fp.spec > 0) return launch_spec(sc, b, block, d_out, d_work, stream);
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
                           (int64_t)std::max(cus, 1) * kWalkLanesPerCu, spec_ok ? 1 : 0, ts);
        // the pick is read back (pass 1 has to finish before pass 2 anyway) and exactly the kernel it names
        // is launched: 1, 2 or 4 lanes per pixel, or kSpecPick + T trails
        RenderPending local;
        RenderPending& P = pend ? *pend : local;
        int pick_stack = 1;
        if (!P.host_pick) {
            if (pend) return hipErrorInvalidValue;   // a deferred pass 2 needs the caller's (pinned) int
            P.host_pick = &pick_stack;               // pageable: this call waits itself
        }
        e = hipMemcpyAsync(P.host_pick, ts, sizeof(int), hipMemcpyDeviceToHost, stream);
        if (e != hipSuccess) return e;
        P.pick = true;
        P.b = b;
        P.spec_ok = spec_ok;
        if (pend) return hipSuccess;
        return launch_render_finish(sc, traversal, block, d_out, d_work, stream, P);
    }
    return launch_render_pass(sc, b, traversal, block, d_out, nullptr, d_work, stream);
}

hipError_t launch_render_finish(const DevScene& sc, int traversal, int block, float* d_out, unsigned int* d_work,
                                hipStream_t stream, RenderPending& P) {
    if (!P.pick) return hipSuccess;
    P.pick = false;
    hipError_t e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return e;
    const int pick = *P.host_pick;
    FrameParams b = P.b;
    if (P.spec_ok && pick > kSpecPick) {
        b.spec = pick - kSpecPick;
        return launch_spec(sc, b, block, d_out, d_work, stream);
    }
    b.walk_team = pick;
    return launch_render_pass(sc, b, traversal, block, d_out, nullptr, d_work, stream);
}

// the launches whose FAST walk is the BVH2 item-step resumable kernel (launch_fast's choice), the walk
// rt_spec.hip continues
bool spec_walk(const DevScene& sc, const FrameParams& fp) {
    const size_t scene_bytes = (size_t)(kNodeF4 * sc.nnodes + 3 * sc.ntri) * sizeof(float4);
    const bool smem = sc.ntri > 0 && sc.nbrute == 0 && scene_bytes <= kLdsSceneMax;
    const bool resume = sc.ntri > 0 && sc.nbrute == 0 && fp.resume_min > 0;
    const bool step = fp.step == 1 || (fp.step == 0 && (size_t)sc.nnodes * kNodeF4 * 16 <= kStepMaxBytes);
    return resume && !smem && step && !(fp.wide && sc.wnodes);
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
