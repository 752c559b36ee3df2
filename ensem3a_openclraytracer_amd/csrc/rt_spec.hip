// Sample-parallel speculation for small tiles (option "spec"): pass 2 of a pilot launch of the BVH2
// tree walk, when a tile has about one pixel per resident lane (the row tiles of an N-GPU frame), with
// TR = 2, 4 or 8 trails per pixel (chosen on the device, pilot_team_pick_kernel).
//
// A pixel's samples are one chain (Raytracing.cl:191-209): sample k starts with the RNG words after
// D_k draws from the pixel seed (Raytracing.cl:171-172, MathLib.cl:294-310) and its colour and draw
// count are a function of D_k alone -- the camera hit is cached (Raytracing.cl:184-187), and the glass
// prefix and first shadow ray the per-pixel caches keep are the same in every sample.  Such a tile
// lasts as long as its longest chain.  Here TR lanes carry one pixel as TR trails:
//   trail 0 continues the chain from the pass-1 state (offset D0 = pilot_draws, sample s0);
//   trail t > 0 starts at a guessed offset G_t = D0 + t (spp - s0) / TR * mu, mu = D0 / s0 the pixel's
//   draws per pilot sample, with the RNG words stepped there, and logs every sample it completes as
//   (offset, colour) in its own log (spec_log: one per resident lane, reused from record 0 for the
//   team's next pixel).
// At every sample start a trail looks its offset up in the logs of the trails ahead of it (a cursor per
// log: offsets only grow).  Trails meet wherever one lands on an offset another computed: from there
// on their samples coincide.  A trail t > 0 that meets stops; trail 0 that meets becomes the stitcher:
// it adds the logged colours in chain order to its sum -- exactly the float additions of the serial
// chain -- following the trail it met (and the one that trail met, and so on), and computes on its own
// again from the first offset no trail holds.  The pixel is written when the chain has its spp samples;
// the other trails of the team then drop what they were doing.  Trails t > 0 stop after spec_cap
// records or at a sample that draws nothing (fixed_point: every later sample repeats it).
// So the frame is the serial one bit for bit whatever the guesses; only the work and the chain's
// latency depend on them (tools/chain_speculation.py prices both on the CPU oracle).
#include <mutex>
#include <vector>

#include "rt_device.h"

namespace rt {

namespace {

enum TrailMode { TM_IDLE = 0, TM_COMPUTE = 1, TM_STITCH = 2, TM_STOPPED = 3, TM_DONE = 4 };
constexpr int PARK = 6;   // phase of a trail that traces nothing until its team's pixel is done (beside rt_device.h Phase)
constexpr int SPEC_SUN_UNKNOWN = -2;
constexpr unsigned kFixedBit = 0x80000000u;   // log record offset word: the sample drew nothing

// the RNG words after n more draws: rtm_rand as the samplers call it, (seed1, seed0), without the float
__device__ __forceinline__ void rng_skip(uint32_t& seed0, uint32_t& seed1, int n) {
    for (int k = 0; k < n; ++k) {
        seed1 = 36969u * (seed0 & 65535u) + (seed0 >> 16);
        seed0 = 18000u * (seed1 & 65535u) + (seed1 >> 16);
    }
}

template <bool OVF, int TR>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
spec_kernel(DevScene S, FrameParams F, float* __restrict__ out, unsigned int* __restrict__ work_counter,
            const LaunchConst* __restrict__ lconst) {
    static_assert(TR == 2 || TR == 4 || TR == 8, "trails per pixel");
    extern __shared__ int lds_stack[];
    Cnt c{};
    const LaunchConst& C = *lconst;
    const LaneStack lst = lane_stack(S, lds_stack);
    const char* const nb = reinterpret_cast<const char*>(S.nodes);
    const char* const tb = reinterpret_cast<const char*>(S.tri_fast);
    const int W = F.width;
    const float e3 = F.env[3], e4 = F.env[4];
    const int spp = F.spp, maxB = F.max_bounce;
    const unsigned nloc = (unsigned)F.nloc;
    const int cap = F.spec_cap;
    const int lane = threadIdx.x & 63;
    const int tau = lane & (TR - 1);           // this lane's trail
    const int team0 = lane - tau;
    const bool leader = tau == 0;
    const unsigned long long leaders = TR == 2 ? 0x5555555555555555ull : TR == 4 ? 0x1111111111111111ull : 0x0101010101010101ull;
    // record k of trail u (>= 1) of the team's pixel: the log of the trail's lane (launch_spec: grid x block
    // <= the logs allocated)
    const unsigned glane0 = blockIdx.x * blockDim.x + (threadIdx.x - (unsigned)tau);
    auto log_at = [&](int u, int k) -> float4* {
        return F.spec_log + (size_t)(glane0 + (unsigned)u) * (size_t)cap + (size_t)k;
    };

    int phase = FETCH;
    bool tracing = false;
    PixelQueue pq;
    pq.per = (F.handout && F.pass != 2) ? (unsigned)((F.nloc + kGroups - 1) / kGroups) : 0u;   // pass 2: cost order, interleaved
    FastRay T;
    T.item = 0; T.soff = 0; T.bk = 1000.0f; T.bt = -1; T.brank = -1; T.any = false;
    T.o = rtm_v3(0, 0, 0); T.d = rtm_v3(0, 0, 1); T.ix = T.iy = T.iz = 0.0f;
    int p = 0, i = 0;
    uint32_t seed0 = 0, seed1 = 0;
    rtm_f3 cd = rtm_v3(0, 0, 0);
    float kc = 1000.0f;
    int tc = -1;
    rtm_f3 so = rtm_v3(1, 1, 1);
    int tri = -1, j = 0;
    rtm_f3 Bd = rtm_v3(0, 0, 0);
    rtm_f3 acc = rtm_v3(0, 0, 0);   // trail 0: the chain's sum
    int s = 0;                      // trail 0: chain samples done; trail t > 0: records logged
    bool drew = false;
    bool pre = false;
    int pre_j = 0, pre_tri = -1;
    rtm_f3 pre_so = rtm_v3(1, 1, 1), pre_o = rtm_v3(0, 0, 0), pre_d = rtm_v3(0, 0, 1);
    float pre_k = 1000.0f;
    int sun_c = SPEC_SUN_UNKNOWN;
    bool fdb = false;
    // trail state
    int mode = TM_IDLE;
    int D = 0;                      // RNG offset at the start of the current sample
    int dcur = 0;                   // draws of the current sample so far
    int D0 = 0;                     // the pass-1 offset and words: the words at any offset >= D0 are stepped from them
    uint32_t w00 = 0, w10 = 0;
    int cur[TR - 1];                // cursors into the logs of trails tau+1.. (trail u at [u - 1])
#pragma unroll
    for (int u = 0; u < TR - 1; ++u) cur[u] = 0;
    int src = 0, sj = 0;            // trail 0 stitching: the trail it follows and the next record

    auto restart_sample = [&]() __attribute__((always_inline)) {   // sample start from the cached camera hit / prefix
        tri = tc; j = 0;
        so = rtm_v3(1, 1, 1);
        drew = false;
        dcur = 0;
        if (pre) {
            tri = pre_tri; j = pre_j;
            so = pre_so;
            T.o = pre_o; T.d = pre_d; T.bk = pre_k;
        }
        phase = PREP;
    };
    // is offset x in trail u's log (u > tau)?  advances the cursor; returns the record index or -1
    auto find_in = [&](int u, int& cu, int x, int produced) -> int {
        while (cu < produced) {
            const int o = (int)(__float_as_uint(log_at(u, cu)->x) & ~kFixedBit);
            if (o > x) return -1;
            if (o == x) return cu;
            ++cu;
        }
        return -1;
    };

    while (true) {
        // -- a finished pixel: every trail of its team lets go and the team takes the next pixel --
        const unsigned long long fin = __ballot(leader && mode == TM_DONE);
        if ((fin >> team0) & 1ull) {
            phase = FETCH;
            mode = TM_IDLE;
            tracing = false;
        }
        const unsigned long long need = __ballot(phase == FETCH) & leaders;
        if (need) {
            const unsigned q = take_pixel(pq, need, team0, work_counter, nloc, lane);
            if (phase == FETCH) {
                bool ok = q < nloc;
                if (ok) {
                    p = (int)F.pilot_order[q];
                    const int krow = p / W;
                    const int64_t i64 = ((int64_t)F.row0 + (int64_t)krow * F.row_step) * W + (p - krow * W);
                    ok = i64 < F.npix;
                    i = (int)i64;
                }
                if (ok) {
                    const float4 a = F.pilot_state[2 * (int64_t)p], b = F.pilot_state[2 * (int64_t)p + 1];
                    kc = a.w;
                    tc = __float_as_int(b.z);
                    const int s0 = __float_as_int(b.w);
                    D0 = (int)F.pilot_draws[p];
                    w00 = __float_as_uint(b.x);
                    w10 = __float_as_uint(b.y);
                    seed0 = w00;
                    seed1 = w10;
                    cd = camera_dir(C, W, i);
                    pre = false;
                    sun_c = SPEC_SUN_UNKNOWN;
#pragma unroll
                    for (int u = 0; u < TR - 1; ++u) cur[u] = 0;
                    if (s0 >= spp) {
                        phase = FETCH;   // finished in pass 1: already written
                    } else if (leader) {
                        acc = rtm_v3(a.x, a.y, a.z);
                        s = s0;
                        D = D0;
                        mode = TM_COMPUTE;
                        restart_sample();
                    } else {
                        // the guess: tau (spp - s0) / TR more samples at the pilot's draws per sample, even
                        const float mu = s0 > 0 ? (float)D0 / (float)s0 : 2.0f;
                        const int ahead = 2 * (int)(0.5f * mu * (float)(tau * (spp - s0)) / (float)TR + 0.5f);
                        D = D0 + ahead;
                        rng_skip(seed0, seed1, ahead);
                        s = 0;
                        mode = TM_COMPUTE;
                        restart_sample();
                    }
                } else {
                    phase = (q < nloc) ? FETCH : DONE;   // padding pixel past the frame / tile exhausted
                    mode = TM_IDLE;
                }
            }
        }
        if (__all(phase == DONE)) break;

        // -- the team's trails, after the hand-out (records are append-only: a count
        //    taken before this iteration's logging is a lower bound) --
        // (s | mode << 16 of every trail of the team, and its offset, by one shuffle each)
        int sm_[TR], dn_[TR];
#pragma unroll
        for (int u = 1; u < TR; ++u) {
            sm_[u] = __shfl(s | (mode << 16), team0 + u, 64);
            dn_[u] = __shfl(D, team0 + u, 64);
        }
        // the records those counts cover were stored by lanes of this wave in earlier iterations (release
        // fence after each log store): the acquire keeps the log reads below after the counts were taken
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // trail u's value, for a runtime u (a select chain: the arrays stay in registers)
        auto pick = [&](const int* a, int u) __attribute__((always_inline)) {
            int v = 0;
#pragma unroll
            for (int w = 1; w < TR; ++w) v = u == w ? a[w] : v;
            return v;
        };
        auto produced = [&](int u) { return pick(sm_, u) & 0xffff; };
        auto mode_of = [&](int u) { return pick(sm_, u) >> 16; };
        auto dnow_of = [&](int u) { return pick(dn_, u); };
        // the first trail ahead of `from` whose log holds offset x: (trail, record) or (0, -1); one copy of
        // the log scan, the cursors read and written by select chains (they stay in registers)
        auto search = [&](int from, int x, int* rec) -> int {
            for (int u = from + 1; u < TR; ++u) {
                int cu = 0;
#pragma unroll
                for (int w = 1; w < TR; ++w) cu = u == w ? cur[w - 1] : cu;
                const int r = find_in(u, cu, x, produced(u));
#pragma unroll
                for (int w = 1; w < TR; ++w) cur[w - 1] = u == w ? cu : cur[w - 1];
                if (r >= 0) {
                    *rec = r;
                    return u;
                }
            }
            return 0;
        };


        // -- trail 0 stitching: add the logged colours of the trail it follows, in chain order (up to 8
        //    records loaded at once, a few batches per iteration) --
        if (leader && mode == TM_STITCH) {
            for (int batch = 0; batch < 4 && mode == TM_STITCH; ++batch) {
                const int avail = produced(src) - sj;
                if (avail > 0) {
                    const int nr = min(avail, 8);
                    float4 r[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        if (k < nr) r[k] = *log_at(src, sj + k);
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        if (k < nr && mode == TM_STITCH) {
                            const rtm_f3 col = rtm_v3(r[k].y, r[k].z, r[k].w);
                            ++sj;
                            acc = rtm_add(acc, col);
                            ++s;
                            if ((__float_as_uint(r[k].x) & kFixedBit) && F.fixed_point)
                                for (; s < spp; ++s) acc = rtm_add(acc, col);   // every later sample repeats it
                            if (s >= spp) {
                                store_pixel(out, p, acc, spp);
                                mode = TM_DONE;
                            }
                        }
                    }
                } else if (mode_of(src) == TM_STOPPED) {
                    // the followed trail stopped: the chain goes on at its next offset, in a trail further
                    // ahead or (none holds it) computed here
                    const int x = dnow_of(src);
                    int r = -1;
                    const int u = search(src, x, &r);
                    if (u > 0) {
                        src = u;
                        sj = r;
                    } else {
                        D = x;
                        seed0 = w00;
                        seed1 = w10;
                        rng_skip(seed0, seed1, x - D0);
                        mode = TM_COMPUTE;
                        restart_sample();
                    }
                } else {
                    break;   // the followed trail has not logged the next sample yet
                }
            }
        }

        // -- advance every computing trail without a ray in flight until it needs one --
        if (!tracing && mode == TM_COMPUTE && phase != FETCH && phase != DONE && phase != PARK) {
            // a sample ended: trail 0 adds it to the chain, a trail ahead logs it; then the next sample
            // starts, unless a trail ahead already holds its offset
            auto end_sample = [&]() __attribute__((always_inline)) {
                const bool fixed = F.fixed_point && !drew;
                if (leader) {
                    acc = rtm_add(acc, so);
                    ++s;
                    if (fixed) for (; s < spp; ++s) acc = rtm_add(acc, so);
                    if (s >= spp) {
                        store_pixel(out, p, acc, spp);
                        mode = TM_DONE;
                        phase = PARK;
                        return;
                    }
                } else {
                    *log_at(tau, s) = make_float4(__uint_as_float((uint32_t)D | (fixed ? kFixedBit : 0u)), so.x,
                                                     so.y, so.z);
                    // published to the wave's other trails through the count s, read by a shuffle in a later
                    // iteration (acquire fence there): the record is ordered before that count
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    ++s;
                    if (fixed || s >= cap) {
                        D += dcur;
                        mode = TM_STOPPED;
                        phase = PARK;   // no more work until the team's pixel is done
                        return;
                    }
                }
                D += dcur;
                int r = -1;
                const int u = search(tau, D, &r);
                if (u > 0) {
                    if (leader) {
                        mode = TM_STITCH;
                        src = u;
                        sj = r;
                    } else {
                        mode = TM_STOPPED;
                    }
                    phase = PARK;
                    return;
                }
                restart_sample();
            };
            // the traced ray's result (render_resume_kernel: BOUNCE / SUN)
            Hit h{T.bk, T.bt};
            if (phase == BOUNCE) {
                if (h.tri >= 0) {
                    tri = h.tri;
                    const Mat bm = load_mat(S.mat, __float_as_int(S.tri_shade[h.tri].w));
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
                } else {
                    phase = SUN;
                    if (F.sun_skip) {
                    } else if (fdb && sun_c != SPEC_SUN_UNKNOWN) {
                        h.tri = sun_c;
                    } else {
                        tracing = !fast_init<false>(S, T, T.o, C.sun, c);
                        T.any = F.sun_any != 0;
                    }
                }
            }
            if (phase == SUN && !tracing && mode == TM_COMPUTE) {   // Raytracing.cl:125-137
                rtm_f3 sunLight = rtm_v3(0, 0, 0);
                if (fdb) sun_c = h.tri;
                const Mat cm = load_mat(S.mat, __float_as_int(S.tri_shade[tri].w));
                if (h.tri < 0 && cm.type != 3) sunLight = rtm_v3(e3, e3, e3);
                if (h.tri >= 0) {
                    const Mat sm = load_mat(S.mat, __float_as_int(S.tri_shade[h.tri].w));
                    if (sm.type == 3) sunLight = rtm_scale(sm.color, e3);
                }
                const rtm_f3 envLight = rtm_scale(sample_ibl_if<false>(S, C, Bd, e4, c), e4);
                so = rtm_mul(so, rtm_add(sunLight, envLight));
                end_sample();
            }
            // naiveGI loop heads (Raytracing.cl:46-79) until a ray is needed or the trail pauses
            while (phase == PREP && mode == TM_COMPUTE) {
                const bool cam = j == 0;
                const rtm_f3 Ro = cam ? C.position : T.o, Rd = cam ? cd : T.d;
                const float k = cam ? kc : T.bk;
                if (j > maxB) {
                    end_sample();
                } else if (tri < 0) {
                    so = rtm_scale(rtm_mul(so, sample_ibl_if<false>(S, C, Rd, e4, c)), e4);
                    end_sample();
                } else {
                    const float4 sh = S.tri_shade[tri];
                    const rtm_f3 n = xyz(sh);
                    const Mat cm = load_mat(S.mat, __float_as_int(sh.w));
                    if (cm.type == 0) {
                        so = rtm_scale(so, cm.rough);
                        end_sample();
                    } else {
                        const float4 f2 = S.tri_frame[3 * tri + 2];
                        const rtm_f3 nn = xyz(f2);
                        float invPdf = 0.0f;
                        rtm_f3 brdf = rtm_v3(0, 0, 0);
                        if (F.fixed_point && cm.type != 3 && !drew && j > 0 && !pre) {
                            pre = true;
                            pre_j = j; pre_tri = tri;
                            pre_so = so;
                            pre_o = T.o; pre_d = T.d; pre_k = T.bk;
                        }
                        fdb = F.sun_cache && cm.type != 3 && !drew && !F.sun_skip;
                        drew = drew || cm.type != 3;
                        if (cm.type != 3) {
                            dcur += 2;
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
                        const float att = invPdf * rtm_fabs(rtm_dot(Bd, nn));
                        so = rtm_scale(rtm_mul(so, brdf), att);
                        phase = BOUNCE;
                        tracing = !fast_init<false>(S, T, Bo, Bd, c);
                        T.any = false;
                    }
                }
            }
        }

        // -- traversal steps until resume_min / 64 of the lanes still rendering have no ray in flight --
        // parked trails and finished lanes take no part in the threshold (render_resume_kernel)
        const unsigned long long alive = __ballot(phase != DONE && phase != PARK);
        const int rthr = F.resume_min * __popcll(alive);
        while (true) {
            if (tracing && fast_step<false, false, OVF>(S, T, nb, tb, lst, 16u, c)) tracing = false;
            const unsigned long long tr = __ballot(tracing);
            if (tr == 0 || 64 * __popcll(alive & ~tr) >= rthr) break;
        }
    }
}

template <bool OVF, int TR>
const void* spec_fn() {
    return (const void*)spec_kernel<OVF, TR>;
}

}  // namespace

size_t spec_log_bytes(const FrameParams& fp, int cus) {
    if (fp.spec == 0) return 0;
    return (size_t)std::max(cus, 1) * kWalkLanesPerCu * (size_t)std::max(fp.spec_cap, 1) * sizeof(float4);
}

hipError_t launch_spec(const DevScene& sc, const FrameParams& fp, int block, float* d_out, unsigned int* d_work,
                       hipStream_t stream) {
    if ((fp.spec != 2 && fp.spec != 4 && fp.spec != 8) || fp.pass != 2 || !fp.spec_log || !fp.pilot_draws || fp.spec_cap <= 0)
        return hipErrorInvalidValue;
    const bool ovf = sc.stack_lds < sc.depth;
    const void* fn = fp.spec == 2   ? (ovf ? spec_fn<true, 2>() : spec_fn<false, 2>())
                     : fp.spec == 4 ? (ovf ? spec_fn<true, 4>() : spec_fn<false, 4>())
                                    : (ovf ? spec_fn<true, 8>() : spec_fn<false, 8>());
    const size_t lds = (size_t)2 * std::max(sc.stack_lds, 1) * (size_t)block * sizeof(int);
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    {
        // blocks per CU of each (instantiation, block, LDS), queried once per device (a context may hold
        // devices of different kinds): the host query costs more than the launch
        struct Occ { int dev; const void* fn; int block; size_t lds; int per_cu; };
        static std::mutex mu;
        static std::vector<Occ> seen;
        std::lock_guard<std::mutex> g(mu);
        for (const Occ& o : seen)
            if (o.dev == dev && o.fn == fn && o.block == block && o.lds == lds) per_cu = o.per_cu;
        if (per_cu == 0) {
            e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, block, lds);
            if (e != hipSuccess) return e;
            seen.push_back({dev, fn, block, lds, per_cu});
        }
    }
    const int cap_cu = fp.max_waves > 0 ? std::max(1, fp.max_waves * 4 * 64 / block) : INT_MAX;
    // at most kWalkLanesPerCu lanes per CU: one trail log each (spec_log_bytes)
    const int cap_logs = std::max(1, kWalkLanesPerCu / block);
    const int64_t resident = (int64_t)std::max(1, cus) * std::max(1, std::min({per_cu, cap_cu, cap_logs}));
    const int64_t grid = std::min<int64_t>((fp.nloc * fp.spec + block - 1) / block, resident);
    // the work block's counters and launch constants were set up by pass 1's launch (launch_t): pass 2
    // re-zeroes the counters and recomputes the constants the same way
    e = hipMemsetAsync(d_work, 0, (size_t)kGroups * kCounterStride, stream);
    if (e != hipSuccess) return e;
    LaunchConst* lc = reinterpret_cast<LaunchConst*>(reinterpret_cast<char*>(d_work) + kConstOffset);
    hipLaunchKernelGGL(make_const_kernel, dim3(1), dim3(64), 0, stream, fp, lc);
    DevScene a0 = sc;
    FrameParams a1 = fp;
    float* a2 = d_out;
    unsigned int* a3 = d_work;
    const LaunchConst* a4 = lc;
    void* args[] = {&a0, &a1, &a2, &a3, &a4};
    e = hipLaunchKernel(fn, dim3((unsigned)grid), dim3(block), args, lds, stream);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

}  // namespace rt
