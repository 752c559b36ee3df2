// C-ABI of the MI355X path tracer (include/rt_api.h, include/rt_debug.h).
//
// Replaces the pyopencl side of the reference's KernelLauncher
// (KernelLauncher.py:8-103): device selection, buffer/image uploads, the
// kernel enqueue and the blocking read-back.  Scene arrays arrive in the
// reference's flat AoS layouts (FileManager.Scene / BVH.exportArray) and are
// repacked here into the device layout of rt_internal.h:
//   * triangles pre-gathered (a.p, e1, e2) + hit record (a.n, material),
//   * BVH2 nodes holding both child boxes in BFS order (FAST traversal),
//   * the untouched 9-float export (REF traversal).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <algorithm>
#include <array>
#include <chrono>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rt_api.h"
#include "../../include/rt_debug.h"
#include "rt_internal.h"
#include "scene_pack.h"

// FAST tree walk: resumable traversal threshold (rt_set_option "resume_min"; -1 = auto), out of 64
// lanes still rendering: 36 on the BVH2 walk (C3 / C4 ms at 32 / 36 / 40: 138.8 / 136.8 / 136.5,
// 446.8 / 452.6 / 455.0), 48 on the 4-wide walk (C5 at 40 / 48 / 52: 5,805 / 5,705 / 5,772)
constexpr int kResumeMinBvh2 = 36, kResumeMinWide = 48;

using rt::HostScene;

namespace {

thread_local std::string g_thread_error;

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

struct Device {
    int id = 0;
    hipStream_t stream = nullptr;
    int cus = 0;                  // compute units (sizes the FAST stack overflow buffer)
    DevBuf stack_ovf;             // FAST traversal stack entries beyond the LDS part
    DevBuf nodes, wnodes, wleaves, tri_fast, brute, brute_box, bvh9, tri_geo, tri_shade, tri_frame, mat, ibl, ibl_sum, out, out8, counts, work, scratch_a, scratch_b;
    DevBuf pilot;                 // two-pass launches: per-pixel state, cost and order (FrameParams::pilot_*)
    DevBuf spec;                  // speculation: the trails' sample logs (FrameParams::spec_log)
    DevBuf slice;                 // sample slices: per-pixel state + samples done (FrameParams::slice_*)
    char* host_stage = nullptr;   // pinned staging for rt_render / rt_render_rgb8
    int* host_pick = nullptr;     // pinned: a two-pass launch's pass-2 pick, read back (rt::RenderPending)
    size_t host_stage_bytes = 0;
    // Every launch of this context on the device shares `work` (pixel counters + launch constants)
    // and reads the scene buffers, so launches are ordered across streams: `done` is recorded after
    // each launch on its stream `last`; a launch on another stream, and every scene / IBL upload,
    // first waits for it (order_after_last).
    hipEvent_t done = nullptr;
    hipStream_t last = nullptr;
    bool pending = false;
};

}  // namespace

struct rt_ctx {
    std::vector<Device> devs;
    HostScene hs;
    bool have_scene = false;
    bool have_env = false;
    int ibl_w = 0, ibl_h = 0;
    int traversal = RT_TRAVERSAL_FAST;
    int bvh_layout = RT_BVH_SAH;
    int brute_max = RT_BRUTE_MAX_DEFAULT;
    int resume_min = -1;
    int team = 0;  // brute-force lanes per pixel, 0 = auto
    int walk_team = 0;  // tree walk (BVH2 item steps): lanes per pixel walking each ray together, 0 = auto
    int max_waves = 0;  // persistent grid cap in waves per SIMD, 0 = occupancy limit
    int step = 0;       // tree-walk traversal loop: 0 auto, 1 one item per step, 2 descend-until-leaf rounds
    int sun_skip = 1;   // FAST: do not trace shadow rays of an unlit sun (FrameParams::sun_skip)
    int sun_any = 1;    // FAST tree walk: shadow rays end at their first hit when no material is glass
    int block = 128;
    int bvh_width = 0;  // FAST tree walk: 2 = BVH2 nodes, 4 = the 4-wide quantised layout, 0 = auto (option "bvh_width")
    int fixed_point = 1;  // sum the repeats of a sample that draws no random number (FrameParams::fixed_point)
    int sun_cache = 1;    // trace the first drawing bounce's shadow ray once per pixel (FrameParams::sun_cache)
    int pilot = -1;       // two-pass launches: pilot samples per pixel (0 = one pass, -1 = auto; FrameParams::pilot)
    int pilot_chunk = 0;  // pixels ordered together (0 = auto: 64 brute force, 1 tree walk)
    int pilot_levels = 0; // cost bins of the order (0 = auto: 256)
    int stack_lds = 0;    // FAST stack entries per lane kept in LDS (0 = auto: rt::kStackLds, kStackLdsWide)
    int ref_stack = 20;   // REF traversal stack capacity (20 = the reference's, stack.cl:4)
    int spec = -1;        // small tiles: speculative trails per pixel in pass 2 (0 = off, 2, 4 or 8, -1 = auto)
    int wdq = 1;          // 4-wide walk: origin-folded dequantisation where the builder's gap covers the frame (option "wdq")
    int handout = -1;     // pixel hand-out: 0 = interleaved chunks, 1 = a contiguous block per XCD group, -1 = auto
    int slices = -1;      // one-pass tree-walk launches: sample slices per pixel (FrameParams::slices; 0 off, -1 auto)
    // host wall times of the last calls (rt_debug_timings), ms: rt_set_scene's validation + packing and its
    // uploads (+ the per-triangle frame kernel), rt_set_env (upload + texel-sum kernel), rt_render's
    // blocking render + read-back
    double t_pack_ms = 0, t_upload_ms = 0, t_env_ms = 0, t_render_ms = 0;
    std::string err;
};

namespace {

int set_err(rt_ctx* ctx, int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (ctx) ctx->err = buf;
    g_thread_error = buf;
    return code;
}

#define HIP_OR_RET(ctx, call)                                                                           \
    do {                                                                                                \
        hipError_t e_ = (call);                                                                         \
        if (e_ != hipSuccess)                                                                           \
            return set_err((ctx), RT_ERR_HIP, "%s failed: %s", #call, hipGetErrorString(e_));           \
    } while (0)

hipError_t ensure(DevBuf& b, size_t bytes) {
    if (b.bytes >= bytes && b.p) return hipSuccess;
    if (b.p) {
        hipError_t e = hipFree(b.p);
        if (e != hipSuccess) return e;
        b.p = nullptr;
        b.bytes = 0;
    }
    if (bytes == 0) return hipSuccess;
    hipError_t e = hipMalloc(&b.p, bytes);
    if (e == hipSuccess) b.bytes = bytes;
    return e;
}

void release(DevBuf& b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
}

}  // namespace

namespace {

// HBM part of the FAST traversal stack: (depth - kStackLdsMin) entries for every lane a
// persistent render grid can hold (option "stack_lds" may keep as few as kStackLdsMin in LDS).
constexpr int kStackLdsMin = 8;
hipError_t ensure_stack_ovf(Device& d, const HostScene& hs) {
    const int64_t extra = (int64_t)std::max(hs.depth, hs.wdepth) - kStackLdsMin;
    if (extra <= 0) return hipSuccess;
    return ensure(d.stack_ovf, (size_t)std::max(d.cus, 1) * rt::kMaxLanesPerCu * (size_t)extra * sizeof(int2));
}

hipError_t order_after_last(Device& d, hipStream_t s) {
    if (d.pending && d.last != s) return hipStreamWaitEvent(s, d.done, 0);
    return hipSuccess;
}

hipError_t mark_launch(Device& d, hipStream_t s) {
    d.last = s;
    d.pending = true;
    return hipEventRecord(d.done, s);
}

template <typename T>
hipError_t upload(DevBuf& b, const std::vector<T>& v, hipStream_t s) {
    const size_t bytes = v.size() * sizeof(T);
    hipError_t e = ensure(b, bytes > 0 ? bytes : 16);
    if (e != hipSuccess || bytes == 0) return e;
    return hipMemcpyAsync(b.p, v.data(), bytes, hipMemcpyHostToDevice, s);
}

int effective_traversal(const rt_ctx* ctx) {
    return (ctx->traversal == RT_TRAVERSAL_FAST && ctx->hs.fast_ok) ? RT_TRAVERSAL_FAST : RT_TRAVERSAL_REF;
}

// The 4-wide layout serves the walk when chosen, or (auto) when the BVH2 node array exceeds
// rt::kWideMinBytes.
bool use_wide(const rt_ctx* ctx) {
    if (ctx->hs.wnodes.empty() || ctx->bvh_width == 2) return false;
    return ctx->bvh_width == 4 || (size_t)ctx->hs.nnodes * 16 * rt::kNodeF4 > rt::kWideMinBytes;
}

rt::DevScene dev_scene(const rt_ctx* ctx, const Device& d) {
    rt::DevScene s{};
    s.nodes = (const float4*)d.nodes.p;
    s.nnodes = ctx->hs.nnodes;
    s.root_ref = ctx->hs.root_ref;
    const bool wide = use_wide(ctx);
    s.wnodes = wide ? (const float4*)d.wnodes.p : nullptr;
    s.wleaves = wide ? (const float4*)d.wleaves.p : nullptr;
    s.wroot_ref = ctx->hs.wroot_ref;
    s.wdq_omax = wide ? ctx->hs.wdq_omax : 0.0f;
    for (int k = 0; k < 6; ++k) s.root_box[k] = ctx->hs.root_box[k];
    s.bvh9 = (const float*)d.bvh9.p;
    s.nbvh9 = ctx->hs.nbvh9;
    s.ref_stack = ctx->ref_stack;
    s.tri_geo = (const float4*)d.tri_geo.p;
    s.tri_fast = (const float4*)d.tri_fast.p;
    s.tri_shade = (const float4*)d.tri_shade.p;
    s.tri_frame = (const float4*)d.tri_frame.p;
    s.ntri = ctx->hs.ntri;
    s.mat = (const float*)d.mat.p;
    s.nmat = ctx->hs.nmat;
    s.ibl_sum = (const uint32_t*)d.ibl_sum.p;
    s.ibl_w = ctx->ibl_w;
    s.ibl_h = ctx->ibl_h;
    // stack sized for whichever layout the launch picks (launch_fast uses the wide one only for the
    // resumable walk of scenes not staged in LDS)
    s.depth = wide ? std::max(ctx->hs.depth, ctx->hs.wdepth) : ctx->hs.depth;
    s.brute = (const float4*)d.brute.p;
    s.brute_box = (const float4*)d.brute_box.p;
    s.nbrute = ctx->hs.nbrute;
    s.nbox = ctx->hs.nbox;
    s.stack_lds = std::min<int32_t>(s.depth > 0 ? s.depth : 1,
                                    ctx->stack_lds > 0 ? ctx->stack_lds : wide ? rt::kStackLdsWide : rt::kStackLds);
    s.stack_ovf = (int2*)d.stack_ovf.p;
    return s;
}

int check_frame(rt_ctx* ctx, const float* cam, const float* env, int64_t npix, int spp, int row0, int row_step,
                rt::FrameParams* fp) {
    if (!ctx) return set_err(nullptr, RT_ERR_ARG, "null context");
    if (!ctx->have_scene) return set_err(ctx, RT_ERR_STATE, "rt_set_scene has not been called");
    if (!ctx->have_env) return set_err(ctx, RT_ERR_STATE, "rt_set_env has not been called");
    if (!cam || !env) return set_err(ctx, RT_ERR_ARG, "cam/env must not be NULL");
    if (!(cam[6] >= 1.0f) || !(cam[6] < 2147483648.0f))
        return set_err(ctx, RT_ERR_ARG, "cam[6] (row width) must be >= 1, got %g", (double)cam[6]);
    if (npix <= 0 || npix > 0x7fffffff) return set_err(ctx, RT_ERR_ARG, "pixel count %lld out of range", (long long)npix);
    if (spp < 0) return set_err(ctx, RT_ERR_ARG, "spp must be >= 0");
    if (row0 < 0 || row_step <= 0) return set_err(ctx, RT_ERR_ARG, "bad row tiling (%d, %d)", row0, row_step);
    std::memcpy(fp->cam, cam, sizeof fp->cam);
    std::memcpy(fp->env, env, sizeof fp->env);
    fp->width = (int32_t)cam[6];
    fp->npix = npix;
    fp->spp = spp;
    fp->row0 = row0;
    fp->row_step = row_step;
    fp->nloc = rt_tile_rows(npix, fp->width, row0, row_step) * fp->width;
    fp->log_pixel = -1;
    fp->resume_min = ctx->resume_min >= 0 ? ctx->resume_min : use_wide(ctx) ? kResumeMinWide : kResumeMinBvh2;
    fp->step = ctx->step;
    fp->sun_skip = (ctx->sun_skip && env[3] == 0.0f && env[4] >= 0.0f && ctx->hs.colors_finite) ? 1 : 0;
    fp->sun_any = (ctx->sun_any && !ctx->hs.has_glass) ? 1 : 0;
    fp->wide = use_wide(ctx) ? 1 : 0;
    fp->wdq = ctx->wdq;
    fp->fixed_point = ctx->fixed_point;
    fp->sun_cache = ctx->fixed_point && ctx->sun_cache ? 1 : 0;
    fp->pass = 0;
    fp->pilot = 0;
    fp->pilot_chunk = 1;
    fp->pilot_levels = 256;
    fp->pilot_state = nullptr;
    fp->pilot_draws = nullptr;
    fp->spec = 0;
    fp->spec_log = nullptr;
    fp->spec_cap = 0;
    fp->slices = 0;
    fp->slice_state = nullptr;
    fp->slice_ready = nullptr;
    fp->pilot_cost = nullptr;
    fp->pilot_order = nullptr;
    fp->team = ctx->team;
    fp->walk_team = ctx->walk_team;
    fp->max_waves = ctx->max_waves;
    // auto: contiguous per-XCD blocks on the 4-wide walk (C5, same-box A/B twice: 4,998 / 4,984 -> 4,952 /
    // 4,958 ms per frame; its L2-missing walk keeps neighbouring pixels on one XCD's L2), interleaved chunks
    // elsewhere (C3 / C4 -0.5 / +1 %, brute force untested)
    fp->handout = ctx->handout >= 0 ? ctx->handout : (use_wide(ctx) && effective_traversal(ctx) == RT_TRAVERSAL_FAST);
    fp->log_buf = nullptr;
    fp->log_cap = 0;
    fp->log_count = nullptr;
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int rt_create(int n_devices, const int* device_ids, rt_ctx** out) {
    if (!out) return set_err(nullptr, RT_ERR_ARG, "out must not be NULL");
    *out = nullptr;
    int avail = 0;
    hipError_t e = hipGetDeviceCount(&avail);
    if (e != hipSuccess || avail <= 0)
        return set_err(nullptr, RT_ERR_HIP, "no HIP device available (%s)", hipGetErrorString(e));
    if (n_devices <= 0) n_devices = 1;
    // explicit ids may repeat one GPU (KernelLauncher(device=[0, 0]): two row-interleaved slots, each
    // with its own stream and buffers); without ids the first n_devices GPUs must exist
    if (!device_ids && n_devices > avail)
        return set_err(nullptr, RT_ERR_ARG, "requested %d devices, %d available", n_devices, avail);
    if (n_devices > 64) return set_err(nullptr, RT_ERR_ARG, "at most 64 device slots, got %d", n_devices);
    rt_ctx* ctx = new rt_ctx();
    ctx->devs.resize(n_devices);
    for (int i = 0; i < n_devices; ++i) {
        const int id = device_ids ? device_ids[i] : i;
        if (id < 0 || id >= avail) {
            delete ctx;
            return set_err(nullptr, RT_ERR_ARG, "device id %d out of range", id);
        }
        ctx->devs[i].id = id;
        if ((e = hipSetDevice(id)) != hipSuccess ||
            (e = hipStreamCreateWithFlags(&ctx->devs[i].stream, hipStreamNonBlocking)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&ctx->devs[i].done, hipEventDisableTiming)) != hipSuccess ||
            (e = hipDeviceGetAttribute(&ctx->devs[i].cus, hipDeviceAttributeMultiprocessorCount, id)) != hipSuccess) {
            rt_destroy(ctx);
            return set_err(nullptr, RT_ERR_HIP, "device %d init failed: %s", id, hipGetErrorString(e));
        }
    }
    *out = ctx;
    return RT_OK;
}

void rt_destroy(rt_ctx* ctx) {
    if (!ctx) return;
    for (auto& d : ctx->devs) {
        if (hipSetDevice(d.id) != hipSuccess) continue;
        if (d.pending) (void)hipEventSynchronize(d.done);
        if (d.stream) (void)hipStreamSynchronize(d.stream);
        for (DevBuf* b : {&d.stack_ovf, &d.nodes, &d.wnodes, &d.wleaves, &d.tri_fast, &d.brute, &d.brute_box, &d.bvh9, &d.tri_geo, &d.tri_shade, &d.tri_frame, &d.mat, &d.ibl, &d.ibl_sum, &d.out,
                          &d.out8, &d.counts, &d.work, &d.scratch_a, &d.scratch_b, &d.pilot, &d.spec, &d.slice})
            release(*b);
        if (d.host_stage) (void)hipHostFree(d.host_stage);
        if (d.host_pick) (void)hipHostFree(d.host_pick);
        if (d.stream) (void)hipStreamDestroy(d.stream);
        if (d.done) (void)hipEventDestroy(d.done);
    }
    delete ctx;
}

const char* rt_last_error(rt_ctx* ctx) { return ctx ? ctx->err.c_str() : g_thread_error.c_str(); }

int rt_set_option(rt_ctx* ctx, const char* key, int64_t value) {
    if (!ctx || !key) return set_err(ctx, RT_ERR_ARG, "null argument");
    if (!std::strcmp(key, "traversal")) {
        if (value != RT_TRAVERSAL_FAST && value != RT_TRAVERSAL_REF)
            return set_err(ctx, RT_ERR_ARG, "traversal must be 0 (fast) or 1 (ref)");
        ctx->traversal = (int)value;
        return RT_OK;
    }
    if (!std::strcmp(key, "bvh") || !std::strcmp(key, "brute_max")) {
        if (!std::strcmp(key, "bvh")) {
            if (value != RT_BVH_REFERENCE && value != RT_BVH_SAH)
                return set_err(ctx, RT_ERR_ARG, "bvh must be 0 (reference tree) or 1 (sah)");
            ctx->bvh_layout = (int)value;
        } else {
            if (value < 0 || value > 4096) return set_err(ctx, RT_ERR_ARG, "brute_max must be in 0..4096");
            ctx->brute_max = (int)value;
        }
        if (!ctx->have_scene) return RT_OK;
        HostScene& hs = ctx->hs;   // repack the FAST nodes of the current scene
        std::string why;
        rt::pack_checked(hs, hs.bvh9.data(), hs.nbvh9, hs.ntri, ctx->bvh_layout, ctx->brute_max, why);
        for (auto& d : ctx->devs) {
            HIP_OR_RET(ctx, hipSetDevice(d.id));
            HIP_OR_RET(ctx, order_after_last(d, d.stream));
            // a launch in flight on another stream may still read the buffers upload() can free
            HIP_OR_RET(ctx, hipStreamSynchronize(d.stream));
            HIP_OR_RET(ctx, upload(d.nodes, hs.nodes, d.stream));
            HIP_OR_RET(ctx, upload(d.wnodes, hs.wnodes, d.stream));
            HIP_OR_RET(ctx, upload(d.wleaves, hs.wleaves, d.stream));
            HIP_OR_RET(ctx, upload(d.brute, hs.brute, d.stream));
            HIP_OR_RET(ctx, upload(d.brute_box, hs.brute_box, d.stream));
            HIP_OR_RET(ctx, upload(d.tri_geo, hs.tri_geo, d.stream));
            HIP_OR_RET(ctx, upload(d.tri_fast, hs.tri_fast, d.stream));
            HIP_OR_RET(ctx, ensure_stack_ovf(d, hs));
            HIP_OR_RET(ctx, hipStreamSynchronize(d.stream));
        }
        if (!hs.fast_ok) ctx->err = "FAST traversal unavailable (" + why + "); REF traversal will be used";
        return RT_OK;
    }
    if (!std::strcmp(key, "resume_min")) {
        if (value < -1 || value > 64) return set_err(ctx, RT_ERR_ARG, "resume_min must be -1 (auto) or 0..64");
        ctx->resume_min = (int)value;
        return RT_OK;
    }
    if (!std::strcmp(key, "team")) {
        if (value != 0 && value != 1 && value != 2 && value != 4 && value != 8)
            return set_err(ctx, RT_ERR_ARG, "team must be 0 (auto), 1, 2, 4 or 8");
        ctx->team = (int)value;
        return RT_OK;
    }
    if (!std::strcmp(key, "walk_team")) {
        if (value != 0 && value != 1 && value != 2 && value != 4 && value != 8)
            return set_err(ctx, RT_ERR_ARG, "walk_team must be 0 (auto), 1, 2, 4 or 8");
        ctx->walk_team = (int)value;
        return RT_OK;
    }
    if (!std::strcmp(key, "sun_any")) {
        if (value != 0 && value != 1) return set_err(ctx, RT_ERR_ARG, "sun_any must be 0 or 1");
        ctx->sun_any = (int)value;
        return RT_OK;
    }
    if (!std::strcmp(key, "sun_skip")) {
        if (value != 0 && value != 1) return set_err(ctx, RT_ERR_ARG, "sun_skip must be 0 or 1");
        ctx->sun_skip = (int)value;
        return RT_OK;
    }
    if (!std::strcmp(key, "step")) {
        if (value < 0 || value > 2) return set_err(ctx, RT_ERR_ARG, "step must be 0 (auto), 1 (item) or 2 (round)");
        ctx->step = (int)value;
        return RT_OK;
    }
    if (!std::strcmp(key, "waves")) {
        if (value < 0 || value > 8) return set_err(ctx, RT_ERR_ARG, "waves must be in 0..8");
        ctx->max_waves = (int)value;
        return RT_OK;
    }
    if (!std::strcmp(key, "pilot")) {
        if (value < -1 || value > (1 << 20)) return set_err(ctx, RT_ERR_ARG, "pilot must be -1 (auto), 0 (off) or a sample count");
        ctx->pilot = (int)value;
        return RT_OK;
    }
    if (!std::strcmp(key, "pilot_chunk")) {
        if (value < 0 || value > 4096) return set_err(ctx, RT_ERR_ARG, "pilot_chunk must be in 0..4096 (0 = auto)");
        ctx->pilot_chunk = (int)value;
        return RT_OK;
    }
    if (!std::strcmp(key, "pilot_levels")) {
        if (value != 0 && (value < 2 || value > 256)) return set_err(ctx, RT_ERR_ARG, "pilot_levels must be 0 (auto) or 2..256");
        ctx->pilot_levels = (int)value;
        return RT_OK;
    }
    if (!std::strcmp(key, "stack_lds")) {
        if (value != 0 && (value < kStackLdsMin || value > rt::kStackLds))
            return set_err(ctx, RT_ERR_ARG, "stack_lds must be 0 (auto) or %d..%d", kStackLdsMin, rt::kStackLds);
        ctx->stack_lds = (int)value;
        return RT_OK;
    }
    if (!std::strcmp(key, "sun_cache")) {
        if (value != 0 && value != 1) return set_err(ctx, RT_ERR_ARG, "sun_cache must be 0 or 1");
        ctx->sun_cache = (int)value;
        return RT_OK;
    }
    if (!std::strcmp(key, "fixed_point")) {
        if (value != 0 && value != 1) return set_err(ctx, RT_ERR_ARG, "fixed_point must be 0 or 1");
        ctx->fixed_point = (int)value;
        return RT_OK;
    }
    if (!std::strcmp(key, "bvh_width")) {
        if (value != 0 && value != 2 && value != 4) return set_err(ctx, RT_ERR_ARG, "bvh_width must be 0 (auto), 2 or 4");
        ctx->bvh_width = (int)value;
        return RT_OK;
    }
    if (!std::strcmp(key, "ref_stack")) {
        if (value < 20 || value > 64) return set_err(ctx, RT_ERR_ARG, "ref_stack must be in 20..64 (20 = the reference's)");
        ctx->ref_stack = (int)value;
        return RT_OK;
    }
    if (!std::strcmp(key, "slices")) {
        if (value < -1 || value > 16) return set_err(ctx, RT_ERR_ARG, "slices must be -1 (auto), 0 (off) or 1..16");
        ctx->slices = (int)value;
        return RT_OK;
    }
    if (!std::strcmp(key, "wdq")) {
        if (value != 0 && value != 1) return set_err(ctx, RT_ERR_ARG, "wdq must be 0 or 1");
        ctx->wdq = (int)value;
        return RT_OK;
    }
    if (!std::strcmp(key, "handout")) {
        if (value < -1 || value > 1) return set_err(ctx, RT_ERR_ARG, "handout must be -1 (auto), 0 or 1");
        ctx->handout = (int)value;
        return RT_OK;
    }
    if (!std::strcmp(key, "spec")) {
        if (value != -1 && value != 0 && value != 2 && value != 4 && value != 8)
            return set_err(ctx, RT_ERR_ARG, "spec must be -1 (auto), 0 (off), 2, 4 or 8");
        ctx->spec = (int)value;
        return RT_OK;
    }
    if (!std::strcmp(key, "block")) {
        if (value != 64 && value != 128 && value != 256) return set_err(ctx, RT_ERR_ARG, "block must be 64/128/256");
        ctx->block = (int)value;
        return RT_OK;
    }
    return set_err(ctx, RT_ERR_ARG, "unknown option '%s'", key);
}

int rt_set_scene(rt_ctx* ctx, const float* vp, int64_t nvp, const float* vn, int64_t nvn, const float* vuv,
                 int64_t nvuv, const int32_t* face, int64_t nface, const float* mat, int64_t nmat, const float* bvh9,
                 int64_t nbvh) {
    (void)vuv;
    (void)nvuv;  // uv is carried by hitInfo but never consumed by the reference kernel
    if (!ctx) return set_err(nullptr, RT_ERR_ARG, "null context");
    const auto t0 = std::chrono::steady_clock::now();
    HostScene hs;
    std::string msg, why;
    const int rc = rt::scene_prepare(hs, vp, nvp, vn, nvn, face, nface, mat, nmat, bvh9, nbvh, ctx->bvh_layout,
                                     ctx->brute_max, msg, why);
    if (rc != RT_OK) return set_err(ctx, rc, "%s", msg.c_str());
    const auto t1 = std::chrono::steady_clock::now();
    for (auto& d : ctx->devs) {
        HIP_OR_RET(ctx, hipSetDevice(d.id));
        HIP_OR_RET(ctx, order_after_last(d, d.stream));
        // a launch in flight on another stream may still read the buffers upload() / ensure() free
        HIP_OR_RET(ctx, hipStreamSynchronize(d.stream));
        HIP_OR_RET(ctx, upload(d.nodes, hs.nodes, d.stream));
        HIP_OR_RET(ctx, upload(d.wnodes, hs.wnodes, d.stream));
        HIP_OR_RET(ctx, upload(d.wleaves, hs.wleaves, d.stream));
        HIP_OR_RET(ctx, upload(d.brute, hs.brute, d.stream));
        HIP_OR_RET(ctx, upload(d.brute_box, hs.brute_box, d.stream));
        HIP_OR_RET(ctx, ensure_stack_ovf(d, hs));
        HIP_OR_RET(ctx, upload(d.bvh9, hs.bvh9, d.stream));
        HIP_OR_RET(ctx, upload(d.tri_geo, hs.tri_geo, d.stream));
        HIP_OR_RET(ctx, upload(d.tri_fast, hs.tri_fast, d.stream));
        HIP_OR_RET(ctx, upload(d.tri_shade, hs.tri_shade, d.stream));
        HIP_OR_RET(ctx, upload(d.mat, hs.mat, d.stream));
        HIP_OR_RET(ctx, ensure(d.tri_frame, (size_t)std::max<int64_t>(hs.ntri, 1) * 3 * sizeof(float4)));
        HIP_OR_RET(ctx, ensure(d.work, rt::kWorkBytes));
        HIP_OR_RET(ctx, hipStreamSynchronize(d.stream));
    }
    ctx->hs = std::move(hs);
    for (auto& d : ctx->devs) {
        HIP_OR_RET(ctx, hipSetDevice(d.id));
        HIP_OR_RET(ctx, rt::launch_prep_frames(dev_scene(ctx, d), (float4*)d.tri_frame.p, d.stream));
        HIP_OR_RET(ctx, hipStreamSynchronize(d.stream));
    }
    ctx->have_scene = true;
    ctx->t_pack_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    ctx->t_upload_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
    if (!ctx->hs.fast_ok) ctx->err = "FAST traversal unavailable (" + why + "); REF traversal will be used";
    return RT_OK;
}

int rt_set_env(rt_ctx* ctx, const uint8_t* rgba, int w, int h) {
    if (!ctx) return set_err(nullptr, RT_ERR_ARG, "null context");
    if (!rgba || w <= 0 || h <= 0) return set_err(ctx, RT_ERR_ARG, "bad IBL image (%d x %d)", w, h);
    const size_t bytes = (size_t)w * h * 4;
    const auto t0 = std::chrono::steady_clock::now();
    for (auto& d : ctx->devs) {
        HIP_OR_RET(ctx, hipSetDevice(d.id));
        HIP_OR_RET(ctx, order_after_last(d, d.stream));
        HIP_OR_RET(ctx, hipStreamSynchronize(d.stream));   // the old IBL buffer may be freed by ensure
        HIP_OR_RET(ctx, ensure(d.ibl, bytes));
        HIP_OR_RET(ctx, ensure(d.ibl_sum, (size_t)(w + 1) * (size_t)(h + 1) * sizeof(uint32_t)));
        HIP_OR_RET(ctx, hipMemcpyAsync(d.ibl.p, rgba, bytes, hipMemcpyHostToDevice, d.stream));
        HIP_OR_RET(ctx, rt::launch_ibl_sum((const uchar4*)d.ibl.p, w, h, (uint32_t*)d.ibl_sum.p, d.stream));
        HIP_OR_RET(ctx, hipStreamSynchronize(d.stream));
    }
    ctx->ibl_w = w;
    ctx->ibl_h = h;
    ctx->have_env = true;
    ctx->t_env_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return RT_OK;
}

int64_t rt_tile_rows(int64_t npix, int width, int row0, int row_step) {
    if (npix <= 0 || width <= 0 || row0 < 0 || row_step <= 0) return 0;
    const int64_t H = (npix + width - 1) / width;
    if (row0 >= H) return 0;
    return (H - row0 + row_step - 1) / row_step;
}

namespace {
// Sample slices per pixel (setup_slices): auto on the 4-wide walk, and on BVH2 tiles of at least
// kSlicesMinPerLane pixels per resident lane, where they replace the two-pass pilot.  r05 (ms, pilot auto
// vs slices 8 with the pilot off; rows 0::N): C3 N=1 126.5 / 114.8, N=2 78.7 / 65.6, N=4 54.3 / 84.8
// (teams + trails); C4 N=1 303.6 / 284.8, N=2 181.5 / 254.9 (3/4 of C4's pixels are sky, finished by
// the pilot pass: the rest is one pixel per lane, where trails win), N=4 121.4 / 318.4
constexpr int kSlicesWide = 8;
constexpr int kSlicesWideSmall = 12;
constexpr int64_t kSlicesMinPerLane = 4;

// Two-pass launches (FrameParams::pass): FAST tree-walk renders of tiles with more pixels than the
// device keeps lanes resident get a pilot pass of spp / 8 samples (option "pilot": -1 auto, 0 off,
// or K), whose per-pixel costs order the rest of the frame, most expensive first (rt_kernels.hip
// launch_render).  Sets fp's pilot fields and sizes the device's scratch for them.
hipError_t setup_pilot(rt_ctx* ctx, Device& d, rt::FrameParams& fp) {
    if (ctx->pilot == 0 || effective_traversal(ctx) != RT_TRAVERSAL_FAST || fp.nloc <= 0 || use_wide(ctx))
        return hipSuccess;   // (the 4-wide walk is one-pass: its pilot measured slower, r02-r03)
    int k = ctx->pilot;
    if (k < 0) {   // auto: the tree walk on tiles of 1-16 pixels per resident lane (where the tail is long)
        const int64_t lanes = (int64_t)std::max(d.cus, 1) * rt::kWalkLanesPerCu;
        // not on the 4-wide walk (C5), whose L2-missing walk loses the coherence of neighbouring pixels
        // when they are reordered: r03 row tiles 1/2, 1/4, 1/8: 3,005 / 1,626 / 937 ms without the pilot,
        // 3,185 / 1,694 / 938 with it
        if (ctx->hs.nbrute > 0 || use_wide(ctx) || fp.spp < 16 || fp.nloc > 16 * lanes) return hipSuccess;
        // tiles of kSlicesMinPerLane or more pixels per resident lane take sample slices instead (setup_slices)
        if (ctx->slices != 0 && fp.nloc >= kSlicesMinPerLane * lanes) return hipSuccess;
        // spp/8 samples, small tiles (multi-GPU row tiles, whose pass 2 takes teams or speculative trails)
        // included: r04 1/8 tiles with trails, pilot spp/16 / spp/8 / 3spp/16: C4 80.8 / 78.3 / 77.0 ms,
        // C3 35.3 / 33.9 / 35.1 ms; 1/4 tiles C4 120.7 / 119.9 / 129.1, C3 54.8 / 54.8 / 56.1 (r03, teams
        // without trails, had preferred spp/16: C3 49.3 vs 49.9, C4 142 vs 146)
        k = fp.spp / 8;
    }
    if (k >= fp.spp) return hipSuccess;
    const size_t n = (size_t)fp.nloc;
    // state 32 B | cost 4 B | order 4 B per pixel, bin totals + offsets (2 x 256), the chunk costs +
    // chunk order (at most one chunk per pixel), the sort's segment histograms (256 per 256 chunks) and
    // each pixel's pass-1 RNG offset (4 B, pilot_draws)
    const size_t need = n * 40 + 2 * 256 * sizeof(uint32_t) + 2 * (n + 1) * sizeof(uint32_t) +
                        (n + 256) * sizeof(uint32_t) + n * sizeof(uint32_t);
    hipError_t e = hipSuccess;
    // growing frees the old buffer from the host: the last launch (any stream) may still use it
    if (d.pilot.bytes < need && d.pending) e = hipEventSynchronize(d.done);
    if (e == hipSuccess) e = ensure(d.pilot, need);
    if (e != hipSuccess) return e;
    char* base = (char*)d.pilot.p;
    fp.pilot = k;
    fp.pilot_chunk = ctx->pilot_chunk > 0 ? ctx->pilot_chunk : (ctx->hs.nbrute > 0 ? 64 : 1);
    fp.pilot_levels = ctx->pilot_levels > 0 ? ctx->pilot_levels : 256;
    fp.pilot_state = (float4*)base;
    fp.pilot_cost = (uint32_t*)(base + n * 32);
    fp.pilot_order = (const uint32_t*)(base + n * 36);
    fp.pilot_draws = (uint32_t*)(base + need - n * sizeof(uint32_t));
    // speculation (option "spec"): small tiles of the BVH2 walk continue as trails in pass 2
    const int64_t lanes = (int64_t)std::max(d.cus, 1) * rt::kWalkLanesPerCu;
    // up to 4 pixels per resident lane: pass 1 finishes the pixels that draw nothing (sky), and the device
    // picks trails only when the rest is at most one pixel per lane (pilot_team_pick_kernel)
    // (auto); a set trail count applies to any tile
    // (auto); a set trail count applies to any tile.  A trail's record count shares a word with its mode
    // (rt_spec.hip): spp < 2^16
    if (ctx->spec != 0 && (ctx->spec > 0 || fp.nloc <= 4 * lanes) && fp.spp < 65536 && !use_wide(ctx) &&
        ctx->hs.nbrute == 0) {
        fp.spec = ctx->spec;   // 2, 4 or 8 trails, or -1: chosen on the device from the pixels pass 1 left
        // records per trail: a trail t >= 1 starts t (spp - k) / T samples ahead, so it never needs more than
        // spp - k records; past kSpecCapMax it stops and the chain goes on in a trail further ahead or in
        // trail 0 (rt_spec.hip) -- the frame does not depend on the cap, the log size (CUs x lanes x cap x
        // 16 B, at most 1 GB on 256 CUs) no longer grows with spp
        fp.spec_cap = std::min(fp.spp - k, rt::kSpecCapMax);
        const size_t lbytes = rt::spec_log_bytes(fp, d.cus);
        if (d.spec.bytes < lbytes && d.pending) e = hipEventSynchronize(d.done);
        if (e == hipSuccess) e = ensure(d.spec, lbytes);
        if (e != hipSuccess) {
            if (ctx->spec > 0) return e;
            // auto: a device short of memory renders pass 2 without trails (same frame) instead of failing
            (void)hipGetLastError();
            fp.spec = 0;
            fp.spec_cap = 0;
            return hipSuccess;
        }
        fp.spec_log = (float4*)d.spec.p;
    }
    return hipSuccess;
}
}  // namespace

namespace {
// Sample slices (FrameParams::slices; option "slices": -1 auto, 0 or 1 off, K): one-pass launches of the
// resumable tree walk hand out each pixel's samples as K slices, slice-major, so that a tile ends on a
// slice rather than on a whole pixel.  Auto: on the 4-wide walk (C5, whose pixels are all about equally
// long: a tile of n pixels per resident lane ends after ceil(n) pixel times, 2.26 -> 3 on an eighth of
// C5), K = kSlicesWide.  r05, C5 tiles rows 0::N (ms, K = off / 2 / 4 / 8): N=8 826 / 724 / 664 / 635,
// N=4 1,395 / 1,273 / 1,221 / 1,197, N=2 2,536 / 2,409 / 2,361 / 2,343, N=1 4,796 / 4,692 / 4,642 / 4,648
// (the wave cap of 6 instead: 838 / 1,444 / 2,651 / 5,066).  Sets fp's slice fields, sizes the device's
// state buffer and zeroes the samples-done words on stream s (the launch's stream).
hipError_t setup_slices(rt_ctx* ctx, Device& d, rt::FrameParams& fp, hipStream_t s) {
    fp.slices = 0;
    if (effective_traversal(ctx) != RT_TRAVERSAL_FAST || fp.nloc <= 0 || ctx->hs.nbrute > 0 || fp.resume_min <= 0 ||
        ctx->slices == 0)
        return hipSuccess;
    const int64_t lanes = (int64_t)std::max(d.cus, 1) * rt::kWalkLanesPerCu;
    // pilot launches: pass 2 slices the samples after the pilot's when the device gives it one lane per pixel
    // (pilot_team_pick_kernel: more unfinished pixels than lanes); the team and trail kernels take none
    int k = ctx->slices > 0 ? ctx->slices
                            : (use_wide(ctx) || fp.pilot > 0 || fp.nloc >= kSlicesMinPerLane * lanes) ? kSlicesWide : 1;
    // the 4-wide walk's small tiles (under kSlicesMinPerLane pixels per resident lane: C5's eighth, 2.26) take
    // finer slices: 1/8 tile 629.7 / 620.8 ms at 8 / 12 (whole frame 4,594 / 4,612: 8 kept there)
    if (ctx->slices < 0 && use_wide(ctx) &&
        fp.nloc < kSlicesMinPerLane * (int64_t)std::max(d.cus, 1) * rt::kWideWaves * 4 * 64)
        k = kSlicesWideSmall;
    k = std::min(k, (fp.spp - std::max(fp.pilot, 0)) / 2);   // every slice at least two samples
    if (k <= 1 || (int64_t)fp.nloc * k >= ((int64_t)1 << 32)) return hipSuccess;
    const size_t n = (size_t)fp.nloc;
    const size_t need = n * 32 + n * sizeof(uint32_t);
    hipError_t e = hipSuccess;
    // growing frees the old buffer from the host: the last launch (any stream) may still use it
    if (d.slice.bytes < need && d.pending) e = hipEventSynchronize(d.done);
    if (e == hipSuccess) e = ensure(d.slice, need);
    if (e == hipSuccess) e = hipMemsetAsync((char*)d.slice.p + n * 32, 0, n * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    fp.slices = k;
    fp.slice_state = (float4*)d.slice.p;
    fp.slice_ready = (uint32_t*)((char*)d.slice.p + n * 32);
    return hipSuccess;
}

}  // namespace

int rt_render_device(rt_ctx* ctx, int device_index, const float cam[10], const float env[5], int64_t npix, int spp,
                     int max_bounce, int row0, int row_step, float* d_out, void* stream) {
    rt::FrameParams fp;
    int st = check_frame(ctx, cam, env, npix, spp, row0, row_step, &fp);
    if (st) return st;
    if (device_index < 0 || device_index >= (int)ctx->devs.size())
        return set_err(ctx, RT_ERR_ARG, "device index %d out of range", device_index);
    if (!d_out && fp.nloc > 0) return set_err(ctx, RT_ERR_ARG, "d_out must not be NULL");
    if (max_bounce > 4096) return set_err(ctx, RT_ERR_ARG, "maxBounce %d > 4096", max_bounce);
    fp.max_bounce = max_bounce;
    Device& d = ctx->devs[device_index];
    HIP_OR_RET(ctx, hipSetDevice(d.id));
    hipStream_t s = (hipStream_t)stream;  // NULL = the device's default (null) stream, HIP convention
    HIP_OR_RET(ctx, order_after_last(d, s));
    HIP_OR_RET(ctx, setup_pilot(ctx, d, fp));
    HIP_OR_RET(ctx, setup_slices(ctx, d, fp, s));
    HIP_OR_RET(ctx, rt::launch_render(dev_scene(ctx, d), fp, effective_traversal(ctx), ctx->block, d_out, nullptr,
                                      (unsigned int*)d.work.p, s));
    HIP_OR_RET(ctx, mark_launch(d, s));
    return RT_OK;
}

namespace {
// The host half of the read-back: the pinned stage into the caller's (pageable) array, split over up
// to 8 threads for frames of several MB (C2's 12.6 MB: one thread ~0.6 ms, the memory bus takes more
// from several).
void par_copy(char* dst, const char* src, size_t n) {
    constexpr size_t kPiece = 2u << 20;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t k = std::min<size_t>(std::min(8u, hw), n / kPiece);
    if (k <= 1) {
        std::memcpy(dst, src, n);
        return;
    }
    const size_t chunk = ((n + k - 1) / k + 4095) & ~(size_t)4095;
    std::vector<std::thread> ts;
    size_t i = 1;
    // a thread that cannot be created (a thread / cgroup limit) must not throw across the C ABI: the
    // chunks no thread took are copied here
    try {
        for (; i < k && i * chunk < n; ++i)
            ts.emplace_back([=] { std::memcpy(dst + i * chunk, src + i * chunk, std::min(chunk, n - i * chunk)); });
    } catch (...) {
    }
    for (size_t r = i; r < k && r * chunk < n; ++r) std::memcpy(dst + r * chunk, src + r * chunk, std::min(chunk, n - r * chunk));
    std::memcpy(dst, src, std::min(chunk, n));
    for (auto& t : ts) t.join();
}

// rt_render / rt_render_rgb8: every device renders its rows (row r on device r mod n), then, for
// rgb8 >= 0, quantizes them on the device (rgb8 = 1: gamma first) so 1 byte per channel crosses
// PCIe; the host de-interleaves the rows into out (elem = 4 or 1 bytes per channel).
int render_host_(rt_ctx* ctx, const float cam[10], const float env[5], int64_t npix, int spp, int max_bounce,
                 void* out, int rgb8);

int render_host(rt_ctx* ctx, const float cam[10], const float env[5], int64_t npix, int spp, int max_bounce,
                void* out, int rgb8) {
    const auto t0 = std::chrono::steady_clock::now();
    const int st = render_host_(ctx, cam, env, npix, spp, max_bounce, out, rgb8);
    if (ctx) ctx->t_render_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return st;
}

int render_host_(rt_ctx* ctx, const float cam[10], const float env[5], int64_t npix, int spp, int max_bounce,
                 void* out, int rgb8) {
    rt::FrameParams fp0;
    int st = check_frame(ctx, cam, env, npix, spp, 0, 1, &fp0);
    if (st) return st;
    if (!out) return set_err(ctx, RT_ERR_ARG, "output must not be NULL");
    if (max_bounce > 4096) return set_err(ctx, RT_ERR_ARG, "maxBounce %d > 4096", max_bounce);
    const int nd = (int)ctx->devs.size();
    const int W = fp0.width;
    const size_t elem = rgb8 >= 0 ? 1 : sizeof(float);
    // Launch every device, then read back: devices run concurrently.  A two-pass launch's second pass
    // waits for the device's pick after its first pass (rt::RenderPending): every device's first pass is
    // enqueued before the host waits for any.
    std::vector<rt::RenderPending> pend(nd);
    for (int k = 0; k < nd; ++k) {
        Device& d = ctx->devs[k];
        rt::FrameParams fp = fp0;
        fp.row0 = k;
        fp.row_step = nd;
        fp.max_bounce = max_bounce;
        fp.nloc = rt_tile_rows(npix, W, k, nd) * W;
        HIP_OR_RET(ctx, hipSetDevice(d.id));
        const size_t bytes = (size_t)fp.nloc * 3 * elem;
        if (bytes == 0) continue;
        HIP_OR_RET(ctx, ensure(d.out, (size_t)fp.nloc * 3 * sizeof(float)));
        if (d.host_stage_bytes < bytes) {
            if (d.host_stage) HIP_OR_RET(ctx, hipHostFree(d.host_stage));
            d.host_stage = nullptr;
            d.host_stage_bytes = 0;
            HIP_OR_RET(ctx, hipHostMalloc((void**)&d.host_stage, bytes, hipHostMallocDefault));
            d.host_stage_bytes = bytes;
        }
        HIP_OR_RET(ctx, order_after_last(d, d.stream));
        HIP_OR_RET(ctx, setup_pilot(ctx, d, fp));
        HIP_OR_RET(ctx, setup_slices(ctx, d, fp, d.stream));
        if (!d.host_pick) HIP_OR_RET(ctx, hipHostMalloc((void**)&d.host_pick, sizeof(int), hipHostMallocDefault));
        pend[k].host_pick = d.host_pick;
        HIP_OR_RET(ctx, rt::launch_render(dev_scene(ctx, d), fp, effective_traversal(ctx), ctx->block,
                                          (float*)d.out.p, nullptr, (unsigned int*)d.work.p, d.stream, &pend[k]));
        HIP_OR_RET(ctx, mark_launch(d, d.stream));   // (again after pass 2 below; an error in between leaves it ordered)
    }
    for (int k = 0; k < nd; ++k) {
        Device& d = ctx->devs[k];
        const int64_t nloc = rt_tile_rows(npix, W, k, nd) * W;
        const size_t bytes = (size_t)nloc * 3 * elem;
        if (bytes == 0) continue;
        HIP_OR_RET(ctx, hipSetDevice(d.id));
        HIP_OR_RET(ctx, rt::launch_render_finish(dev_scene(ctx, d), effective_traversal(ctx), ctx->block,
                                                 (float*)d.out.p, (unsigned int*)d.work.p, d.stream, pend[k]));
        HIP_OR_RET(ctx, mark_launch(d, d.stream));
        const void* src = d.out.p;
        if (rgb8 >= 0) {
            HIP_OR_RET(ctx, ensure(d.out8, bytes));
            HIP_OR_RET(ctx, rt::launch_rgb8((const float*)d.out.p, (uint8_t*)d.out8.p, nloc * 3, rgb8 == 1,
                                            d.stream));
            src = d.out8.p;
        }
        HIP_OR_RET(ctx, hipMemcpyAsync(d.host_stage, src, bytes, hipMemcpyDeviceToHost, d.stream));
    }
    char* dst = static_cast<char*>(out);
    for (int k = 0; k < nd; ++k) {
        Device& d = ctx->devs[k];
        HIP_OR_RET(ctx, hipSetDevice(d.id));
        HIP_OR_RET(ctx, hipStreamSynchronize(d.stream));
        const int64_t rows = rt_tile_rows(npix, W, k, nd);
        if (nd == 1) {
            par_copy(dst, d.host_stage, (size_t)npix * 3 * elem);
            continue;
        }
        for (int64_t r = 0; r < rows; ++r) {
            const int64_t gr = (int64_t)k + r * nd;
            const int64_t first = gr * W;
            const int64_t count = std::min<int64_t>(W, npix - first);
            std::memcpy(dst + 3 * first * elem, d.host_stage + 3 * r * W * elem, (size_t)count * 3 * elem);
        }
    }
    return RT_OK;
}
}  // namespace

int rt_render(rt_ctx* ctx, const float cam[10], const float env[5], int64_t npix, int spp, int max_bounce,
              float* out_rgb) {
    return render_host(ctx, cam, env, npix, spp, max_bounce, out_rgb, -1);
}

int rt_render_rgb8(rt_ctx* ctx, const float cam[10], const float env[5], int64_t npix, int spp, int max_bounce,
                   int gamma, uint8_t* out_rgb8) {
    if (ctx && gamma != 0 && gamma != 1) return set_err(ctx, RT_ERR_ARG, "gamma must be 0 or 1");
    return render_host(ctx, cam, env, npix, spp, max_bounce, out_rgb8, gamma);
}

int rt_rgb8_device(rt_ctx* ctx, int device_index, const float* d_in, uint8_t* d_out, int64_t n, int gamma,
                   void* stream) {
    if (!ctx) return set_err(nullptr, RT_ERR_ARG, "null context");
    if (device_index < 0 || device_index >= (int)ctx->devs.size())
        return set_err(ctx, RT_ERR_ARG, "device_index %d out of range", device_index);
    if (n < 0 || (n > 0 && (!d_in || !d_out)) || (gamma != 0 && gamma != 1))
        return set_err(ctx, RT_ERR_ARG, "bad arguments");
    if (((uintptr_t)d_in & 15) || ((uintptr_t)d_out & 3))
        return set_err(ctx, RT_ERR_ARG, "d_in must be 16-byte and d_out 4-byte aligned");
    HIP_OR_RET(ctx, hipSetDevice(ctx->devs[device_index].id));
    HIP_OR_RET(ctx, rt::launch_rgb8(d_in, d_out, n, gamma == 1, (hipStream_t)stream));
    return RT_OK;
}

int rt_rgb8(rt_ctx* ctx, const float* in, uint8_t* out, int64_t n, int gamma) {
    if (!ctx) return set_err(nullptr, RT_ERR_ARG, "null context");
    if (n < 0 || (n > 0 && (!in || !out)) || (gamma != 0 && gamma != 1))
        return set_err(ctx, RT_ERR_ARG, "bad arguments");
    if (n == 0) return RT_OK;
    Device& d = ctx->devs[0];
    HIP_OR_RET(ctx, hipSetDevice(d.id));
    HIP_OR_RET(ctx, ensure(d.scratch_a, (size_t)n * sizeof(float)));
    HIP_OR_RET(ctx, ensure(d.scratch_b, (size_t)n));
    HIP_OR_RET(ctx, hipMemcpyAsync(d.scratch_a.p, in, (size_t)n * sizeof(float), hipMemcpyHostToDevice, d.stream));
    HIP_OR_RET(ctx, rt::launch_rgb8((const float*)d.scratch_a.p, (uint8_t*)d.scratch_b.p, n, gamma == 1, d.stream));
    HIP_OR_RET(ctx, hipMemcpyAsync(out, d.scratch_b.p, (size_t)n, hipMemcpyDeviceToHost, d.stream));
    HIP_OR_RET(ctx, hipStreamSynchronize(d.stream));
    return RT_OK;
}

namespace {
int count_all(rt_ctx* ctx, const float cam[10], const float env[5], int64_t npix, int spp, int max_bounce, int row0,
              int row_step, uint64_t* counts, int n) {
    rt::FrameParams fp;
    int st = check_frame(ctx, cam, env, npix, spp, row0, row_step, &fp);
    if (st) return st;
    if (!counts) return set_err(ctx, RT_ERR_ARG, "counts must not be NULL");
    if (max_bounce > 4096) return set_err(ctx, RT_ERR_ARG, "maxBounce %d > 4096", max_bounce);
    fp.max_bounce = max_bounce;
    Device& d = ctx->devs[0];
    HIP_OR_RET(ctx, hipSetDevice(d.id));
    const size_t bytes = (size_t)fp.nloc * 3 * sizeof(float);
    HIP_OR_RET(ctx, ensure(d.out, bytes > 0 ? bytes : 16));
    unsigned long long h[16] = {0};
    HIP_OR_RET(ctx, ensure(d.counts, sizeof h));
    HIP_OR_RET(ctx, hipMemsetAsync(d.counts.p, 0, sizeof h, d.stream));
    HIP_OR_RET(ctx, order_after_last(d, d.stream));
    HIP_OR_RET(ctx, rt::launch_render(dev_scene(ctx, d), fp, effective_traversal(ctx), ctx->block, (float*)d.out.p,
                                      (unsigned long long*)d.counts.p, (unsigned int*)d.work.p, d.stream));
    HIP_OR_RET(ctx, mark_launch(d, d.stream));
    HIP_OR_RET(ctx, hipMemcpyAsync(h, d.counts.p, sizeof h, hipMemcpyDeviceToHost, d.stream));
    HIP_OR_RET(ctx, hipStreamSynchronize(d.stream));
    for (int q = 0; q < n; ++q) counts[q] = h[q];
    return RT_OK;
}
}  // namespace

int rt_count_work(rt_ctx* ctx, const float cam[10], const float env[5], int64_t npix, int spp, int max_bounce,
                  int row0, int row_step, uint64_t counts[5]) {
    return count_all(ctx, cam, env, npix, spp, max_bounce, row0, row_step, counts, 5);
}

int rt_count_work_detail(rt_ctx* ctx, const float cam[10], const float env[5], int64_t npix, int spp, int max_bounce,
                         int row0, int row_step, uint64_t counts[16]) {
    return count_all(ctx, cam, env, npix, spp, max_bounce, row0, row_step, counts, 16);
}

int rt_debug_wave_counts(rt_ctx* ctx, const float cam[10], const float env[5], int64_t npix, int spp, int max_bounce,
                         uint64_t counts[9]) {
    return count_all(ctx, cam, env, npix, spp, max_bounce, 0, 1, counts, 9);
}

int rt_work_bytes(rt_ctx* ctx, double out[4]) {
    // Algorithmic bytes per unit: 32 B per box test (24 B AABB + 8 B child/leaf
    // refs), 36 B per triangle test (v0, e1, e2), 40 B per hit record, 16 B per IBL lookup.
    if (!ctx || !out) return set_err(ctx, RT_ERR_ARG, "null argument");
    // out[0] prices counts[9] (box tests) of rt_count_work_detail: a BVH2 node tests 2 child boxes, a
    // 4-wide node up to 4, a wide leaf its exact box again, a REF node 1 -- so every layout is priced
    // per box actually tested
    out[0] = 32.0;
    out[1] = 36.0;
    out[2] = 40.0;
    out[3] = 16.0;
    return RT_OK;
}

int rt_gamma(rt_ctx* ctx, const float* in, float* out, int64_t n) {
    if (!ctx) return set_err(nullptr, RT_ERR_ARG, "null context");
    if (n < 0 || (n > 0 && (!in || !out))) return set_err(ctx, RT_ERR_ARG, "bad arguments");
    if (n == 0) return RT_OK;
    Device& d = ctx->devs[0];
    HIP_OR_RET(ctx, hipSetDevice(d.id));
    const size_t bytes = (size_t)n * sizeof(float);
    HIP_OR_RET(ctx, ensure(d.scratch_a, bytes));
    HIP_OR_RET(ctx, ensure(d.scratch_b, bytes));
    HIP_OR_RET(ctx, hipMemcpyAsync(d.scratch_a.p, in, bytes, hipMemcpyHostToDevice, d.stream));
    HIP_OR_RET(ctx, rt::launch_gamma((const float*)d.scratch_a.p, (float*)d.scratch_b.p, n, d.stream));
    HIP_OR_RET(ctx, hipMemcpyAsync(out, d.scratch_b.p, bytes, hipMemcpyDeviceToHost, d.stream));
    HIP_OR_RET(ctx, hipStreamSynchronize(d.stream));
    return RT_OK;
}

int rt_debug_math(rt_ctx* ctx, int fn, const float* x, const float* y, float* out, int64_t n) {
    if (!ctx || !x || !out || n < 0) return set_err(ctx, RT_ERR_ARG, "bad arguments");
    Device& d = ctx->devs[0];
    HIP_OR_RET(ctx, hipSetDevice(d.id));
    const size_t bytes = (size_t)n * sizeof(float);
    if (!bytes) return RT_OK;
    HIP_OR_RET(ctx, ensure(d.scratch_a, 3 * bytes));
    float* dx = (float*)d.scratch_a.p;
    float* dy = dx + n;
    float* dout = dy + n;
    HIP_OR_RET(ctx, hipMemcpyAsync(dx, x, bytes, hipMemcpyHostToDevice, d.stream));
    if (y) HIP_OR_RET(ctx, hipMemcpyAsync(dy, y, bytes, hipMemcpyHostToDevice, d.stream));
    else HIP_OR_RET(ctx, hipMemsetAsync(dy, 0, bytes, d.stream));
    HIP_OR_RET(ctx, rt::launch_debug_math(fn, dx, dy, dout, n, d.stream));
    HIP_OR_RET(ctx, hipMemcpyAsync(out, dout, bytes, hipMemcpyDeviceToHost, d.stream));
    HIP_OR_RET(ctx, hipStreamSynchronize(d.stream));
    return RT_OK;
}

int rt_debug_trace(rt_ctx* ctx, int traversal, const float* rays, float* out, int64_t n) {
    if (!ctx || !rays || !out || n < 0) return set_err(ctx, RT_ERR_ARG, "bad arguments");
    if (!ctx->have_scene) return set_err(ctx, RT_ERR_STATE, "no scene");
    if (traversal == RT_TRAVERSAL_FAST && !ctx->hs.fast_ok)
        return set_err(ctx, RT_ERR_STATE, "FAST traversal unavailable for this scene");
    if (!n) return RT_OK;
    Device& d = ctx->devs[0];
    HIP_OR_RET(ctx, hipSetDevice(d.id));
    HIP_OR_RET(ctx, ensure(d.scratch_a, (size_t)n * 6 * sizeof(float)));
    HIP_OR_RET(ctx, ensure(d.scratch_b, (size_t)n * 2 * sizeof(float)));
    HIP_OR_RET(ctx, hipMemcpyAsync(d.scratch_a.p, rays, (size_t)n * 6 * sizeof(float), hipMemcpyHostToDevice, d.stream));
    HIP_OR_RET(ctx, order_after_last(d, d.stream));
    HIP_OR_RET(ctx, rt::launch_debug_trace(dev_scene(ctx, d), traversal, (const float*)d.scratch_a.p,
                                           (float*)d.scratch_b.p, n, d.stream));
    HIP_OR_RET(ctx, hipMemcpyAsync(out, d.scratch_b.p, (size_t)n * 2 * sizeof(float), hipMemcpyDeviceToHost, d.stream));
    HIP_OR_RET(ctx, hipStreamSynchronize(d.stream));
    return RT_OK;
}

int rt_debug_pixel_log(rt_ctx* ctx, int traversal, const float cam[10], const float env[5], int64_t npix, int spp,
                       int max_bounce, int64_t pixel, float* log, int cap, int* n_events, float out3[3]) {
    rt::FrameParams fp;
    if (!cam) return set_err(ctx, RT_ERR_ARG, "null cam");
    const int W = (int)cam[6];
    if (W <= 0 || pixel < 0 || pixel >= npix) return set_err(ctx, RT_ERR_ARG, "pixel out of range");
    int st = check_frame(ctx, cam, env, npix, spp, (int)(pixel / W), (int)npix, &fp);
    if (st) return st;
    if (!log || cap <= 0 || !n_events || !out3) return set_err(ctx, RT_ERR_ARG, "bad log buffer");
    if (traversal == RT_TRAVERSAL_FAST && !ctx->hs.fast_ok) traversal = RT_TRAVERSAL_REF;
    fp.max_bounce = max_bounce;
    fp.sun_skip = 0;   // the event log records every ray the reference traces, with its closest hit
    fp.sun_any = 0;
    Device& d = ctx->devs[0];
    HIP_OR_RET(ctx, hipSetDevice(d.id));
    const size_t obytes = (size_t)fp.nloc * 3 * sizeof(float);
    const size_t lbytes = (size_t)cap * 16 * sizeof(float);
    HIP_OR_RET(ctx, ensure(d.scratch_a, obytes + lbytes + 16));
    float* dout = (float*)d.scratch_a.p;
    fp.log_buf = dout + fp.nloc * 3;
    fp.log_count = (int32_t*)(fp.log_buf + (size_t)cap * 16);
    fp.log_cap = cap;
    fp.log_pixel = pixel;
    HIP_OR_RET(ctx, hipMemsetAsync(fp.log_count, 0, sizeof(int32_t), d.stream));
    HIP_OR_RET(ctx, order_after_last(d, d.stream));
    HIP_OR_RET(ctx, rt::launch_debug_log(dev_scene(ctx, d), fp, traversal, dout, (unsigned int*)d.work.p, d.stream));
    HIP_OR_RET(ctx, mark_launch(d, d.stream));
    int32_t n = 0;
    HIP_OR_RET(ctx, hipMemcpyAsync(&n, fp.log_count, sizeof n, hipMemcpyDeviceToHost, d.stream));
    HIP_OR_RET(ctx, hipStreamSynchronize(d.stream));
    if (n > cap) n = cap;
    HIP_OR_RET(ctx, hipMemcpy(log, fp.log_buf, (size_t)n * 16 * sizeof(float), hipMemcpyDeviceToHost));
    HIP_OR_RET(ctx, hipMemcpy(out3, dout + 3 * (pixel % W), 3 * sizeof(float), hipMemcpyDeviceToHost));
    *n_events = n;
    return RT_OK;
}

int rt_debug_timings(rt_ctx* ctx, double out[4]) {
    if (!ctx || !out) return set_err(ctx, RT_ERR_ARG, "bad arguments");
    out[0] = ctx->t_pack_ms;
    out[1] = ctx->t_upload_ms;
    out[2] = ctx->t_env_ms;
    out[3] = ctx->t_render_ms;
    return RT_OK;
}

int rt_debug_scene_info(rt_ctx* ctx, int64_t out[8]) {
    if (!ctx || !out) return set_err(ctx, RT_ERR_ARG, "bad arguments");
    out[0] = ctx->hs.fast_ok ? 1 : 0;
    out[1] = ctx->hs.depth;
    out[2] = ctx->hs.nnodes;
    out[3] = ctx->hs.ntri;
    out[4] = effective_traversal(ctx) == RT_TRAVERSAL_FAST ? ctx->hs.nbrute : 0;
    out[5] = out[4] ? ctx->hs.nbox : 0;
    // the 4-wide layout's origin bound of the origin-folded dequantisation, in millionths (0: none)
    out[6] = ctx->hs.wnodes.empty() ? 0 : (int64_t)std::llround((double)ctx->hs.wdq_omax * 1e6);
    out[7] = 0;
    return RT_OK;
}

}  // extern "C"
