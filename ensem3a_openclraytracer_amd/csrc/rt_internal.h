// Internal interface between the C-ABI layer (rt_api.hip) and the kernels
// (rt_kernels.hip).  Not part of the public boundary.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "rt_layout.h"

namespace rt {

// Device view of one uploaded scene (all pointers are device pointers).
struct DevScene {
    // FAST traversal: BVH2 nodes holding both child boxes, 4 x float4 each:
    //   [0] = c0.min.x, c0.max.x, c0.min.y, c0.max.y
    //   [1] = c1.min.x, c1.max.x, c1.min.y, c1.max.y
    //   [2] = c0.min.z, c0.max.z, c1.min.z, c1.max.z
    //   [3] = child refs (int bits): >= 0 internal node, < 0 leaf = ~(48 * triangle), its tri_geo byte offset
    const float4* nodes;
    int32_t nnodes;        // internal nodes in `nodes`
    int32_t root_ref;      // ref of the root (~(48 * tri) when the root is a leaf)
    // the same tree collapsed to 4-wide nodes with quantised child boxes (rt_api.hip emit_wide):
    // 64 bytes per node, 64-byte leaf records (exact leaf box + a.p, e1, e2 + index) in reference
    // DFS rank order; refs >= 0 node, < 0 ~(64 * rank), INT_MIN empty slot
    const float4* wnodes;
    const float4* wleaves;
    int32_t wroot_ref;
    // every quantised child bound with q > 0 lies 2^-17 P outside its exact bound (rt_api.hip emit_wide),
    // which makes the origin-folded dequantisation conservative for ray origins with |o| <= wdq_omax
    // (about 20 P; 0: no gap, exact form only); launch_fast checks the camera against it per frame
    float wdq_omax;
    float root_box[6];     // min.xyz, max.xyz of the root
    // REF traversal: the reference's own AoS export, 9 floats per node
    const float* bvh9;
    int32_t nbvh9;
    // REF traversal stack capacity: 20 = the reference's (stack.cl:4; a push onto a full stack is dropped,
    // stack.cl:23-24); up to 64 (option "ref_stack") renders the reference's DFS without drops, which
    // separates the pixels a drop changes from those the FAST slab rounding changes
    int32_t ref_stack;
    // triangles in reference order: 3 x float4 (a.p | rank, e1 | index, e2 | 0); REF traversal
    const float4* tri_geo;
    // the same records in the order the FAST tree's leaves are met depth-first (the FAST leaf refs
    // are byte offsets into this array; e1.w gives the triangle's reference index)
    const float4* tri_fast;
    // hit record per triangle: first-vertex normal | material index bits
    const float4* tri_shade;
    // hemisphere frame per triangle (prep_frames_kernel): q, qinv, normalize(n) | colinear flag
    const float4* tri_frame;
    int32_t ntri;
    // materials: the reference's 6 floats [type, r, g, b, roughness, ior] padded to kMatF = 8 (two float4)
    const float* mat;
    int32_t nmat;
    // IBL: the 2x2 texel sums the reference's lookup averages (ibl_sum_kernel), one word per clamped
    // integer coordinate (X, Y) in [0, ibl_w] x [0, ibl_h]: r | g << 10 | b << 20 (each <= 4 x 255)
    const uint32_t* ibl_sum;
    int32_t ibl_w, ibl_h;
    int32_t depth;         // max number of FAST stack entries a ray can need
    // FAST traversal stack: the first stack_lds entries of each lane in LDS, deeper ones
    // (rare) in stack_ovf, a device buffer of (depth - stack_lds) x resident lanes int2 entries
    int32_t stack_lds;
    int2* stack_ovf;
    // FAST on small scenes: one 64-byte record per reachable triangle in reference DFS order
    // (leaf box, a.p, e1, e2, triangle index); nbrute = 0 when the BVH path is used
    const float4* brute;
    int32_t nbrute;
    // the distinct leaf boxes, 2 float4 each (lo.x hi.x lo.y hi.y | lo.z hi.z q0 q1): q0 (and q1 >= 0,
    // int bits) are the records whose leaf box it is.  Padded to whole groups of kBoxGroup with boxes
    // no ray reaches: the lock-step loop loads a group with one scalar wait
    const float4* brute_box;
    int32_t nbox;
};

struct FrameParams {
    float cam[10];
    float env[5];
    int32_t width;       // (int)cam[6]
    int64_t npix;        // frame pixel count (reference imgSize)
    int32_t spp;
    int32_t max_bounce;
    int32_t row0, row_step;
    int64_t nloc;        // pixels in this tile = rows * width
    int32_t resume_min;  // FAST tree walk: resumable traversal, shade once this many lanes are free (0 = off)
    int32_t team;        // brute-force path: lanes per pixel (1, 2, 4, 8; 0 = chosen at launch from the tile size)
    int32_t walk_team;   // FAST tree walk (BVH2 item steps): lanes per pixel walking each ray together (1, 2, 4, 8; 0 = auto)
    int32_t max_waves;   // persistent grid: at most this many waves per SIMD (0 = as many as stay resident)
    int32_t handout;     // pixel hand-out: 0 = chunks interleaved over the XCD groups, 1 = a contiguous block per group
    int32_t step;        // FAST tree walk: 1 = one item per traversal step, 2 = descend-until-leaf rounds, 0 = auto
    // FAST: skip the shadow ray when its result cannot change the sample: envData[3] (sun power) == 0,
    // envData[4] >= 0 and every material colour finite make the sun term of Raytracing.cl:125-137
    // exactly zero whatever the ray hits (set by the host, never for debug logs)
    int32_t sun_skip;
    // FAST tree walk: with no glass material the sun term depends only on whether the shadow ray hits
    // anything (Raytracing.cl:125-137), so its traversal ends at the first accepted triangle
    int32_t sun_any;
    int32_t wide;        // FAST tree walk over the 4-wide quantised layout (DevScene::wnodes)
    int32_t wdq;         // ... with origin-folded dequantisation when DevScene::wdq_omax covers the camera (1, default)
    // a sample that draws no random number (it ends at its first loop head: camera ray escaped or
    // on an emitter) is every later sample of its pixel: the rest are summed without re-running it
    int32_t fixed_point;
    // the shadow ray of a sample's first diffuse or glossy bounce leaves from the same point towards
    // the same sun in every sample of the pixel: traced once, its hit kept (implies fixed_point)
    int32_t sun_cache;
    // Two-pass launches (launch_render, option "pilot"): pass 1 renders the first `pilot` samples of
    // every pixel and saves each unfinished pixel's state (pilot_state: acc.xyz | kc, seed0 seed1 tc s)
    // and the rays it traced (pilot_cost); the pixels are then ordered by that cost, most first
    // (pilot_order); pass 2 continues them in that order, so the last pixels a frame starts are the
    // short ones.  pass 0 = one pass.
    int32_t pass;
    int32_t pilot;
    int32_t pilot_chunk;   // pixels ordered together (consecutive tile pixels; 1 = single pixels)
    int32_t pilot_levels;  // cost bins of the order (2..256); within a bin the chunks keep tile order
    float4* pilot_state;
    uint32_t* pilot_cost;
    uint32_t* pilot_draws;   // BVH2 walk: random numbers each pixel drew in pass 1 (its RNG offset at pilot_state)
    // Pass 2 with sample-parallel speculation (rt_spec.hip, option "spec"): spec trails per pixel, each
    // trail's log of (RNG offset, sample colour) records, spec_cap records per trail; one log per resident
    // lane (a team's trails log the pixel it holds; the logs are reused from record 0 for its next pixel)
    int32_t spec;
    float4* spec_log;
    int32_t spec_cap;
    // Sample slices (option "slices", one-pass launches of the tree walk): each pixel's samples are
    // `slices` jobs of spp / slices samples, handed out slice-major (take_pixel), so a lane's last job
    // is a slice, not a whole pixel: the frame's tail shrinks by that factor.  A job that ends a slice
    // stores the pixel's state (slice_state: acc.xyz | kc, seed0 seed1 tc s; write-through) and then the
    // samples done (slice_ready); the job of the next slice, on any lane, waits for that count and
    // continues from the state.  Every pixel's samples run in order: the frame is the one-pass frame.
    int32_t slices;
    float4* slice_state;
    uint32_t* slice_ready;
    const uint32_t* pilot_order;
    // debug event log of one pixel (rt_debug_pixel_log only; unused by the product launches)
    int64_t log_pixel;
    float* log_buf;
    int32_t log_cap;
    int32_t* log_count;
};

// A two-pass launch's second pass, waiting for the first: pass 2 launches the kernel the device picked
// (pilot_team_pick_kernel) from the pixels pass 1 left, so the host reads that pick back first.
// launch_render with a RenderPending stops once the pick's copy into pinned host memory is enqueued;
// launch_render_finish waits for it and launches pass 2 (render_host starts every device before it
// waits for any).  Without one, launch_render waits itself.
struct RenderPending {
    bool pick = false;        // pass 2 still to launch
    int* host_pick = nullptr; // pinned host int (the caller's)
    FrameParams b{};          // pass 2's parameters
    bool spec_ok = false;
};
// Launch the render kernel; counts != nullptr selects the instrumented build
// (device pointer to 5 uint64 accumulators).
// d_work: kWorkBytes of device scratch (layout above; the counters are zeroed by the launch).
hipError_t launch_render(const DevScene& sc, const FrameParams& fp, int traversal, int block,
                         float* d_out, unsigned long long* d_counts, unsigned int* d_work, hipStream_t stream,
                         RenderPending* pend = nullptr);
hipError_t launch_render_finish(const DevScene& sc, int traversal, int block, float* d_out, unsigned int* d_work,
                                hipStream_t stream, RenderPending& pend);
hipError_t launch_prep_frames(const DevScene& sc, float4* frame, hipStream_t stream);
// the IBL's 2x2 texel-sum table (DevScene::ibl_sum) from the RGBA8 image: (w + 1) x (h + 1) words
hipError_t launch_ibl_sum(const uchar4* rgba, int w, int h, uint32_t* sum, hipStream_t stream);
hipError_t launch_gamma(const float* d_in, float* d_out, int64_t n, hipStream_t stream);
hipError_t launch_rgb8(const float* d_in, uint8_t* d_out, int64_t n, bool gamma, hipStream_t stream);
// Sample-parallel speculation (rt_spec.hip): pass 2 of a pilot launch of the BVH2 walk with fp.spec
// trails per pixel; spec_log_bytes = the size of fp.spec_log it needs on a device of `cus` CUs (one log
// per resident lane, launch_spec keeps the grid within them); at most kSpecTrails trails per pixel;
// the device pick of pass 2 (pilot_team_pick_kernel, read back by launch_render) encodes "T trails" as kSpecPick + T
constexpr int kSpecTrails = 8;
constexpr int kSpecPick = 10;
constexpr int kSpecCapMax = 256;   // records per trail log at most (FrameParams::spec_cap)
// resident lanes per CU of the BVH2 walks (render_resume_kernel, spec_kernel: 4 waves per SIMD)
constexpr int kWalkLanesPerCu = 4 * 4 * 64;
size_t spec_log_bytes(const FrameParams& fp, int cus);
hipError_t launch_spec(const DevScene& sc, const FrameParams& fp, int block, float* d_out, unsigned int* d_work,
                       hipStream_t stream);
bool spec_walk(const DevScene& sc, const FrameParams& fp);
// test hooks
hipError_t launch_debug_math(int fn, const float* x, const float* y, float* out, int64_t n, hipStream_t stream);
hipError_t launch_debug_log(const DevScene& sc, const FrameParams& fp, int traversal, float* d_out,
                            unsigned int* d_work, hipStream_t stream);
hipError_t launch_debug_trace(const DevScene& sc, int traversal, const float* rays, float* out, int64_t n,
                              hipStream_t stream);

}  // namespace rt
