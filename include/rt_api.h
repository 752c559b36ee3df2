/* rt_api.h -- C ABI of the MI355X path-tracing integrator.
 *
 * This is the drop-in boundary for the reference's device path:
 *   KernelLauncher(context, platform, device, queue)      KernelLauncher.py:8-31
 *   KernelLauncher.launch_Raytracing(h_img_out, ...)       KernelLauncher.py:33-87
 *   KernelLauncher.launch_ImgProcessing(h_src, h_out, N)   KernelLauncher.py:90-103
 * which build and enqueue the OpenCL kernels
 *   __kernel Raytracing      Kernels/Raytracing.cl:161-221
 *   __kernel ImgProcessing   Kernels/ImgProcessing.cl:1-10
 * The Python mirror of KernelLauncher (ensem3a_openclraytracer_amd/KernelLauncher.py)
 * binds these entry points with ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions: every function returns 0 on success and a non-zero rt_status
 * otherwise; rt_last_error(ctx) (or rt_last_error(NULL) for failures without
 * a context) then describes the failure.  Host pointers are borrowed for the
 * duration of the call only.  Calls on one context are not thread-safe; use
 * one context per host thread.  No torch types cross this boundary.
 */
#ifndef RT_API_H
#define RT_API_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_ctx rt_ctx;

enum rt_status {
    RT_OK = 0,
    RT_ERR_ARG = 1,       /* invalid argument (shape, index out of range, ...) */
    RT_ERR_HIP = 2,       /* HIP runtime error */
    RT_ERR_STATE = 3,     /* call out of order (e.g. render before set_scene) */
    RT_ERR_SCENE = 4,     /* scene data the kernels cannot accept (bad material type, malformed BVH) */
    RT_ERR_DEGENERATE = 5 /* BVH build would not terminate in the reference (duplicate centroids) */
};

/* Traversal algorithm (rt_set_option "traversal"). */
enum rt_traversal {
    RT_TRAVERSAL_FAST = 0, /* closest-first BVH2 with t-culling and DFS-rank tie break (default) */
    RT_TRAVERSAL_REF = 1   /* the reference's own DFS (MathLib.cl:234-288): no culling, 20-slot stack */
};

/* Tree the FAST traversal walks (rt_set_option "bvh").  Both trees hold the
 * reference's leaf boxes bit for bit and give identical hits; SAH regroups
 * them so fewer nodes are visited. */
enum rt_bvh_layout {
    RT_BVH_REFERENCE = 0, /* the BVH.py tree as exported */
    RT_BVH_SAH = 1        /* surface-area-heuristic regrouping (default) */
};

/* Create a context on n_devices HIP devices (device_ids may be NULL = 0..n-1; explicit ids may
 * repeat a device: each slot renders its own interleaved rows with its own stream and buffers).
 * Replaces the pyopencl Context/CommandQueue/Program build of
 * KernelLauncher.__init__ (KernelLauncher.py:8-31). */
int rt_create(int n_devices, const int* device_ids, rt_ctx** out);
void rt_destroy(rt_ctx* ctx);
/* Last error message of ctx (or of the calling thread when ctx is NULL). */
const char* rt_last_error(rt_ctx* ctx);

/* Upload the scene (replaces the per-launch cl.Buffer uploads of
 * KernelLauncher.py:41-57).  Arrays are the reference's flat layouts:
 * vp/vn float32[3*N], vuv float32[2*N] (may be NULL/empty, never read),
 * face int32[10*T] = [mat, uv0..2, n0..2, p0..2], mat float32[6*M],
 * bvh9 float32[9*nodes] = BVH.py export [L, R, min.xyz, max.xyz, tri|-1].
 * Counts are element counts.  The arrays are copied; the caller may free them. */
int rt_set_scene(rt_ctx* ctx, const float* vp, int64_t nvp, const float* vn, int64_t nvn,
                 const float* vuv, int64_t nvuv, const int32_t* face, int64_t nface,
                 const float* mat, int64_t nmat, const float* bvh9, int64_t nbvh);

/* Upload the IBL environment map: RGBA8, row-major, w*h texels (replaces the
 * cl.Image of KernelLauncher.py:71-72). */
int rt_set_env(rt_ctx* ctx, const uint8_t* rgba, int w, int h);

/* Integer options of the drop-in contract:
 *   "traversal"  an rt_traversal value: FAST (default) or REF = the reference's own DFS, stack.cl's 20 slots;
 *   "bvh"        an rt_bvh_layout value: the tree the FAST walk uses, SAH by default -- same hits;
 *   "bvh_width"  FAST tree walk: 2 = BVH2 nodes, 4 = the 4-wide quantised layout, 0 = auto (4-wide when
 *                the BVH2 node array exceeds 16 MB) -- same frame;
 *   "brute_max"  FAST on scenes of at most this many triangles tests every leaf box in lock-step instead
 *                of walking a tree (default 64, 0 = always walk) -- same hits;
 *   "ref_stack"  REF's stack slots (20 = the reference's; more = no silent drops: the only option that
 *                changes a frame);
 *   "block"      threads per block: 64, 128 or 256.
 * "bvh" and "brute_max" may be changed after rt_set_scene.  Every other key rt_set_option accepts is a
 * scheduling / equivalence knob listed in rt_debug.h: each renders the same frame, and the automatic
 * values are the measured defaults. */
int rt_set_option(rt_ctx* ctx, const char* key, int64_t value);

/* Render one frame, blocking, into caller-owned host memory out_rgb[3*npix]
 * (row-major RGB, clamped to [0,1]).  Semantics of
 * launch_Raytracing(out, ..., cam, envData, imgDim=npix, spp, maxBounce, IBL):
 * the row width is (int)cam[6] and pixel i gets RNG seeds (i % npix, i / npix).
 * With several devices the rows are interleaved over them (row r on device
 * r mod n) and each device copies its rows back. */
int rt_render(rt_ctx* ctx, const float cam[10], const float env[5], int64_t npix, int spp,
              int max_bounce, float* out_rgb);

/* Asynchronous render of the rows row0, row0+row_step, ... (row width
 * (int)cam[6], frame of npix pixels) on device device_index into DEVICE
 * memory d_out (packed: row k of the tile at d_out[3*W*k]), enqueued on the
 * HIP stream `stream` (a hipStream_t; NULL = the default stream).  Used
 * by the multi-process (one rank per GPU) path and the benchmark.  Returns
 * after the launch is enqueued. */
int rt_render_device(rt_ctx* ctx, int device_index, const float cam[10], const float env[5],
                     int64_t npix, int spp, int max_bounce, int row0, int row_step,
                     float* d_out, void* stream);

/* Number of rows rt_render_device writes for (npix, W, row0, row_step). */
int64_t rt_tile_rows(int64_t npix, int width, int row0, int row_step);

/* Same traversal as the render, instrumented: accumulates
 * counts[0] = BVH node fetches, [1] = triangle tests, [2] = rays traced,
 * [3] = environment lookups, [4] = stack overflows (REF traversal drops),
 * for the given tile (device 0, blocking).  Feeds the algorithmic-byte
 * roofline of bench.py. */
int rt_count_work(rt_ctx* ctx, const float cam[10], const float env[5], int64_t npix, int spp,
                  int max_bounce, int row0, int row_step, uint64_t counts[5]);

/* Every counter of the instrumented render of the tile (device 0, blocking):
 * counts[0..4] as rt_count_work, [5] traversal-loop iterations per wave,
 * [6] render-loop iterations per wave, [7]/[8] clock cycles the resumable
 * kernel's waves spend shading / traversing, [9] ray-box slab tests (a FAST
 * node tests 2 boxes, a REF node 1, the brute-force path one per distinct
 * leaf box), [10]/[11]/[12] shading events (naiveGI bounces,
 * Raytracing.cl:58-78) on materials of type 1 (diffuse) / 2 (glossy) /
 * 3 (glass), [13] sun terms evaluated (Raytracing.cl:115-137), [14] samples,
 * [15] 0.  Feeds the VALU roofline of bench.py. */
int rt_count_work_detail(rt_ctx* ctx, const float cam[10], const float env[5], int64_t npix, int spp,
                         int max_bounce, int row0, int row_step, uint64_t counts[16]);

/* Algorithmic bytes per unit of the counters above:
 * out[0] = 32 B per ray-box slab test (counts[9] of rt_count_work_detail:
 * a BVH2 node tests 2 child boxes, a 4-wide node up to 4, a wide leaf its
 * exact box, a REF node 1), out[1] = 36 per triangle test, out[2] = 40 per
 * ray hit record, out[3] = 16 per environment lookup. */
int rt_work_bytes(rt_ctx* ctx, double out[4]);

/* Gamma kernel of ImgProcessing.cl:1-10: out[k] = powr(min(in[k],1), 2.2)
 * for k < n, blocking, host memory. */
int rt_gamma(rt_ctx* ctx, const float* in, float* out, int64_t n);

/* Output stage (8-bit frame), replacing FileManager.saveImg's quantization
 * (FileManager.py:334-336: (data*255).astype('uint8')) and, with gamma = 1,
 * the ImgProcessing.cl gamma applied first (KernelLauncher.launch_ImgProcessing,
 * KernelLauncher.py:90-103): out[k] = (uint8)(v * 255) with v = in[k] or
 * powr(min(in[k],1), 2.2).  Exact truncation for v*255 in [0, 256) -- every
 * rendered value, the frame being clamped to [0,1]; saturating outside it
 * (NaN -> 0).
 *   rt_render_rgb8: rt_render, then quantize on the device(s); 3*npix bytes
 *                   (row-major RGB) into caller-owned host memory, blocking.
 *   rt_rgb8_device: quantize device memory d_in[n] -> d_out[n] on device
 *                   device_index, enqueued on `stream` (the gather of the
 *                   multi-process path moves these bytes); d_in 16-byte and
 *                   d_out 4-byte aligned.
 *   rt_rgb8:        host memory in -> out, blocking (device 0). */
int rt_render_rgb8(rt_ctx* ctx, const float cam[10], const float env[5], int64_t npix, int spp,
                   int max_bounce, int gamma, uint8_t* out_rgb8);
int rt_rgb8_device(rt_ctx* ctx, int device_index, const float* d_in, uint8_t* d_out, int64_t n,
                   int gamma, void* stream);
int rt_rgb8(rt_ctx* ctx, const float* in, uint8_t* out, int64_t n, int gamma);

/* BVH.py export built natively (bit-identical, see bvh_build.cpp):
 * out must hold 9*(2T-1) floats, T = nface/10; *out_nodes = nodes written. */
int rt_bvh_build(const int32_t* face, int64_t nface, const float* vp, int64_t nvp,
                 float* out, int64_t* out_nodes);

/* Device count visible to HIP (0 when no GPU). */
int rt_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* RT_API_H */
