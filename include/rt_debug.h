/* rt_debug.h -- test hooks of the native library (not part of the drop-in
 * boundary).  Used by tests/ to check the device numerics and single-ray
 * traversal against the CPU oracle. */
#ifndef RT_DEBUG_H
#define RT_DEBUG_H

#include <stdint.h>
#include "rt_api.h"

/* Scheduling and equivalence knobs of rt_set_option (rt_api.h lists the contract's options).  Each
 * renders the same frame as its automatic value (the GPU tests check that bit for bit); the automatic
 * values are the measured defaults.  -1 / 0 = auto where noted.
 *   "resume_min"   resumable tree walk: shade once this many of 64 lanes are free (-1 auto 36 / 48)
 *   "step"         tree-walk traversal loop: 1 one item per step, 2 descend-until-leaf rounds (0 auto)
 *   "team"         brute force: lanes per pixel 1/2/4/8 (0 auto by tile size)
 *   "walk_team"    BVH2 walk: lanes walking each ray of a pixel together 1/2/4/8 (0 auto)
 *   "spec"         pass 2 of a pilot launch: speculative trails per pixel 2/4/8 (0 off, -1 auto)
 *   "slices"       one-pass tree-walk launches: sample slices per pixel 2..16 (0 off, -1 auto)
 *   "pilot"        two-pass launches: pilot samples per pixel (0 one pass, -1 auto);
 *   "pilot_chunk", "pilot_levels"  the pass-2 order's chunk of pixels and cost bins (0 auto)
 *   "handout"      pixel hand-out: 1 a contiguous block per XCD group, 0 interleaved chunks (-1 auto)
 *   "wdq"          4-wide walk: origin-folded dequantisation where the builder's gap covers the camera (1)
 *   "waves"        persistent grid: at most this many waves per SIMD (0 = occupancy limit)
 *   "stack_lds"    FAST stack entries per lane kept in LDS, deeper ones in HBM (0 auto)
 *   "sun_skip", "sun_any", "fixed_point", "sun_cache"  exact shortcuts of the shading loop (1 = on) */

#ifdef __cplusplus
extern "C" {
#endif

/* Evaluate a function of the numerics contract (rtm.h) on device 0 over host
 * arrays: fn 0 sin, 1 cos, 2 tan, 3 asin, 4 acos, 5 atan2(x, y), 6 sqrt,
 * 7 x / y, 8 the FAST walks' Moller-Trumbore reciprocal of x (rt_device.h mt_recip: equal to
 * 1.0f / x for 1e-7 <= |x| <= 2^126 and for infinities and NaN), 9 the kernels' sqrtf, 10 their
 * 1.0f / sqrtf(x) (rt_device.h dev_sqrt / dev_inv_sqrt: the IEEE results for every x), 11 their
 * 1.0f / x (dev_recip, likewise).  y may be NULL for unary functions. */
int rt_debug_math(rt_ctx* ctx, int fn, const float* x, const float* y, float* out, int64_t n);

/* Trace n rays (rays[6*i..] = dir.xyz, origin.xyz) through the uploaded
 * scene with the given traversal on device 0; out[2*i] = k, out[2*i+1] =
 * triangle index (-1 = miss). */
int rt_debug_trace(rt_ctx* ctx, int traversal, const float* rays, float* out, int64_t n);

/* Render pixel `pixel` of the frame and record its path events (16 floats
 * each: kind 1 bounce ray / 2 sun ray / 3 sample end, j, o.xyz, d.xyz, k or
 * -1, material, sampleOut.xyz, 0,0,0), up to cap events, on device 0. */
int rt_debug_pixel_log(rt_ctx* ctx, int traversal, const float cam[10], const float env[5], int64_t npix, int spp,
                       int max_bounce, int64_t pixel, float* log, int cap, int* n_events, float out3[3]);

/* rt_count_work's five counters for the whole frame plus two wave-level
 * ones: out[5] = traversal-loop iterations issued by waves (an iteration
 * counts once per wave however many lanes take part), out[6] = render-loop
 * iterations of all waves.  out[0] + out[1] over 64 * out[5] is the SIMD
 * efficiency of the traversal loop.  Resumable tree walk only: out[7] / out[8] =
 * clock cycles the waves spent outside / inside the traversal rounds. */
int rt_debug_wave_counts(rt_ctx* ctx, const float cam[10], const float env[5], int64_t npix, int spp,
                         int max_bounce, uint64_t out[9]);

/* Scene facts: out[0] = FAST layout available (1/0), out[1] = FAST stack
 * depth, out[2] = internal nodes, out[3] = triangles, out[4] = brute-force
 * records (0: the tree walk renders), out[5] = distinct leaf boxes of the
 * brute-force path, out[6] = the largest camera coordinate magnitude for which
 * the 4-wide walk dequantises origin-folded, in millionths (0: never), out[7] = 0. */
int rt_debug_scene_info(rt_ctx* ctx, int64_t out[8]);

/* Host wall times (ms) of the context's last calls, the parts of SURVEY.md 8(d)'s cold t_render
 * (KernelLauncher.py:33-87 pays all of them on every launch_Raytracing): [0] rt_set_scene's validation
 * and repacking (SAH / 4-wide layouts), [1] its uploads and the per-triangle frame kernel, [2]
 * rt_set_env (IBL upload + texel-sum kernel), [3] the last blocking rt_render / rt_render_rgb8
 * (render + read-back). */
int rt_debug_timings(rt_ctx* ctx, double out[4]);

/* Host-only (no device): the per-axis quantisation of the 4-wide layout (rt_api.hip emit_wide).
 * For up to n = 4 child intervals [lo[c], hi[c]] against the lower corner p, returns the biased
 * exponent byte e (scale 2^(e-127)) and byte bounds with p + qlo[c] * 2^(e-127) <= lo[c] and
 * p + qhi[c] * 2^(e-127) >= hi[c] in fp32 and, for every byte q > 0, at least `gap` outside the
 * interval in exact arithmetic (p + qlo s <= lo - gap, p + qhi s >= hi + gap; gap >= 0), or -1 when
 * no scale up to 2^100 does (non-finite bounds, extents beyond 255 * 2^100): the scene then keeps the
 * BVH2 walk (gap = 0) or quantises without the gap (emit_wide). */
int rt_debug_quantise_axis(float p, const float* lo, const float* hi, int n, float gap, uint8_t* qlo, uint8_t* qhi);

#ifdef __cplusplus
}
#endif
#endif /* RT_DEBUG_H */
