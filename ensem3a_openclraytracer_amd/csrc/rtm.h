/* rtm.h -- the numerics contract of the path tracer.
 *
 * The reference kernel (Kernels/Raytracing.cl, Kernels/MathLib.cl) calls
 * OpenCL builtins (sin, cos, tan, acos, asin, atan2, sqrt, dot, cross,
 * normalize, fmin, fmax) whose exact results are implementation-defined
 * (OpenCL 1.2 s7.4 allows 4 ulp for the trigonometric functions and leaves
 * dot/cross/normalize to the vendor) and compiles under FP_CONTRACT ON, so
 * the vendor decides where a*b+c fuses.  This header pins ONE
 * implementation of each of those builtins, written only with IEEE-754
 * basic operations (+ - * /, correctly rounded sqrtf) and explicit fmaf, so
 * the same source gives bit-identical results when compiled by gcc for x86
 * (the CPU oracle) and by hipcc for gfx950 (the product kernels).  Every
 * translation unit that includes it must be built with -ffp-contract=off and
 * without -ffast-math; contraction happens only where a function below calls
 * fmaf.
 *
 * Accuracy (measured against float64 numpy in tests/test_numerics.py):
 * sin/cos <= 2 ulp on |x| < 1e5, asin/acos/atan2 <= 3 ulp, tan <= 4 ulp --
 * inside the OpenCL bounds, so this is a conforming implementation of the
 * reference's builtins.
 *
 * Plain C99 and HIP C++ both accept this file.
 */
#ifndef RTM_H
#define RTM_H

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RTM_FN __host__ __device__ static inline
#else
#include <math.h>
#include <stdint.h>
#define RTM_FN static inline
#endif

typedef struct { float x, y, z; } rtm_f3;
typedef struct { float x, y, z, w; } rtm_f4;

RTM_FN rtm_f3 rtm_v3(float x, float y, float z) { rtm_f3 r; r.x = x; r.y = y; r.z = z; return r; }
RTM_FN rtm_f4 rtm_v4(float x, float y, float z, float w) { rtm_f4 r; r.x = x; r.y = y; r.z = z; r.w = w; return r; }
RTM_FN rtm_f3 rtm_add(rtm_f3 a, rtm_f3 b) { return rtm_v3(a.x + b.x, a.y + b.y, a.z + b.z); }
RTM_FN rtm_f3 rtm_sub(rtm_f3 a, rtm_f3 b) { return rtm_v3(a.x - b.x, a.y - b.y, a.z - b.z); }
RTM_FN rtm_f3 rtm_mul(rtm_f3 a, rtm_f3 b) { return rtm_v3(a.x * b.x, a.y * b.y, a.z * b.z); }
RTM_FN rtm_f3 rtm_scale(rtm_f3 a, float s) { return rtm_v3(a.x * s, a.y * s, a.z * s); }
RTM_FN rtm_f3 rtm_div(rtm_f3 a, float s) { return rtm_v3(a.x / s, a.y / s, a.z / s); }

RTM_FN uint32_t rtm_as_uint(float f) { uint32_t u; __builtin_memcpy(&u, &f, 4); return u; }
RTM_FN float rtm_as_float(uint32_t u) { float f; __builtin_memcpy(&f, &u, 4); return f; }
RTM_FN float rtm_nan(void) { return rtm_as_float(0x7fc00000u); }
RTM_FN float rtm_fabs(float x) { return rtm_as_float(rtm_as_uint(x) & 0x7fffffffu); }

/* float -> int with one definition on every platform (C's cast is undefined
 * outside the int range and the CPU and GPU disagree there): NaN -> 0,
 * out-of-range values saturate. */
RTM_FN int rtm_f2i(float x) {
    if (!(x == x)) return 0;
    if (x >= 2147483520.0f) return 2147483647;
    if (x <= -2147483648.0f) return (-2147483647 - 1);
    return (int)x;
}

/* IEEE-754 maxNum/minNum (a NaN operand yields the other one), with equal
 * operands -- including +0/-0 -- resolved to b so the sign of a zero result
 * never depends on the platform's min/max instruction. */
RTM_FN float rtm_fmax(float a, float b) { return (a > b || b != b) ? a : b; }
RTM_FN float rtm_fmin(float a, float b) { return (a < b || b != b) ? a : b; }

/* dot/cross/normalize: the fused forms a vendor library uses. */
RTM_FN float rtm_dot(rtm_f3 a, rtm_f3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
RTM_FN float rtm_dot4(rtm_f4 a, rtm_f4 b) { return fmaf(a.w, b.w, fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x))); }
RTM_FN rtm_f3 rtm_cross(rtm_f3 a, rtm_f3 b) {
    return rtm_v3(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
RTM_FN rtm_f3 rtm_normalize(rtm_f3 v) {
    const float s = 1.0f / sqrtf(rtm_dot(v, v));
    return rtm_scale(v, s);
}
RTM_FN rtm_f4 rtm_normalize4(rtm_f4 v) {
    const float s = 1.0f / sqrtf(rtm_dot4(v, v));
    return rtm_v4(v.x * s, v.y * s, v.z * s, v.w * s);
}

/* ---- trigonometry ------------------------------------------------------ */
#define RTM_PIO2_HI 0x1.921fb6p+0f
#define RTM_PIO2_LO (-0x1.777a5cp-25f)
#define RTM_PIO2_L2 (-0x1.ee59dap-50f)
#define RTM_PI_HI 0x1.921fb6p+1f
#define RTM_PI_LO (-0x1.777a5cp-24f)
#define RTM_PIO4_HI 0x1.921fb6p-1f
#define RTM_PIO4_LO (-0x1.777a5cp-26f)
#define RTM_TWO_OVER_PI 0x1.45f306p-1f

/* sin and cos of x together.  Reduction x = k*pi/2 + r, |r| <= pi/4, by a
 * three-part Cody-Waite constant with fmaf (exact for |k| < 2^17); k is
 * rounded to nearest by the 1.5*2^23 trick (valid for |x| < 6.5e6, beyond
 * which the result is deterministic but meaningless).  Polynomials are the
 * Cephes single-precision minimax fits. */
RTM_FN void rtm_sincos(float x, float* s_out, float* c_out) {
    float kf = x * RTM_TWO_OVER_PI;
    kf = (kf + 12582912.0f) - 12582912.0f;
    float r = fmaf(-kf, RTM_PIO2_HI, x);
    r = fmaf(-kf, RTM_PIO2_LO, r);
    r = fmaf(-kf, RTM_PIO2_L2, r);
    const int q = rtm_f2i(kf) & 3;
    const float z = r * r;
    const float ps = fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
    const float sn = fmaf(ps * z, r, r);
    const float pc = fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
    const float cs = fmaf(pc * z, z, fmaf(-0.5f, z, 1.0f));
    float s, c;
    if (q == 0) { s = sn; c = cs; }
    else if (q == 1) { s = cs; c = -sn; }
    else if (q == 2) { s = -sn; c = -cs; }
    else { s = -cs; c = sn; }
    if (x != x) { s = x; c = x; }
    *s_out = s; *c_out = c;
}
RTM_FN float rtm_sin(float x) { float s, c; rtm_sincos(x, &s, &c); return s; }
RTM_FN float rtm_cos(float x) { float s, c; rtm_sincos(x, &s, &c); return c; }
RTM_FN float rtm_tan(float x) { float s, c; rtm_sincos(x, &s, &c); return s / c; }

/* asin core on [0, 0.5]: w + w^3 P(w^2) (Cephes asinf). */
RTM_FN float rtm_asin_core(float w, float z) {
    const float p = fmaf(fmaf(fmaf(fmaf(4.2163199048e-2f, z, 2.4181311049e-2f), z, 4.5470025998e-2f), z,
                              7.4953002686e-2f), z, 1.6666752422e-1f);
    return fmaf(p * z, w, w);
}
RTM_FN float rtm_asin(float x) {
    const float a = rtm_fabs(x);
    if (!(a <= 1.0f)) return rtm_nan();
    float r;
    if (a > 0.5f) {
        const float z = 0.5f * (1.0f - a);
        const float s = sqrtf(z);
        const float t = rtm_asin_core(s, z);
        r = (RTM_PIO2_HI - (t + t)) + RTM_PIO2_LO;
    } else {
        r = rtm_asin_core(a, a * a);
    }
    return (x < 0.0f) ? -r : r;
}
RTM_FN float rtm_acos(float x) {
    if (!(rtm_fabs(x) <= 1.0f)) return rtm_nan();
    if (x < -0.5f) {
        const float z = 0.5f * (1.0f + x);
        const float s = sqrtf(z);
        const float t = rtm_asin_core(s, z);
        return (RTM_PI_HI - (t + t)) + RTM_PI_LO;
    }
    if (x > 0.5f) {
        const float z = 0.5f * (1.0f - x);
        const float s = sqrtf(z);
        const float t = rtm_asin_core(s, z);
        return t + t;
    }
    return (RTM_PIO2_HI - rtm_asin_core(x, x * x)) + RTM_PIO2_LO;
}

/* atan on all of R (Cephes atanf reduction to |x| <= tan(pi/8)). */
RTM_FN float rtm_atan(float x) {
    float a = rtm_fabs(x);
    float yh, yl;
    if (a > 2.414213562373095f) { yh = RTM_PIO2_HI; yl = RTM_PIO2_LO; a = -1.0f / a; }
    else if (a > 0.4142135623730950f) { yh = RTM_PIO4_HI; yl = RTM_PIO4_LO; a = (a - 1.0f) / (a + 1.0f); }
    else { yh = 0.0f; yl = 0.0f; }
    const float z = a * a;
    const float p = fmaf(fmaf(fmaf(8.05374449538e-2f, z, -1.38776856032e-1f), z, 1.99777106478e-1f), z,
                         -3.33329491539e-1f);
    const float r = yh + (fmaf(p * z, a, a) + yl);
    if (x != x) return x;
    return (x < 0.0f) ? -r : r;
}
/* atan2 with the C99 special cases for signed zeros. */
RTM_FN float rtm_atan2(float y, float x) {
    if (x != x || y != y) return x + y;
    const int xneg = (int)(rtm_as_uint(x) >> 31);
    const int yneg = (int)(rtm_as_uint(y) >> 31);
    if (y == 0.0f) {
        if (!xneg) return y;
        return yneg ? -(RTM_PI_HI + RTM_PI_LO) : (RTM_PI_HI + RTM_PI_LO);
    }
    if (x == 0.0f) return yneg ? -(RTM_PIO2_HI + RTM_PIO2_LO) : (RTM_PIO2_HI + RTM_PIO2_LO);
    const float z = rtm_atan(y / x);
    if (!xneg) return z;
    return yneg ? ((z - RTM_PI_LO) - RTM_PI_HI) : ((z + RTM_PI_LO) + RTM_PI_HI);
}

/* ---- quaternion rotation (MathLib.cl:51-65) ------------------------------
 * quaternion_mult(q,p) = (q.x*p.x - dot(q.yzw,p.yzw),
 *                         q.yzw*p.x + p.yzw*q.x + cross(q.yzw,p.yzw))
 * contracted where OpenCL's FP_CONTRACT ON forms a*b+c. */
RTM_FN rtm_f4 rtm_qmul(rtm_f4 q, rtm_f4 p) {
    const rtm_f3 qv = rtm_v3(q.y, q.z, q.w), pv = rtm_v3(p.y, p.z, p.w);
    const float w = fmaf(q.x, p.x, -rtm_dot(qv, pv));
    const rtm_f3 c = rtm_cross(qv, pv);
    return rtm_v4(w, fmaf(qv.x, p.x, pv.x * q.x) + c.x, fmaf(qv.y, p.x, pv.y * q.x) + c.y,
                  fmaf(qv.z, p.x, pv.z * q.x) + c.z);
}
/* rotateVec(angle, axis, v) (MathLib.cl:56-65), split in two so a rotation
 * whose angle and axis are known ahead (camera, sun, IBL frame, the hemisphere
 * frame of a triangle) is prepared once and applied many times with exactly
 * the same arithmetic:
 *   q    = (cos(angle/2), normalize(axis) * sin(angle/2))
 *   qinv = normalize((q.x, -q.yzw) * (q.x^2 + |q.yzw|^2))
 *   v'   = (q * (0, v) * qinv).yzw                                        */
typedef struct { rtm_f4 q, qinv; } rtm_rot;
RTM_FN rtm_rot rtm_rot_prepare(float angle, rtm_f3 axis) {
    float s, c;
    rtm_sincos(angle * 0.5f, &s, &c);
    const rtm_f3 an = rtm_normalize(axis);
    rtm_rot r;
    r.q = rtm_v4(c, an.x * s, an.y * s, an.z * s);
    const float n2 = fmaf(r.q.x, r.q.x, rtm_dot(rtm_v3(r.q.y, r.q.z, r.q.w), rtm_v3(r.q.y, r.q.z, r.q.w)));
    const rtm_f4 qc = rtm_v4(r.q.x * n2, (r.q.y * -1.0f) * n2, (r.q.z * -1.0f) * n2, (r.q.w * -1.0f) * n2);
    r.qinv = rtm_normalize4(qc);
    return r;
}
RTM_FN rtm_f3 rtm_rot_apply(rtm_rot r, rtm_f3 v) {
    const rtm_f4 V = rtm_v4(0.0f, v.x, v.y, v.z);
    const rtm_f4 t = rtm_qmul(rtm_qmul(r.q, V), r.qinv);
    return rtm_v3(t.y, t.z, t.w);
}
RTM_FN rtm_f3 rtm_rotate(float angle, rtm_f3 axis, rtm_f3 v) {
    return rtm_rot_apply(rtm_rot_prepare(angle, axis), v);
}

/* ---- RNG (MathLib.cl:294-310) -------------------------------------------
 * Two 16-bit multiply-with-carry halves; returns a float in [0,1). */
RTM_FN float rtm_rand(uint32_t* s0, uint32_t* s1) {
    *s0 = 36969u * ((*s1) & 65535u) + ((*s1) >> 16);
    *s1 = 18000u * ((*s0) & 65535u) + ((*s0) >> 16);
    const uint32_t ires = ((*s0) << 16) + (*s1);
    const float f = rtm_as_float((ires & 0x007fffffu) | 0x40000000u);
    return (f - 2.0f) / 2.0f;
}

#endif /* RTM_H */
