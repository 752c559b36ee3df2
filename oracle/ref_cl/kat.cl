// kat.cl -- TEST INFRASTRUCTURE ONLY.  Known-answer-test wrappers around the
// reference's own device functions.  Compiled by oracle/Makefile together with
// the reference sources it includes (-I <reference>/Kernels); nothing from the
// reference is copied here.  Each kernel evaluates one reference function per
// work-item on host-provided inputs so the CPU oracle can be pinned to the
// reference implementation as executed by the ROCm OpenCL runtime.
#include "Raytracing.cl"

__kernel void kat_rand(__global const uint* seeds, const int nd, __global float* out, __global uint* st) {
    int t = get_global_id(0);
    unsigned int s0 = seeds[2 * t], s1 = seeds[2 * t + 1];
    for (int k = 0; k < nd; ++k) out[t * nd + k] = rand(&s0, &s1);
    st[2 * t] = s0;
    st[2 * t + 1] = s1;
}

__kernel void kat_camera(__global float* cam, __global const int* idx, __global float* out) {
    int t = get_global_id(0);
    ray r = genCameraRay(idx[t], cam);
    out[6 * t + 0] = r.dir.x; out[6 * t + 1] = r.dir.y; out[6 * t + 2] = r.dir.z;
    out[6 * t + 3] = r.o.x; out[6 * t + 4] = r.o.y; out[6 * t + 5] = r.o.z;
}

__kernel void kat_rotate(__global const float* in, __global float* out) {
    int t = get_global_id(0);
    __global const float* p = in + 7 * t;
    float3 r = rotateVec(p[0], (float3)(p[1], p[2], p[3]), (float3)(p[4], p[5], p[6]));
    out[3 * t + 0] = r.x; out[3 * t + 1] = r.y; out[3 * t + 2] = r.z;
}

__kernel void kat_intersect(__global const float* in, __global float* out) {
    int t = get_global_id(0);
    __global const float* p = in + 15 * t;
    tri T;
    T.m = 0;
    T.a.uv = (float2)(0, 0); T.b.uv = (float2)(0, 0); T.c.uv = (float2)(0, 0);
    T.a.n = (float3)(0, 0, 0); T.b.n = (float3)(0, 0, 0); T.c.n = (float3)(0, 0, 0);
    T.a.p = (float3)(p[0], p[1], p[2]);
    T.b.p = (float3)(p[3], p[4], p[5]);
    T.c.p = (float3)(p[6], p[7], p[8]);
    ray r;
    r.dir = (float3)(p[9], p[10], p[11]);
    r.o = (float3)(p[12], p[13], p[14]);
    hitInfo h = intersect(T, r);
    out[2 * t + 0] = h.k;
    out[2 * t + 1] = h.bHit ? 1.0f : 0.0f;
}

__kernel void kat_box(__global const float* in, __global int* out) {
    int t = get_global_id(0);
    __global const float* p = in + 12 * t;
    ray r;
    r.dir = (float3)(p[0], p[1], p[2]);
    r.o = (float3)(p[3], p[4], p[5]);
    box b;
    b.min = (float3)(p[6], p[7], p[8]);
    b.max = (float3)(p[9], p[10], p[11]);
    b.center = (float3)(0, 0, 0);
    out[t] = intersectBox(r, b) ? 1 : 0;
}

__kernel void kat_trace(__constant float* vertex_p, __constant float* vertex_n, __constant float* vertex_uv,
                        __constant int* face_data, __constant float* BVH, const int triCount,
                        __global const float* rays, __global float* out) {
    int t = get_global_id(0);
    ray r;
    r.dir = (float3)(rays[6 * t + 0], rays[6 * t + 1], rays[6 * t + 2]);
    r.o = (float3)(rays[6 * t + 3], rays[6 * t + 4], rays[6 * t + 5]);
    hitInfo h = rayTrace(r, vertex_p, vertex_n, vertex_uv, face_data, triCount, BVH);
    out[8 * t + 0] = h.n.x; out[8 * t + 1] = h.n.y; out[8 * t + 2] = h.n.z;
    out[8 * t + 3] = h.k; out[8 * t + 4] = (float)h.mat; out[8 * t + 5] = h.bHit ? 1.0f : 0.0f;
    out[8 * t + 6] = 0.0f; out[8 * t + 7] = 0.0f;
}

__kernel void kat_ggx(__global float* in, __global float* out) {
    int t = get_global_id(0);
    __global float* p = in + 15 * t;
    material m = extractMaterial(p, 0);
    float3 v = (float3)(p[6], p[7], p[8]);
    float3 l = (float3)(p[9], p[10], p[11]);
    float3 n = (float3)(p[12], p[13], p[14]);
    float3 r = BRDF_GGX(m, v, l, n);
    out[3 * t + 0] = r.x; out[3 * t + 1] = r.y; out[3 * t + 2] = r.z;
}

__kernel void kat_ibl(__read_only image2d_t IBL, __global const float* dirs, __global float* out) {
    int t = get_global_id(0);
    const sampler_t sampler = CLK_NORMALIZED_COORDS_FALSE | CLK_ADDRESS_CLAMP_TO_EDGE | CLK_FILTER_LINEAR;
    float3 d = (float3)(dirs[3 * t + 0], dirs[3 * t + 1], dirs[3 * t + 2]);
    float3 c = sampleIBL(d, sampler, IBL);
    float2 uv = SampleSphericalMap(d);
    out[5 * t + 0] = c.x; out[5 * t + 1] = c.y; out[5 * t + 2] = c.z;
    out[5 * t + 3] = uv.x; out[5 * t + 4] = uv.y;
}

// read_imagef with integer coordinates through the reference's sampler
// (Raytracing.cl:179): pins the texel-filter semantics.
__kernel void kat_texel(__read_only image2d_t IBL, __global const int* xy, __global float* out) {
    int t = get_global_id(0);
    const sampler_t sampler = CLK_NORMALIZED_COORDS_FALSE | CLK_ADDRESS_CLAMP_TO_EDGE | CLK_FILTER_LINEAR;
    float4 p = read_imagef(IBL, sampler, (int2)(xy[2 * t], xy[2 * t + 1]));
    out[4 * t + 0] = p.x; out[4 * t + 1] = p.y; out[4 * t + 2] = p.z; out[4 * t + 3] = p.w;
}

__kernel void kat_hemi(const int kind, __global const float* n, __global uint* seeds, __global float* out) {
    int t = get_global_id(0);
    unsigned int s0 = seeds[2 * t], s1 = seeds[2 * t + 1];
    float inv = 0.0f;
    float3 nn = (float3)(n[3 * t + 0], n[3 * t + 1], n[3 * t + 2]);
    float3 d;
    if (kind == 1) d = rand_hemi_cosine(nn, &s0, &s1, &inv);
    else d = rand_hemi_uniform(nn, &s0, &s1, &inv);
    seeds[2 * t] = s0;
    seeds[2 * t + 1] = s1;
    out[4 * t + 0] = d.x; out[4 * t + 1] = d.y; out[4 * t + 2] = d.z; out[4 * t + 3] = inv;
}

__kernel void kat_math(const int fn, __global const float* x, __global const float* y, __global float* out) {
    int t = get_global_id(0);
    float r = 0.0f;
    switch (fn) {
        case 0: r = sin(x[t]); break;
        case 1: r = cos(x[t]); break;
        case 2: r = tan(x[t]); break;
        case 3: r = asin(x[t]); break;
        case 4: r = acos(x[t]); break;
        case 5: r = atan2(x[t], y[t]); break;
        case 6: r = sqrt(x[t]); break;
        case 7: r = x[t] / y[t]; break;
        default: break;
    }
    out[t] = r;
}

// SampleSphericalMap alone (MathLib.cl:72-80): the direction -> uv mapping of
// the IBL lookup, which needs no image object.
__kernel void kat_sphmap(__global const float* dirs, __global float* out) {
    int t = get_global_id(0);
    float2 uv = SampleSphericalMap((float3)(dirs[3 * t + 0], dirs[3 * t + 1], dirs[3 * t + 2]));
    out[2 * t + 0] = uv.x;
    out[2 * t + 1] = uv.y;
}
