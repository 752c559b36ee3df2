/* rt_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker and the CPU
 * baseline).  Nothing in the product links, imports or calls this file; only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
 *
 * A plain-C restatement of the reference path tracer
 *   Kernels/Raytracing.cl  (kernel Raytracing, naiveGI, genCameraRay, extractMaterial)
 *   Kernels/MathLib.cl     (rayTrace, intersect, intersectBox, samplers, BRDFs, IBL)
 *   Kernels/stack.cl       (the 20-slot traversal stack)
 * one function per reference function, same control flow, same quirks
 * (SURVEY.md Appendix A).  The OpenCL builtins the reference calls
 * (sin/cos/acos/asin/atan2/tan/dot/cross/normalize/fmin/fmax) come from
 * rtm.h, the pinned numerics contract shared with the GPU kernels, so that
 * this oracle and the HIP reference-order traversal are bit-comparable; the
 * oracle is pinned against the reference kernel itself (compiled by ROCm's
 * OpenCL compiler and run by the ROCm OpenCL runtime, oracle/ref_cl/) through
 * the golden fixtures in tests/golden/.
 *
 * Build: oracle/Makefile (gcc -O2 -march=x86-64-v3 -ffp-contract=off -fopenmp).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include "rtm.h"

typedef rtm_f3 float3;

/* ---- reference data structures (MathLib.cl:6-44) ---- */
typedef struct { float u, v; } float2_;
typedef struct { float2_ uv; float3 n, p; } vertex;          /* MathLib.cl:6-10 */
typedef struct { int m; vertex a, b, c; } tri;                /* MathLib.cl:12-16 */
typedef struct { float3 dir, o; } ray;                        /* MathLib.cl:18-21 */
typedef struct { float3 n; float2_ uv; float k; int mat; int bHit; } hitInfo; /* MathLib.cl:23-30 */
typedef struct { int type; float3 color; float roughness; float ior; } material; /* MathLib.cl:32-38 */

typedef struct {
    const float* vp; const float* vn; const float* vuv; const int32_t* face; int32_t triCount;
    const float* mat; int32_t nmat;
    const float* bvh; int64_t nbvh_nodes;
    const uint8_t* ibl; int32_t ibl_w, ibl_h;
} oracle_scene;

/* work counters of the reference traversal (test/diagnostic only) */
typedef struct { uint64_t nodes, tris, rays, env, dropped; } oracle_counts;

/* ---- stack.cl:1-34 ---- */
typedef struct { int top; unsigned capacity; int array[20]; } Stack;
static int st_isFull(Stack* s) { return s->top == (int)(s->capacity - 1); }
static int st_isEmpty(Stack* s) { return s->top == -1; }
static void st_push(Stack* s, int item, oracle_counts* cnt) {
    if (st_isFull(s)) { if (cnt) cnt->dropped++; return; }   /* silently dropped, stack.cl:23-24 */
    s->array[++s->top] = item;
}
static int st_pop(Stack* s) { if (st_isEmpty(s)) return 0; return s->array[s->top--]; }

/* optional event log of one pixel (debug hook oracle_pixel_log; single-threaded use only) */
static float* g_log = NULL;
static int g_log_cap = 0, g_log_n = 0;
static void log_event(float kind, int j, float3 o, float3 d, const hitInfo* h, float3 so) {
    if (!g_log || g_log_n >= g_log_cap) return;
    float* e = g_log + 16 * g_log_n++;
    e[0] = kind; e[1] = (float)j; e[2] = o.x; e[3] = o.y; e[4] = o.z; e[5] = d.x; e[6] = d.y; e[7] = d.z;
    e[8] = h ? (h->bHit ? h->k : -1.0f) : 0.0f; e[9] = h ? (float)h->mat : 0.0f;
    e[10] = so.x; e[11] = so.y; e[12] = so.z; e[13] = 0; e[14] = 0; e[15] = 0;
}

/* ---- Raytracing.cl:5-15 ---- */
static material extractMaterial(const float* mat, int index) {
    material m;
    m.type = (int)mat[index * 6 + 0];
    m.color = rtm_v3(mat[index * 6 + 1], mat[index * 6 + 2], mat[index * 6 + 3]);
    m.roughness = mat[index * 6 + 4];
    m.ior = mat[index * 6 + 5];
    return m;
}

/* ---- Raytracing.cl:18-37 ---- */
static ray genCameraRay(int i, const float* cam) {
    ray r;
    const int W = (int)cam[6];
    const int pixelY = (i + 1) % W;
    const int pixelX = (i - pixelY) / W;
    const float3 focal = rtm_v3(cam[0], cam[1] - (1.0f / (2.0f * rtm_tan(cam[9] / 2.0f))), cam[2]);
    const float3 position = rtm_v3(cam[0], cam[1], cam[2]);
    const float pasX = 1.0f / cam[6];           /* 1.0/cam[6] in double, rounded once to float */
    const float pasY = pasX;
    const float3 pixelCoord = rtm_v3(fmaf((float)pixelY, pasY, -0.5f), 0.0f, fmaf(-(float)pixelX, pasX, 0.5f));
    r.o = position;
    r.dir = rtm_normalize(rtm_sub(rtm_add(position, pixelCoord), focal));
    r.dir = rtm_rotate(cam[3] * (3.14f / 180.0f), rtm_v3(1, 0, 0), r.dir);
    r.dir = rtm_rotate(cam[4] * (3.14f / 180.0f), rtm_v3(0, 1, 0), r.dir);
    r.dir = rtm_rotate(cam[5] * (3.14f / 180.0f), rtm_v3(0, 0, 1), r.dir);
    return r;
}

/* ---- MathLib.cl:72-80 ---- */
static void SampleSphericalMap(float3 d, float* u, float* v) {
    d = rtm_rotate(90.0f * (3.14f / 180.0f), rtm_v3(1, 0, 0), d);
    d = rtm_rotate(90.0f * (3.14f / 180.0f), rtm_v3(0, 1, 0), d);
    float uu = rtm_atan2(d.z, d.x), vv = rtm_asin(d.y);
    uu = uu * 0.1591f; vv = vv * 0.3183f;
    *u = uu + 0.5f; *v = vv + 0.5f;
}

/* read_imagef(IBL, UNNORMALIZED|CLAMP_TO_EDGE|FILTER_LINEAR, int2(x,y)):
 * integer coordinates through a linear sampler = bilinear at (x, y) with texel
 * centres at +0.5, i.e. the equal-weight average of texels (x-1..x, y-1..y),
 * clamped to the edge (pinned by the GPU KAT). */
static float3 ibl_fetch(const oracle_scene* sc, int x, int y) {
    const int W = sc->ibl_w, H = sc->ibl_h;
    int x0 = x > -2147483647 ? x - 1 : x, x1 = x, y0 = y > -2147483647 ? y - 1 : y, y1 = y;
    x0 = x0 < 0 ? 0 : (x0 > W - 1 ? W - 1 : x0);
    x1 = x1 < 0 ? 0 : (x1 > W - 1 ? W - 1 : x1);
    y0 = y0 < 0 ? 0 : (y0 > H - 1 ? H - 1 : y0);
    y1 = y1 < 0 ? 0 : (y1 > H - 1 ? H - 1 : y1);
    const uint8_t* t00 = sc->ibl + 4 * ((int64_t)y0 * W + x0);
    const uint8_t* t10 = sc->ibl + 4 * ((int64_t)y0 * W + x1);
    const uint8_t* t01 = sc->ibl + 4 * ((int64_t)y1 * W + x0);
    const uint8_t* t11 = sc->ibl + 4 * ((int64_t)y1 * W + x1);
    float c[3];
    for (int k = 0; k < 3; ++k) {
        const float s = (float)((int)t00[k] + (int)t10[k] + (int)t01[k] + (int)t11[k]);
        c[k] = s * (1.0f / 1020.0f);
    }
    return rtm_v3(c[0], c[1], c[2]);
}

/* ---- MathLib.cl:84-90 ---- */
static float3 sampleIBL(const oracle_scene* sc, float3 dir, oracle_counts* cnt) {
    float u, v;
    SampleSphericalMap(dir, &u, &v);
    if (cnt) cnt->env++;
    const int x = rtm_f2i(u * (float)sc->ibl_w);   /* (int2)(...) conversion; NaN/overflow pinned by rtm_f2i */
    const int y = rtm_f2i(v * (float)sc->ibl_h);
    return rtm_scale(ibl_fetch(sc, x, y), 1.0f);
}

/* ---- MathLib.cl:117-160 ---- */
static hitInfo intersect(const tri* T, ray r) {
    const float EPSILON = 0.0000001f;
    hitInfo output;
    output.bHit = 0; output.k = 1000.0f; output.mat = 0;
    output.n = rtm_v3(0, 0, 0); output.uv.u = 0; output.uv.v = 0;
    const float3 edge1 = rtm_sub(T->b.p, T->a.p);
    const float3 edge2 = rtm_sub(T->c.p, T->a.p);
    const float3 h = rtm_cross(r.dir, edge2);
    const float a = rtm_dot(edge1, h);
    if (a > -EPSILON && a < EPSILON) return output;
    const float f = 1.0f / a;                     /* 1.0/a: double quotient rounded to float == float quotient */
    const float3 s = rtm_sub(r.o, T->a.p);
    const float u = f * rtm_dot(s, h);
    if (u < 0.0f || u > 1.0f) return output;
    const float3 q = rtm_cross(s, edge1);
    const float v = f * rtm_dot(r.dir, q);
    if (v < 0.0f || u + v > 1.0f) return output;
    const float k = f * rtm_dot(edge2, q);
    if (k > EPSILON) {
        output.n = T->a.n; output.uv = T->a.uv; output.k = k; output.mat = T->m; output.bHit = 1;
    }
    return output;
}

/* ---- MathLib.cl:167-190 (fmin/fmax with NaN-ignoring semantics) ---- */
static int intersectBox(ray r, const float bmin[3], const float bmax[3]) {
    const float tx1 = (bmin[0] - r.o.x) / r.dir.x, tx2 = (bmax[0] - r.o.x) / r.dir.x;
    float tmin = rtm_fmin(tx1, tx2), tmax = rtm_fmax(tx1, tx2);
    const float ty1 = (bmin[1] - r.o.y) / r.dir.y, ty2 = (bmax[1] - r.o.y) / r.dir.y;
    tmin = rtm_fmax(tmin, rtm_fmin(ty1, ty2));
    tmax = rtm_fmin(tmax, rtm_fmax(ty1, ty2));
    const float tz1 = (bmin[2] - r.o.z) / r.dir.z, tz2 = (bmax[2] - r.o.z) / r.dir.z;
    tmin = rtm_fmax(tmin, rtm_fmin(tz1, tz2));
    tmax = rtm_fmin(tmax, rtm_fmax(tz1, tz2));
    return tmax >= tmin;
}

/* ---- MathLib.cl:193-199 ---- */
static int interNode(ray r, const float* BVH, int curr) {
    return intersectBox(r, &BVH[9 * curr + 2], &BVH[9 * curr + 5]);
}

/* ---- MathLib.cl:203-228 ---- */
static tri makeTri(const oracle_scene* sc, int k) {
    tri T;
    T.m = sc->face[k * 10];
    vertex V[3];
    for (int j = 0; j < 3; j++) {
        const int uvId = sc->face[k * 10 + j + 1];
        const int nId = sc->face[k * 10 + j + 4];
        const int pId = sc->face[k * 10 + j + 7];
        V[j].uv.u = sc->vuv ? sc->vuv[uvId * 2 + 0] : 0.0f;
        V[j].uv.v = sc->vuv ? sc->vuv[uvId * 2 + 1] : 0.0f;
        V[j].n = rtm_v3(sc->vn[nId * 3 + 0], sc->vn[nId * 3 + 1], sc->vn[nId * 3 + 2]);
        V[j].p = rtm_v3(sc->vp[pId * 3 + 0], sc->vp[pId * 3 + 1], sc->vp[pId * 3 + 2]);
    }
    T.a = V[0]; T.b = V[1]; T.c = V[2];
    return T;
}

/* ---- MathLib.cl:234-288: pre-order DFS, push left then right (right popped first),
 * no closest-first ordering and no t culling; hits kept when 1e-4 < k < H.k. ---- */
static hitInfo rayTrace(const oracle_scene* sc, ray r, oracle_counts* cnt) {
    hitInfo H;
    H.n = rtm_v3(0, 0, 0); H.uv.u = 0; H.uv.v = 0; H.k = 1000.0f; H.mat = 0; H.bHit = 0;
    if (cnt) cnt->rays++;
    if (sc->nbvh_nodes <= 0) return H;
    const float* BVH = sc->bvh;
    Stack S;
    S.capacity = 20; S.top = -1;
    st_push(&S, 0, cnt);
    while (!st_isEmpty(&S)) {
        const int curr = st_pop(&S);
        if (cnt) cnt->nodes++;
        if (interNode(r, BVH, curr)) {
            if ((int)(BVH[9 * curr + 8]) != -1) {
                const tri T = makeTri(sc, (int)(BVH[9 * curr + 8]));
                if (cnt) cnt->tris++;
                const hitInfo HTemp = intersect(&T, r);
                if (HTemp.bHit && HTemp.k < H.k && HTemp.k > 0.0001f) H = HTemp;
            }
            if ((int)(BVH[9 * curr]) != -1) st_push(&S, (int)(BVH[9 * curr]), cnt);
            if ((int)(BVH[9 * curr + 1]) != -1) st_push(&S, (int)(BVH[9 * curr + 1]), cnt);
        }
    }
    if (H.k <= 0.0001f) { H.bHit = 0; H.k = 0.0f; }
    return H;
}

/* ---- MathLib.cl:313-339 ---- */
static float3 rand_hemi_cosine(float3 dir, uint32_t* seed0, uint32_t* seed1, float* invPdf) {
    const float u = rtm_rand(seed0, seed1);
    const float theta = rtm_rand(seed0, seed1) * 2.0f * 3.14f;
    const float r = sqrtf(u);
    float st, ct;
    rtm_sincos(theta, &st, &ct);
    const float x = r * ct, y = r * st;
    const float3 localV = rtm_v3(x, y, sqrtf(rtm_fmax(0.0f, 1.0f - u)));
    float3 l;
    const float colinear = rtm_fabs(rtm_dot(rtm_normalize(dir), rtm_v3(0.0f, 0.0f, 1.0f)));
    if (colinear == 1.0f) {
        l = rtm_scale(localV, dir.z);
    } else {
        const float3 axis = rtm_cross(rtm_v3(0, 0, 1), dir);
        const float rotAngle = rtm_acos(rtm_dot(dir, rtm_v3(0, 0, 1)));
        l = rtm_normalize(rtm_rotate(rotAngle, axis, localV));
    }
    *invPdf = 3.14f / (rtm_fmax(rtm_dot(l, dir), 0.0f));
    return l;
}

/* ---- MathLib.cl:342-366 ---- */
static float3 rand_hemi_uniform(float3 dir, uint32_t* seed0, uint32_t* seed1, float* invPdf) {
    const float phi = 2.0f * 3.14f * (rtm_rand(seed0, seed1));
    const float theta = rtm_acos(1.0f - (rtm_rand(seed0, seed1)));
    float sp, cp, sth, cth;
    rtm_sincos(phi, &sp, &cp);
    rtm_sincos(theta, &sth, &cth);
    const float3 localV = rtm_v3(cp * sth, sth * sp, cth);
    float3 worldV;
    const float colinear = rtm_fabs(rtm_dot(rtm_normalize(dir), rtm_v3(0.0f, 0.0f, 1.0f)));
    if (colinear == 1.0f) {
        worldV = rtm_scale(localV, dir.z);
    } else {
        const float3 axis = rtm_normalize(rtm_cross(rtm_v3(0.0f, 0.0f, 1.0f), dir));
        const float rotAngle = rtm_acos(rtm_dot(dir, rtm_v3(0, 0, 1.0f)));
        worldV = rtm_rotate(rotAngle, axis, localV);
    }
    *invPdf = 2.0f * 3.14f;
    return worldV;
}

/* ---- MathLib.cl:391-395 ---- */
static float3 rand_sample_Glass(float3 v, float* invPdf) { *invPdf = 1.0f; return v; }

/* ---- MathLib.cl:461-500 (pown(x,2) = x*x, pown(x,5) = ((x*x)*(x*x))*x) ---- */
static float3 BRDF_GGX(material m, float3 v, float3 l, float3 n) {
    const float3 h = rtm_normalize(rtm_add(l, v));
    const float alphaSqr = m.roughness * m.roughness;
    const float ndh = rtm_fmax(rtm_dot(n, h), 0.0f);
    const float dd = fmaf(ndh * ndh, alphaSqr - 1.0f, 1.0f);
    const float D = alphaSqr / (3.14f * (dd * dd));
    const float NdotV = rtm_fmax(rtm_dot(n, v), 0.0f);
    const float k = m.roughness * sqrtf(2.0f / 3.14f);
    const float G1 = NdotV / fmaf(NdotV, 1.0f - k, k);
    const float NdotL = rtm_fmax(rtm_dot(n, l), 0.0f);
    const float G2 = NdotL / fmaf(NdotL, 1.0f - k, k);
    const float G = G1 * G2;
    const float F0 = 0.04f;
    const float om = 1.0f - rtm_fmax(rtm_dot(h, v), 0.0f);
    const float om2 = om * om;
    const float p5 = (om2 * om2) * om;
    const float F = fmaf(1.0f - F0, p5, F0);
    const float specular = (F * G * D) *
        (1.0f / rtm_fmax(4.0f * rtm_fmax(rtm_dot(v, n), 0.0f) * rtm_fmax(rtm_dot(l, n), 0.0f), 0.001f));
    float3 kd = rtm_v3(1.0f - F, 1.0f - F, 1.0f - F);
    kd = rtm_scale(kd, 1.0f - 0.5f);
    const float3 diffuse = rtm_div(rtm_mul(kd, m.color), 3.14f);
    return rtm_v3(diffuse.x + specular, diffuse.y + specular, diffuse.z + specular);
}
/* ---- MathLib.cl:503-512 ---- */
static float3 BRDF_Lambert(material m) { return rtm_scale(m.color, 1.0f / 3.14f); }
static float3 BRDF_Glass(material m) { return m.color; }

/* ---- Raytracing.cl:39-153 ---- */
static float3 naiveGI(float3 sampleOut, int maxBounce, hitInfo H_cam, ray R_cam, material camMat,
                      const oracle_scene* sc, uint32_t* seed0, uint32_t* seed1, const float* envData,
                      oracle_counts* cnt) {
    for (int j = 0; j <= maxBounce; j++) {
        if (H_cam.bHit) {
            if (camMat.type != 0) {
                ray R_bounce;
                float3 BRDF = rtm_v3(0, 0, 0);
                float invPdfBounce = 0.0f;
                R_bounce.dir = rtm_v3(0, 0, 0);
                switch (camMat.type) {
                    case 1:
                        R_bounce.dir = rand_hemi_cosine(H_cam.n, seed1, seed0, &invPdfBounce);
                        BRDF = BRDF_Lambert(camMat);
                        break;
                    case 2:
                        R_bounce.dir = rand_hemi_uniform(H_cam.n, seed1, seed0, &invPdfBounce);
                        BRDF = BRDF_GGX(camMat, rtm_scale(R_cam.dir, -1.0f), R_bounce.dir, H_cam.n);
                        break;
                    case 3:
                        R_bounce.dir = rand_sample_Glass(R_cam.dir, &invPdfBounce);
                        BRDF = BRDF_Glass(camMat);
                        invPdfBounce = (1.0f) / rtm_fabs(rtm_dot(R_bounce.dir, rtm_normalize(H_cam.n)));
                        break;
                    default: break;   /* unreachable: the launcher rejects material types outside 0..3 */
                }
                const float3 nd = rtm_normalize(R_cam.dir);
                R_bounce.o = rtm_v3(fmaf(nd.x, H_cam.k, R_cam.o.x), fmaf(nd.y, H_cam.k, R_cam.o.y),
                                    fmaf(nd.z, H_cam.k, R_cam.o.z));
                const hitInfo H_bounce = rayTrace(sc, R_bounce, cnt);
                const material bounceMat = extractMaterial(sc->mat, H_bounce.mat);
                const float att = invPdfBounce * rtm_fabs(rtm_dot(R_bounce.dir, rtm_normalize(H_cam.n)));
                sampleOut = rtm_scale(rtm_mul(sampleOut, BRDF), att);
                log_event(1.0f, j, R_bounce.o, R_bounce.dir, &H_bounce, sampleOut);
                if (H_bounce.bHit) {
                    R_cam = R_bounce; H_cam = H_bounce; camMat = bounceMat;
                    if (bounceMat.type != 0) {
                        if (j == maxBounce) { sampleOut = rtm_v3(0, 0, 0); break; }
                    } else {
                        sampleOut = rtm_scale(sampleOut, bounceMat.roughness);
                        break;
                    }
                } else {
                    float3 sunVec = rtm_v3(1, 1, 1);
                    sunVec = rtm_rotate(envData[0] * (3.14f / 180.0f), rtm_v3(1, 0, 0), sunVec);
                    sunVec = rtm_rotate(envData[1] * (3.14f / 180.0f), rtm_v3(0, 1, 0), sunVec);
                    sunVec = rtm_rotate(envData[2] * (3.14f / 180.0f), rtm_v3(0, 0, 1), sunVec);
                    float3 sunLight = rtm_v3(0, 0, 0);
                    ray sunRay; sunRay.o = R_bounce.o; sunRay.dir = sunVec;
                    const hitInfo H_sun = rayTrace(sc, sunRay, cnt);
                    log_event(2.0f, j, sunRay.o, sunRay.dir, &H_sun, sampleOut);
                    const material sunMat = extractMaterial(sc->mat, H_sun.mat);
                    if (!H_sun.bHit && camMat.type != 3) sunLight = rtm_v3(envData[3], envData[3], envData[3]);
                    if (H_sun.bHit && sunMat.type == 3) sunLight = rtm_scale(sunMat.color, envData[3]);
                    const float3 envLight = rtm_scale(sampleIBL(sc, R_bounce.dir, cnt), envData[4]);
                    sampleOut = rtm_mul(sampleOut, rtm_add(sunLight, envLight));
                    break;
                }
            } else {
                sampleOut = rtm_scale(sampleOut, camMat.roughness);
                break;
            }
        } else {
            sampleOut = rtm_scale(rtm_mul(sampleOut, sampleIBL(sc, R_cam.dir, cnt)), envData[4]);
            break;
        }
    }
    return sampleOut;
}

/* ---- Raytracing.cl:161-221, one work-item ---- */
static void raytracing_pixel(const oracle_scene* sc, const float* cam, const float* envData, int i,
                             int imgSize, int maxSpp, int maxBounce, float* out3, oracle_counts* cnt) {
    uint32_t seed0 = (uint32_t)(i % imgSize);
    uint32_t seed1 = (uint32_t)(i / imgSize);
    float3 output = rtm_v3(0, 0, 0);
    const ray r = genCameraRay(i, cam);
    const hitInfo H_cam_cache = rayTrace(sc, r, cnt);
    const material camMat_cache = extractMaterial(sc->mat, H_cam_cache.mat);
    int spp = 0;
    while (spp < maxSpp) {
        spp++;
        const float3 baseColor = naiveGI(rtm_v3(1.0f, 1.0f, 1.0f), maxBounce, H_cam_cache, r, camMat_cache,
                                         sc, &seed0, &seed1, envData, cnt);
        output = rtm_add(output, baseColor);
        log_event(3.0f, spp, rtm_v3(0, 0, 0), rtm_v3(0, 0, 0), NULL, baseColor);
    }
    output = rtm_div(output, (float)maxSpp);
    out3[0] = rtm_fmax(rtm_fmin(output.x, 1.0f), 0.0f);
    out3[1] = rtm_fmax(rtm_fmin(output.y, 1.0f), 0.0f);
    out3[2] = rtm_fmax(rtm_fmin(output.z, 1.0f), 0.0f);
}

/* ================= exported test/baseline API ================= */

/* Render rows row0, row0+row_step, ... of the frame whose row width is
 * (int)cam[6] and whose pixel count is npix (the reference's imgSize).
 * out receives the rows packed: out[3*(k*W + c) + ch] for the k-th rendered
 * row.  Returns the number of rows rendered, or -1 on bad arguments. */
int oracle_render(const oracle_scene* sc, const float* cam, const float* env, int32_t npix, int32_t spp,
                  int32_t max_bounce, int32_t row0, int32_t row_step, int32_t nthreads, float* out,
                  oracle_counts* counts) {
    const int W = (int)cam[6];
    if (W <= 0 || npix <= 0 || row_step <= 0 || row0 < 0) return -1;
    const int H = (npix + W - 1) / W;
    const int nrows = row0 < H ? (H - row0 + row_step - 1) / row_step : 0;
    const int64_t nloc = (int64_t)nrows * W;
    oracle_counts total = {0, 0, 0, 0, 0};
#if defined(_OPENMP)
    if (nthreads <= 0) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
#endif
    {
        oracle_counts local = {0, 0, 0, 0, 0};
#if defined(_OPENMP)
#pragma omp for schedule(dynamic, 64)
#endif
        for (int64_t p = 0; p < nloc; ++p) {
            const int k = (int)(p / W), c = (int)(p % W);
            const int i = (row0 + k * row_step) * W + c;
            if (i >= npix) continue;
            raytracing_pixel(sc, cam, env, i, npix, spp, max_bounce, out + 3 * p, counts ? &local : NULL);
        }
        if (counts) {
#if defined(_OPENMP)
#pragma omp critical
#endif
            {
                total.nodes += local.nodes; total.tris += local.tris; total.rays += local.rays;
                total.env += local.env; total.dropped += local.dropped;
            }
        }
    }
    if (counts) *counts = total;
    return nrows;
}

/* Render pixel i alone and record up to cap events of 16 floats:
 * [kind (1 bounce ray, 2 sun ray, 3 sample end), j, o.xyz, d.xyz, k|-1, mat, sampleOut.xyz, 0,0,0]. */
int oracle_pixel_log(const oracle_scene* sc, const float* cam, const float* env, int32_t npix, int32_t spp,
                     int32_t max_bounce, int32_t i, float* log, int32_t cap, float* out3) {
    g_log = log; g_log_cap = cap; g_log_n = 0;
    raytracing_pixel(sc, cam, env, i, npix, spp, max_bounce, out3, NULL);
    const int n = g_log_n;
    g_log = NULL; g_log_cap = 0; g_log_n = 0;
    return n;
}

/* One sample of pixel i as a function of its RNG offset: for every even offset D = 2p < 2P (draws
 * consumed by the pixel's earlier samples), the sample's colour, the draws it consumes and the rays
 * it traces.  A sample depends on nothing else (the primary hit is cached per pixel,
 * Raytracing.cl:184-206), so the reference's pixel is the chain D0 = 0, D(k+1) = D(k) + draws(D(k))
 * summed in order; tools/chain_speculation.py uses this to price sample-parallel speculation. */
int oracle_sample_trail(const oracle_scene* sc, const float* cam, const float* env, int32_t npix, int32_t max_bounce,
                        int32_t i, int32_t P, float* col, int32_t* draws, int32_t* rays) {
    uint32_t a0 = (uint32_t)(i % npix), a1 = (uint32_t)(i / npix);
    const ray r = genCameraRay(i, cam);
    const hitInfo H = rayTrace(sc, r, NULL);
    const material M = extractMaterial(sc->mat, H.mat);
    for (int p = 0; p < P; ++p) {
        uint32_t b0 = a0, b1 = a1;
        oracle_counts cnt = {0, 0, 0, 0, 0};
        const float3 o = naiveGI(rtm_v3(1.0f, 1.0f, 1.0f), max_bounce, H, r, M, sc, &b0, &b1, env, &cnt);
        col[3 * p] = o.x; col[3 * p + 1] = o.y; col[3 * p + 2] = o.z;
        rays[p] = (int32_t)cnt.rays;
        uint32_t t0 = a0, t1 = a1;
        int n = 0;   /* draws: steps of the (swapped-pointer) stream from the start state to the end state */
        while (!(t0 == b0 && t1 == b1) && n < 4 * (max_bounce + 1) + 2) { rtm_rand(&t1, &t0); ++n; }
        draws[p] = n;
        rtm_rand(&a1, &a0); rtm_rand(&a1, &a0);
    }
    return 0;
}

/* ---- per-function known-answer hooks ---- */
void oracle_rand_stream(uint32_t seed0, uint32_t seed1, int n, float* out, uint32_t* state_out) {
    for (int k = 0; k < n; ++k) out[k] = rtm_rand(&seed0, &seed1);
    state_out[0] = seed0; state_out[1] = seed1;
}
void oracle_camera_ray(const float* cam, int i, float* out6) {
    const ray r = genCameraRay(i, cam);
    out6[0] = r.dir.x; out6[1] = r.dir.y; out6[2] = r.dir.z;
    out6[3] = r.o.x; out6[4] = r.o.y; out6[5] = r.o.z;
}
void oracle_rotate(float angle, const float* axis, const float* v, float* out3) {
    const float3 r = rtm_rotate(angle, rtm_v3(axis[0], axis[1], axis[2]), rtm_v3(v[0], v[1], v[2]));
    out3[0] = r.x; out3[1] = r.y; out3[2] = r.z;
}
/* tri9 = pa, pb, pc; ray6 = dir, o; out = k, hit */
void oracle_intersect(const float* tri9, const float* ray6, float* out2) {
    tri T;
    memset(&T, 0, sizeof T);
    T.a.p = rtm_v3(tri9[0], tri9[1], tri9[2]);
    T.b.p = rtm_v3(tri9[3], tri9[4], tri9[5]);
    T.c.p = rtm_v3(tri9[6], tri9[7], tri9[8]);
    ray r; r.dir = rtm_v3(ray6[0], ray6[1], ray6[2]); r.o = rtm_v3(ray6[3], ray6[4], ray6[5]);
    const hitInfo h = intersect(&T, r);
    out2[0] = h.k; out2[1] = (float)h.bHit;
}
int oracle_box(const float* ray6, const float* box6) {
    ray r; r.dir = rtm_v3(ray6[0], ray6[1], ray6[2]); r.o = rtm_v3(ray6[3], ray6[4], ray6[5]);
    return intersectBox(r, box6, box6 + 3);
}
/* out8 = n.xyz, k, mat, bHit, -, - */
void oracle_trace(const oracle_scene* sc, const float* ray6, float* out8) {
    ray r; r.dir = rtm_v3(ray6[0], ray6[1], ray6[2]); r.o = rtm_v3(ray6[3], ray6[4], ray6[5]);
    const hitInfo h = rayTrace(sc, r, NULL);
    out8[0] = h.n.x; out8[1] = h.n.y; out8[2] = h.n.z; out8[3] = h.k; out8[4] = (float)h.mat;
    out8[5] = (float)h.bHit; out8[6] = 0; out8[7] = 0;
}
void oracle_brdf_ggx(const float* mat6, const float* v, const float* l, const float* n, float* out3) {
    const material m = extractMaterial(mat6, 0);
    const float3 r = BRDF_GGX(m, rtm_v3(v[0], v[1], v[2]), rtm_v3(l[0], l[1], l[2]), rtm_v3(n[0], n[1], n[2]));
    out3[0] = r.x; out3[1] = r.y; out3[2] = r.z;
}
void oracle_sample_ibl(const oracle_scene* sc, const float* dir, float* out3) {
    const float3 c = sampleIBL(sc, rtm_v3(dir[0], dir[1], dir[2]), NULL);
    out3[0] = c.x; out3[1] = c.y; out3[2] = c.z;
}
void oracle_spherical_map(const float* dir, float* out2) {
    SampleSphericalMap(rtm_v3(dir[0], dir[1], dir[2]), &out2[0], &out2[1]);
}
/* kind 1 = cosine, 2 = uniform.  io_seeds = seed0, seed1 as passed by naiveGI
 * (the caller passes &seed1, &seed0 in that order, Raytracing.cl:65,69). */
void oracle_hemi(int kind, const float* n, uint32_t* io_seeds, float* out4) {
    float inv = 0;
    float3 d;
    if (kind == 1) d = rand_hemi_cosine(rtm_v3(n[0], n[1], n[2]), &io_seeds[0], &io_seeds[1], &inv);
    else d = rand_hemi_uniform(rtm_v3(n[0], n[1], n[2]), &io_seeds[0], &io_seeds[1], &inv);
    out4[0] = d.x; out4[1] = d.y; out4[2] = d.z; out4[3] = inv;
}
/* elementary-function hooks for the numerics tests */
void oracle_math(int fn, const float* x, const float* y, float* out, int64_t n) {
    for (int64_t i = 0; i < n; ++i) {
        switch (fn) {
            case 0: out[i] = rtm_sin(x[i]); break;
            case 1: out[i] = rtm_cos(x[i]); break;
            case 2: out[i] = rtm_tan(x[i]); break;
            case 3: out[i] = rtm_asin(x[i]); break;
            case 4: out[i] = rtm_acos(x[i]); break;
            case 5: out[i] = rtm_atan2(x[i], y[i]); break;
            case 6: out[i] = sqrtf(x[i]); break;
            case 7: out[i] = x[i] / y[i]; break;
            default: out[i] = 0; break;
        }
    }
}
