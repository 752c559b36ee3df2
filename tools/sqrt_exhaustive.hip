// Exhaustive check of short square-root sequences against the IEEE sqrtf (correctly rounded, as
// hipcc builds it: -fhip-fp32-correctly-rounded-divide-sqrt) and of the composite 1.0f / sqrtf(x) that
// rtm_normalize computes (rtm.h), over all 2^32 bit patterns, on the GPU (v_sqrt_f32 / v_rsq_f32 have
// no CPU model).
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math -o tools/bin/sqrt_exhaustive tools/sqrt_exhaustive.hip
//   tools/bin/sqrt_exhaustive    -> one JSON line: mismatches per candidate and input class
//
// Classes: 0 = x < 2^-96 or x > 2^126 (incl. denormals, zeros, negatives), 1 = 2^-96 <= x <= 2^126,
// 2 = +inf, 3 = NaN.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int NCAND = 5;

__device__ __forceinline__ float recip4(float a) {   // rt_device.h mt_recip
    const float r = __builtin_amdgcn_rcpf(a);
    const float e = fmaf(-a, r, 1.0f);
    return __builtin_amdgcn_div_fixupf(fmaf(e, r, r), a, 1.0f);
}

// the correction core of LLVM's sqrt lowering without its small-input scaling and class fix-up
__device__ __forceinline__ float sqrt_core(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float dn = __uint_as_float(__float_as_uint(s) - 1u);
    const float up = __uint_as_float(__float_as_uint(s) + 1u);
    const float t = fmaf(-dn, s, x) <= 0.0f ? dn : s;
    return fmaf(-up, s, x) > 0.0f ? up : t;
}

// rsq seed, one Newton step (Goldschmidt form)
__device__ __forceinline__ float sqrt_rsq(float x) {
    const float y = __builtin_amdgcn_rsqf(x);
    const float s = x * y;
    const float h = 0.5f * y;
    const float e = fmaf(-s, s, x);
    return fmaf(e, h, s);
}

__device__ __forceinline__ float cand(int c, float x) {
    switch (c) {
        case 0: return sqrt_core(x);                 // vs sqrtf
        case 1: return sqrt_rsq(x);                  // vs sqrtf
        case 2: return recip4(sqrt_core(x));         // vs 1 / sqrtf
        case 3: return recip4(sqrt_rsq(x));          // vs 1 / sqrtf
        default: {                                   // refined rsq directly vs 1 / sqrtf
            const float y = __builtin_amdgcn_rsqf(x);
            const float e = fmaf(-x * y, y, 1.0f);
            return fmaf(0.5f * e, y, y);
        }
    }
}

__device__ __forceinline__ int klass(float x) {
    if (x != x) return 3;
    if (__builtin_isinf(x) && x > 0.0f) return 2;
    return (x >= 0x1p-96f && x <= 0x1p126f) ? 1 : 0;
}

__global__ void check(uint64_t base, unsigned long long* __restrict__ bad, unsigned* __restrict__ first) {
    const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const float x = __uint_as_float((uint32_t)i);
    const float sq = sqrtf(x);
    const float inv = 1.0f / sq;
    const int k = klass(x);
#pragma unroll
    for (int c = 0; c < NCAND; ++c) {
        const float v = cand(c, x);
        const float ref = (c == 0 || c == 1) ? sq : inv;
        const bool same = (ref != ref) ? (v != v) : (__float_as_uint(v) == __float_as_uint(ref));
        if (!same) {
            atomicAdd(&bad[c * 4 + k], 1ull);
            if (k == 1) atomicMin(&first[c], (uint32_t)i);
        }
    }
}

int main() {
    unsigned long long* bad;
    unsigned* first;
    if (hipMalloc(&bad, sizeof(unsigned long long) * NCAND * 4) != hipSuccess) return 1;
    if (hipMalloc(&first, sizeof(unsigned) * NCAND) != hipSuccess) return 1;
    hipMemset(bad, 0, sizeof(unsigned long long) * NCAND * 4);
    hipMemset(first, 0xff, sizeof(unsigned) * NCAND);
    const uint64_t chunk = 1ull << 28;
    for (uint64_t b = 0; b < (1ull << 32); b += chunk)
        hipLaunchKernelGGL(check, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, b, bad, first);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    unsigned long long h[NCAND * 4];
    unsigned f[NCAND];
    hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost);
    hipMemcpy(f, first, sizeof(f), hipMemcpyDeviceToHost);
    const char* names[NCAND] = {"sqrt_core", "sqrt_rsq", "recip(sqrt_core)", "recip(sqrt_rsq)", "rsq+nr"};
    printf("{\"inputs\": 4294967296, \"classes\": [\"outside [2^-96, 2^126]\", \"[2^-96, 2^126]\", \"+inf\", \"nan\"], "
           "\"references\": [\"sqrtf\", \"sqrtf\", \"1/sqrtf\", \"1/sqrtf\", \"1/sqrtf\"], \"mismatches\": {");
    for (int c = 0; c < NCAND; ++c)
        printf("%s\"%s\": [%llu, %llu, %llu, %llu, \"first in range 0x%08x\"]", c ? ", " : "", names[c], h[4 * c],
               h[4 * c + 1], h[4 * c + 2], h[4 * c + 3], f[c]);
    printf("}}\n");
    return 0;
}
