// Exhaustive check of short reciprocal sequences against the IEEE division 1.0f / a (the
// Moller-Trumbore 1/a of MathLib.cl:117-160, rt_device.h mt_core) over all 2^32 bit patterns of a,
// on the GPU (the hardware v_rcp_f32 seed has no CPU model).
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math -o tools/rcp_exhaustive tools/rcp_exhaustive.hip
//   tools/rcp_exhaustive        -> one JSON line: mismatches per candidate and input class
//
// Classes: 0 = |a| < 1e-7 (mt_core's parallel case: 1/a is not used), 1 = other finite, 2 = +-inf,
// 3 = NaN.  A candidate may replace the division iff classes 1-3 have no mismatch (NaN: any NaN).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int NCAND = 4;

__device__ __forceinline__ float cand(int c, float a) {
    const float r = __builtin_amdgcn_rcpf(a);
    const float e = fmaf(-a, r, 1.0f);
    const float r1 = fmaf(e, r, r);
    if (c == 0) return r1;
    if (c == 1) return __builtin_amdgcn_div_fixupf(r1, a, 1.0f);
    const float e2 = fmaf(-a, r1, 1.0f);
    const float r2 = fmaf(e2, r1, r1);
    if (c == 2) return r2;
    return __builtin_amdgcn_div_fixupf(r2, a, 1.0f);
}

__device__ __forceinline__ int klass(float a) {
    if (a != a) return 3;
    if (__builtin_isinf(a)) return 2;
    return (a > -0.0000001f && a < 0.0000001f) ? 0 : 1;
}

__global__ void check(uint64_t base, unsigned long long* __restrict__ bad, unsigned* __restrict__ first) {
    const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const float a = __uint_as_float((uint32_t)i);
    const float ref = 1.0f / a;
    const int k = klass(a);
#pragma unroll
    for (int c = 0; c < NCAND; ++c) {
        const float v = cand(c, a);
        const bool same = (k == 3) ? (v != v) : (__float_as_uint(v) == __float_as_uint(ref));
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
    const char* names[NCAND] = {"rcp+nr", "rcp+nr+fixup", "rcp+nr+nr", "rcp+nr+nr+fixup"};
    printf("{\"inputs\": 4294967296, \"classes\": [\"tiny(unused)\", \"finite\", \"inf\", \"nan\"], \"mismatches\": {");
    for (int c = 0; c < NCAND; ++c)
        printf("%s\"%s\": [%llu, %llu, %llu, %llu, \"first finite 0x%08x\"]", c ? ", " : "", names[c], h[4 * c],
               h[4 * c + 1], h[4 * c + 2], h[4 * c + 3], f[c]);
    printf("}}\n");
    return 0;
}
