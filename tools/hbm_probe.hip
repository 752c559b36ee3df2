// Calibration probe of the L2 memory-side read counters on gfx950 (VERDICT r02 "prove or drop the
// 2x FETCH_SIZE correction for 64-B gathers").  Each kernel reads a KNOWN number of bytes with one
// access pattern; rocprofv3 --pmc passes over this binary give what FETCH_SIZE, TCC_EA0_RDREQ*,
// TCC_BUBBLE and TCC_EA0_RDREQ_DRAM_32B report for it (tools/hbm_probe.sh runs the passes,
// tools/hbm_probe_summary.py writes profiles/r03_hbm_probe.json).
//
//   stream16      16 B per lane, coalesced, over a 1 GiB buffer (the guide's calibrated case)
//   gather64_mall one random 64-byte record per lane (four 16-byte loads) from a 150 MB table:
//                 C5's node/leaf fetch shape and table size (fits the 256 MB Infinity Cache)
//   gather64_dram the same from a 4 GiB table (misses the Infinity Cache)
//   gather16_dram one random 16-byte piece of a 64-byte record per lane, 4 GiB table
//   gather128_dram one random 128-byte record per lane (eight 16-byte loads), 4 GiB table
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/hbm_probe.hip -o tools/bin/hbm_probe
// Prints one JSON line per kernel with its known byte count; every kernel runs twice (the second
// dispatch is the one the summary uses: the first warms the TLB).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {   // integer hash (lowbias32)
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// the loaded values feed a store that never happens (keeps the loads; no write traffic)
__device__ __forceinline__ void sink(float4 a, float* out) {
    const float s = a.x + a.y + a.z + a.w;
    if (s == 1234.5678f) out[threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) stream16(const float4* __restrict__ p, uint64_t n, float* out) {
    float4 acc = make_float4(0, 0, 0, 0);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const float4 v = p[i];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    sink(acc, out);
}

// K records of R bytes (R = 64 or 128) gathered at random, or one 16-byte piece of a 64-byte record;
// TAG only gives each probe its own kernel name (0: the 150 MB table, 1: the 4 GiB table)
template <int F4, bool PIECE, int TAG>
__global__ void __launch_bounds__(256) gather(const float4* __restrict__ tab, uint32_t nrec, uint32_t seed, float* out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t h = mix(t ^ seed);
    const uint32_t r = (uint32_t)(((uint64_t)h * nrec) >> 32);
    const float4* rec = tab + (uint64_t)r * (PIECE ? 4 : F4);
    float4 acc = make_float4(0, 0, 0, 0);
    if (PIECE) {
        acc = rec[mix(h) & 3u];
    } else {
#pragma unroll
        for (int k = 0; k < F4; ++k) {
            const float4 v = rec[k];
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
    }
    sink(acc, out);
}

int main() {
    const uint64_t big = 4ull << 30, mall = 150ull << 20, stream = 1ull << 30;
    float4* buf = nullptr;
    float* out = nullptr;
    CHECK(hipMalloc(&buf, big));
    CHECK(hipMalloc(&out, 4096));
    CHECK(hipMemset(buf, 0, big));
    CHECK(hipDeviceSynchronize());
    const uint32_t lanes = 1u << 24;   // gathers per dispatch
    const dim3 blk(256), grd(lanes / 256);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(stream16, dim3(8192), blk, 0, 0, (const float4*)buf, stream / 16, out);
        hipLaunchKernelGGL((gather<4, false, 0>), grd, blk, 0, 0, (const float4*)buf, (uint32_t)(mall / 64), 11u + rep, out);
        hipLaunchKernelGGL((gather<4, false, 1>), grd, blk, 0, 0, (const float4*)buf, (uint32_t)(big / 64), 23u + rep, out);
        hipLaunchKernelGGL((gather<4, true, 1>), grd, blk, 0, 0, (const float4*)buf, (uint32_t)(big / 64), 37u + rep, out);
        hipLaunchKernelGGL((gather<8, false, 1>), grd, blk, 0, 0, (const float4*)buf, (uint32_t)(big / 128), 41u + rep, out);
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
    }
    std::printf("{\"kernel\": \"stream16\", \"bytes\": %llu}\n", (unsigned long long)stream);
    std::printf("{\"kernel\": \"gather64_mall\", \"bytes\": %llu, \"table\": %llu}\n", 64ull * lanes,
                (unsigned long long)mall);
    std::printf("{\"kernel\": \"gather64_dram\", \"bytes\": %llu, \"table\": %llu}\n", 64ull * lanes,
                (unsigned long long)big);
    std::printf("{\"kernel\": \"gather16_dram\", \"bytes\": %llu, \"table\": %llu}\n", 16ull * lanes,
                (unsigned long long)big);
    std::printf("{\"kernel\": \"gather128_dram\", \"bytes\": %llu, \"table\": %llu}\n", 128ull * lanes,
                (unsigned long long)big);
    CHECK(hipFree(buf));
    CHECK(hipFree(out));
    return 0;
}
