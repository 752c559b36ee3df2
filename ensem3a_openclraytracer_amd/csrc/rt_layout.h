// Layout constants shared by the host scene packer (scene_pack.cpp, no HIP) and the kernels
// (rt_internal.h).  Not part of the public boundary.
#pragma once
#include <cstddef>
#include <cstdint>

namespace rt {

// LDS entries of the FAST traversal stack per lane (int2 each); deeper entries spill to HBM.
constexpr int kStackLds = 20;
// ... and on the 4-wide walk, whose kernel runs 7 waves per SIMD (render_resume_kernel, kWideWaves):
// 11 entries (88 B per lane) leave the LDS room for them (C5 at 7 waves: 5,890 ms with 11 entries,
// 5,915 with 10)
constexpr int kStackLdsWide = 11;
#ifndef RT_WIDE_WAVES
#define RT_WIDE_WAVES 7   // variant builds (tools/variants.py) override it for the spill A/B
#endif
constexpr int kWideWaves = RT_WIDE_WAVES;   // waves per SIMD of the 4-wide walk (rt_kernels.hip)
constexpr int kNodeF4 = 4;             // float4 per FAST BVH2 node (DevScene::nodes)
constexpr int kMaxLanesPerCu = 2048;   // resident threads per CU (gfx950)
#ifndef RT_BOX_GROUP
#define RT_BOX_GROUP 4
#endif
constexpr int kBoxGroup = RT_BOX_GROUP;  // leaf boxes per scalar load group of the brute-force loop (DevScene::brute_box)
#ifndef RT_BRUTE_MAX_DEFAULT
#define RT_BRUTE_MAX_DEFAULT 64   // FAST tests every triangle of scenes up to this size (rt_set_option "brute_max")
#endif
constexpr int kMatF = 8;               // floats per device material row (DevScene::mat)
// FAST tree walk over the 4-wide layout when the BVH2 node array exceeds this (option "bvh_width"
// 0 = auto): trees that do not fit the L2, where the walk is bound by the latency of dependent
// misses and half as many node fetches pay; smaller trees are bound by the item step's VALU.
constexpr size_t kWideMinBytes = 16u << 20;

// Per-launch scratch block (the `work` argument of launch_render): pixel hand-out counters of the
// kGroups block groups (blockIdx.x % kGroups: the blocks one XCD runs under round-robin dispatch),
// kCounterStride bytes apart, then the per-launch constants at kConstOffset.
constexpr int kGroups = 8;
constexpr int kCounterStride = 64;
constexpr int kTeamOffset = 512;    // pilot launches: pixels left after pass 1 (uint32), then the pass-2 team size (int32)
constexpr int kConstOffset = 1024;
constexpr int kWorkBytes = 2048;
// Tile pixels are dealt to the groups in chunks of kChunk consecutive pixels (chunk c to group
// c % kGroups), so each 128-byte line of the frame is written by the blocks of one XCD only.
constexpr int kChunkShift = 10;

}  // namespace rt
