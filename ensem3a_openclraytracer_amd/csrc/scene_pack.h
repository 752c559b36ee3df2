// Host-side scene preparation (no HIP): validates the reference's flat scene arrays and packs
// them into the device layouts of rt_internal.h.  rt_set_scene (rt_api.hip) uploads the result;
// rt_scene_check (include/rt_scene.h) runs it alone, without a GPU.  Not part of the public
// boundary.  Host-only, so it builds with -fsanitize=address,undefined (oracle/Makefile asan).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "rt_layout.h"

namespace rt {

// Host copy of the packed scene (kept to upload on every device).
struct HostScene {
    std::vector<float> nodes;      // 16 floats per internal node
    std::vector<float> wnodes;     // wide layout: 16 floats per 4-wide node (DevScene::wnodes)
    std::vector<float> wleaves;    // wide layout: 16 floats per leaf, in reference DFS rank order
    int32_t nwnodes = 0, wroot_ref = 0, wdepth = 1;
    float wdq_omax = 0.0f;   // the 4-wide layout's dequantisation gap covers ray origins up to this (0: no gap)
    std::vector<float> bvh9;
    std::vector<float> tri_geo;    // 12 floats per triangle
    std::vector<float> tri_fast;   // tri_geo's records in FAST leaf order (DevScene::tri_fast)
    std::vector<float> tri_shade;  // 4 floats per triangle
    std::vector<float> mat;
    std::vector<float> brute;      // 16 floats per triangle, small scenes only (rt_internal.h DevScene::brute)
    std::vector<float> brute_box;  // 8 floats per triangle, padded to whole groups (DevScene::brute_box)
    int32_t nbrute = 0;
    int32_t nbox = 0;              // distinct leaf boxes in brute_box (records with bit-identical boxes share one)
    int32_t nnodes = 0, root_ref = 0, ntri = 0, nmat = 0, nbvh9 = 0, depth = 1;
    float root_box[6] = {0, 0, 0, 0, 0, 0};
    bool fast_ok = false;
    bool colors_finite = true;     // every material colour finite (FrameParams::sun_skip)
    bool has_glass = false;        // some material has type 3 (FrameParams::sun_any)
};


// Validate and pack (KernelLauncher.py:38-72's buffers, FileManager.py:276-282's faceData,
// BVH.py:174-191's export).  Returns RT_OK, or an RT_ERR_* code with `msg` set.  `why` receives the
// reason when the FAST layouts are unavailable (hs.fast_ok false; the REF traversal then serves).
int scene_prepare(HostScene& hs, const float* vp, int64_t nvp, const float* vn, int64_t nvn, const int32_t* face,
                  int64_t nface, const float* mat, int64_t nmat, const float* bvh9, int64_t nbvh, int layout,
                  int brute_max, std::string& msg, std::string& why);

// pack_fast + the limits of the FAST kernels; sets hs.fast_ok (an option change repacks with it).
void pack_checked(HostScene& hs, const float* bvh9, int64_t nb, int64_t ntri, int layout, int brute_max,
                  std::string& why);

}  // namespace rt
