// SAH regrouping of the reference's leaf boxes (bvh_sah.cpp).  Host only.
#pragma once
#include <cstdint>
#include <vector>

namespace rt {

// Binary tree, node 0 = root; per node: children L/R (-1 for a leaf), the
// triangle of a leaf (-1 for an inner node) and its box lo.xyz, hi.xyz.
struct SahTree {
    std::vector<int32_t> L, R, leaf;
    std::vector<float> box;
};

// leaf_boxes: 6 floats (lo.xyz, hi.xyz) per leaf; leaf_ids: the triangle of each leaf.
void sah_build(const float* leaf_boxes, const int32_t* leaf_ids, int64_t n, SahTree& out);

}  // namespace rt
