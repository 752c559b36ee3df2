// Surface-area-heuristic BVH2 over the reference's leaf boxes (FAST layout "sah").
//
// The FAST traversal decides whether a triangle is tested from the box of its
// own leaf only: every ancestor box is a union of leaf boxes, and the slab
// test is monotone in the box bounds, so an ancestor never rejects a ray its
// descendant leaf accepts.  The hit record is the (distance, reference DFS
// rank) minimum over the accepted triangles, so it does not depend on which
// tree groups the leaves -- any tree over the same leaf boxes returns the same
// hit.  This builder therefore keeps the reference's leaf boxes bit for bit
// (one triangle per leaf, as BVH.py:59-67 makes them) and only regroups them
// to minimise the expected number of node visits.
//
// Build: top-down; ranges of up to kSweepMax leaves use an exact sweep over
// the centroids sorted along each axis, larger ranges 32 bins per axis.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <vector>

#include "bvh_sah.h"

namespace rt {
namespace {

#ifndef RT_SAH_SWEEP_MAX
#define RT_SAH_SWEEP_MAX 64
#endif
#ifndef RT_SAH_BINS
#define RT_SAH_BINS 32
#endif
constexpr int kSweepMax = RT_SAH_SWEEP_MAX;
constexpr int kBins = RT_SAH_BINS;

struct Box {
    float lo[3], hi[3];
    void reset() {
        for (int a = 0; a < 3; ++a) { lo[a] = 3.4e38f; hi[a] = -3.4e38f; }
    }
    void grow(const Box& b) {
        for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], b.lo[a]); hi[a] = std::max(hi[a], b.hi[a]); }
    }
    double area() const {
        const double x = (double)hi[0] - lo[0], y = (double)hi[1] - lo[1], z = (double)hi[2] - lo[2];
        if (x < 0 || y < 0 || z < 0) return 0.0;
        return x * y + y * z + z * x;
    }
};

struct Builder {
    const std::vector<Box>& box;
    std::vector<double> cen;          // 3 per leaf
    std::vector<int32_t> idx;
    SahTree& out;
    std::vector<double> suffix;       // scratch for the sweep

    Builder(const std::vector<Box>& b, SahTree& o) : box(b), out(o) {
        const size_t n = b.size();
        cen.resize(3 * n);
        for (size_t i = 0; i < n; ++i)
            for (int a = 0; a < 3; ++a) cen[3 * i + a] = 0.5 * ((double)b[i].lo[a] + (double)b[i].hi[a]);
        idx.resize(n);
        std::iota(idx.begin(), idx.end(), 0);
    }

    int32_t new_node() {
        out.L.push_back(-1);
        out.R.push_back(-1);
        out.leaf.push_back(-1);
        out.box.insert(out.box.end(), 6, 0.0f);
        return (int32_t)out.L.size() - 1;
    }

    void set_box(int32_t node, int b, int e) {
        Box bb;
        bb.reset();
        for (int i = b; i < e; ++i) bb.grow(box[idx[i]]);
        float* o = &out.box[6 * (size_t)node];
        for (int a = 0; a < 3; ++a) { o[a] = bb.lo[a]; o[3 + a] = bb.hi[a]; }
    }

    // Returns the split position m in (b, e) after partitioning idx[b, e).
    int split(int b, int e) {
        const int n = e - b;
        double best = 1e300;
        int best_axis = -1, best_bin = -1;
        double cmin[3], cmax[3];
        for (int a = 0; a < 3; ++a) { cmin[a] = 1e300; cmax[a] = -1e300; }
        for (int i = b; i < e; ++i)
            for (int a = 0; a < 3; ++a) {
                cmin[a] = std::min(cmin[a], cen[3 * idx[i] + a]);
                cmax[a] = std::max(cmax[a], cen[3 * idx[i] + a]);
            }
        if (n <= kSweepMax) {
            std::vector<int32_t> tmp(idx.begin() + b, idx.begin() + e), keep;
            suffix.assign(n + 1, 0.0);
            for (int a = 0; a < 3; ++a) {
                if (!(cmax[a] > cmin[a])) continue;
                std::stable_sort(tmp.begin(), tmp.end(),
                                 [&](int32_t x, int32_t y) { return cen[3 * x + a] < cen[3 * y + a]; });
                Box acc;
                acc.reset();
                for (int i = n - 1; i >= 1; --i) {
                    acc.grow(box[tmp[i]]);
                    suffix[i] = acc.area() * (n - i);
                }
                acc.reset();
                for (int i = 1; i < n; ++i) {
                    acc.grow(box[tmp[i - 1]]);
                    const double c = acc.area() * i + suffix[i];
                    if (c < best) {
                        best = c;
                        best_axis = a;
                        best_bin = i;
                        keep = tmp;
                    }
                }
            }
            if (best_axis < 0) return b + n / 2;  // all centroids coincide: split the range in half
            std::copy(keep.begin(), keep.end(), idx.begin() + b);
            return b + best_bin;
        }
        for (int a = 0; a < 3; ++a) {
            if (!(cmax[a] > cmin[a])) continue;
            const double scale = kBins / (cmax[a] - cmin[a]);
            Box bb[kBins];
            int cnt[kBins] = {0};
            for (auto& x : bb) x.reset();
            for (int i = b; i < e; ++i) {
                int k = (int)((cen[3 * idx[i] + a] - cmin[a]) * scale);
                k = std::min(std::max(k, 0), kBins - 1);
                cnt[k]++;
                bb[k].grow(box[idx[i]]);
            }
            double right[kBins];
            Box acc;
            acc.reset();
            int nr = 0;
            for (int k = kBins - 1; k >= 1; --k) {
                acc.grow(bb[k]);
                nr += cnt[k];
                right[k] = nr ? acc.area() * nr : 0.0;
            }
            acc.reset();
            int nl = 0;
            for (int k = 1; k < kBins; ++k) {
                acc.grow(bb[k - 1]);
                nl += cnt[k - 1];
                if (nl == 0 || nl == n) continue;
                const double c = acc.area() * nl + right[k];
                if (c < best) { best = c; best_axis = a; best_bin = k; }
            }
        }
        if (best_axis < 0) return b + n / 2;
        const double scale = kBins / (cmax[best_axis] - cmin[best_axis]);
        auto mid = std::stable_partition(idx.begin() + b, idx.begin() + e, [&](int32_t x) {
            int k = (int)((cen[3 * x + best_axis] - cmin[best_axis]) * scale);
            k = std::min(std::max(k, 0), kBins - 1);
            return k < best_bin;
        });
        return (int)(mid - idx.begin());
    }

    void build() {
        const int n = (int)idx.size();
        if (n == 0) return;
        struct Item { int b, e; int32_t node; };
        std::vector<Item> work;
        work.push_back({0, n, new_node()});
        while (!work.empty()) {
            const Item it = work.back();
            work.pop_back();
            set_box(it.node, it.b, it.e);
            if (it.e - it.b == 1) {
                out.leaf[it.node] = idx[it.b];
                continue;
            }
            int m = split(it.b, it.e);
            if (m <= it.b || m >= it.e) m = it.b + (it.e - it.b) / 2;
            const int32_t l = new_node(), r = new_node();
            out.L[it.node] = l;
            out.R[it.node] = r;
            work.push_back({m, it.e, r});
            work.push_back({it.b, m, l});
        }
    }
};

}  // namespace

void sah_build(const float* leaf_boxes, const int32_t* leaf_ids, int64_t n, SahTree& out) {
    std::vector<Box> boxes((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        const float* b = leaf_boxes + 6 * i;
        for (int a = 0; a < 3; ++a) { boxes[i].lo[a] = b[a]; boxes[i].hi[a] = b[3 + a]; }
    }
    out.L.clear();
    out.R.clear();
    out.leaf.clear();
    out.box.clear();
    out.L.reserve(2 * n);
    out.R.reserve(2 * n);
    out.leaf.reserve(2 * n);
    out.box.reserve(12 * n);
    Builder bld(boxes, out);
    bld.build();
    for (auto& t : out.leaf)
        if (t >= 0) t = leaf_ids[t];
}

}  // namespace rt
