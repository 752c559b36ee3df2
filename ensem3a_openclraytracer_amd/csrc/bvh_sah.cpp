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
#include <atomic>
#include <cstdint>
#include <cstring>
#include <limits>
#include <numeric>
#include <system_error>
#include <thread>
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
constexpr int kParMin = 4096;   // subtrees of at least this many leaves go to the thread pool

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

// Bin of a centroid: the truncation (int)((c - cmin) * scale) clamped to [0, kBins), computed without
// converting a non-finite or out-of-range double to int (caller-supplied boxes may hold NaN or inf)
inline int bin_of(double c, double cmin, double scale) {
    const double f = (c - cmin) * scale;
    return f >= (double)(kBins - 1) ? kBins - 1 : f > 0.0 ? (int)f : 0;
}

// Centroid sort key: NaN ordered after everything, so the comparator stays a strict weak order
inline double sort_key(double c) { return c == c ? c : std::numeric_limits<double>::infinity(); }

// The leaves' boxes, centroids and the permutation every builder partitions in place (disjoint ranges).
struct Shared {
    const std::vector<Box>& box;
    std::vector<double> cen;          // 3 per leaf
    std::vector<int32_t> idx;

    explicit Shared(const std::vector<Box>& b) : box(b) {
        const size_t n = b.size();
        cen.resize(3 * n);
        for (size_t i = 0; i < n; ++i)
            for (int a = 0; a < 3; ++a) cen[3 * i + a] = 0.5 * ((double)b[i].lo[a] + (double)b[i].hi[a]);
        idx.resize(n);
        std::iota(idx.begin(), idx.end(), 0);
    }
};

// A split depends only on the leaves of its own range (their order in idx included), so subtrees over
// disjoint ranges are built independently -- in parallel below a grain size -- and the tree is the one
// the serial top-down build makes (node numbering aside, which nothing downstream reads: emit_bvh
// renumbers breadth-first from the root).
struct Builder {
    const std::vector<Box>& box;
    const std::vector<double>& cen;
    std::vector<int32_t>& idx;
    SahTree& out;
    // scratch reused across calls: the build allocates nothing per node (allocator contention made the
    // threaded build no faster than the serial one)
    std::vector<double> suffix;       // the sweep's right-side costs
    std::vector<int32_t> tmp, keep, part;

    Builder(Shared& sh, SahTree& o) : box(sh.box), cen(sh.cen), idx(sh.idx), out(o) {}

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
            tmp.assign(idx.begin() + b, idx.begin() + e);
            suffix.assign(n + 1, 0.0);
            for (int a = 0; a < 3; ++a) {
                if (!(cmax[a] > cmin[a])) continue;
                // stable insertion sort by centroid (n <= kSweepMax): the order std::stable_sort gives
                for (int i = 1; i < n; ++i) {
                    const int32_t x = tmp[i];
                    const double kx = sort_key(cen[3 * x + a]);
                    int j = i;
                    for (; j > 0 && kx < sort_key(cen[3 * tmp[j - 1] + a]); --j) tmp[j] = tmp[j - 1];
                    tmp[j] = x;
                }
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
                const int k = bin_of(cen[3 * idx[i] + a], cmin[a], scale);
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
        // stable partition (the order std::stable_partition gives) through the reused scratch
        part.clear();
        int m = b;
        for (int i = b; i < e; ++i) {
            const int32_t x = idx[i];
            if (bin_of(cen[3 * x + best_axis], cmin[best_axis], scale) < best_bin) idx[m++] = x;
            else part.push_back(x);
        }
        std::copy(part.begin(), part.end(), idx.begin() + m);
        return m;
    }

    struct Item { int b, e; int32_t node; };

    // Top-down from the range [b, e) at node `root`; ranges of at most `grain` leaves (other than the
    // root's own) are not built but returned in `deferred`.
    void build(int b0, int e0, int32_t root, int grain, std::vector<Item>* deferred) {
        std::vector<Item> work;
        work.push_back({b0, e0, root});
        while (!work.empty()) {
            const Item it = work.back();
            work.pop_back();
            if (deferred && it.node != root && it.e - it.b <= grain) {
                deferred->push_back(it);
                continue;
            }
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
    if (n == 0) return;
    Shared sh(boxes);
    Builder top(sh, out);
    const int32_t root = top.new_node();
    const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (hw == 1 || n < 4 * kParMin) {
        top.build(0, (int)n, root, 0, nullptr);
    } else {
        // the top of the tree serially, down to ranges of `grain` leaves; those subtrees on hw threads
        const int grain = std::max<int>(kParMin, (int)(n / (8 * (int64_t)hw)));
        std::vector<Builder::Item> tasks;
        top.build(0, (int)n, root, grain, &tasks);
        std::vector<SahTree> sub(tasks.size());
        std::atomic<size_t> next{0};
        auto worker = [&]() {
            for (size_t k; (k = next.fetch_add(1)) < tasks.size();) {
                Builder bb(sh, sub[k]);
                const int32_t r = bb.new_node();
                bb.build(tasks[k].b, tasks[k].e, r, 0, nullptr);
            }
        };
        std::vector<std::thread> pool;
        for (unsigned t = 1; t < hw; ++t) {
            try {
                pool.emplace_back(worker);
            } catch (const std::system_error&) {   // no more threads: the ones started do the rest
                break;
            }
        }
        worker();
        for (auto& t : pool) t.join();
        // stitch: subtree k's node 0 becomes the deferred node, its other nodes are appended
        for (size_t k = 0; k < tasks.size(); ++k) {
            const SahTree& st = sub[k];
            const int32_t base = (int32_t)out.L.size() - 1;   // local node j >= 1 -> base + j
            auto map = [&](int32_t j) { return j < 0 ? j : j == 0 ? tasks[k].node : base + j; };
            const int32_t dn = tasks[k].node;
            out.L[dn] = map(st.L[0]);
            out.R[dn] = map(st.R[0]);
            out.leaf[dn] = st.leaf[0];
            for (int c = 0; c < 6; ++c) out.box[6 * (size_t)dn + c] = st.box[c];
            for (size_t j = 1; j < st.L.size(); ++j) {
                out.L.push_back(map(st.L[j]));
                out.R.push_back(map(st.R[j]));
                out.leaf.push_back(st.leaf[j]);
                out.box.insert(out.box.end(), st.box.begin() + 6 * j, st.box.begin() + 6 * j + 6);
            }
        }
    }
    for (auto& t : out.leaf)
        if (t >= 0) t = leaf_ids[t];
}

}  // namespace rt
