// Host BVH builder reproducing the reference's BVH.py export bit for bit.
//
// Reference algorithm (BVH.py):
//   * Node box = exact float32 min/max of the three vertex positions of every
//     triangle in the node (Node.computeBoundingBox, BVH.py:43-70; epsilon 0).
//   * Split (Node.split, BVH.py:73-117): centroid (a+b+c)/3 in float64
//     (computeTriCenter, BVH.py:30-40); per-axis mean and variance over the
//     node's triangles, accumulated sequentially in list order in float64
//     (np.mean / np.var over axis 0); split axis = first argmax of the variance;
//     pivot = mean on that axis; centroid < pivot goes left, else right, order
//     preserved.  Left child then right child are appended to the node list
//     (BVH.addNode, BVH.py:169-172).
//   * Recursion (BVH.build, BVH.py:147-160) descends into the left child fully
//     before the right one, so node numbering = split order of a left-first DFS.
//   * Leaves hold exactly one triangle.  Export (recursiveRead, BVH.py:174-191):
//     per node float32 [left, right, min.xyz, max.xyz, tri | -1], children -1 on
//     leaves.
//
// A split that leaves one side empty makes the reference corrupt its child
// indices and recurse without end (all centroids equal on the split axis); the
// builder reports that case as an error instead of producing a tree.
#include <cstdint>
#include <cstring>
#include <cmath>
#include <vector>
#include <algorithm>
#include <new>

namespace {

struct BuildNode {
    int32_t left = -1, right = -1;
    float bmin[3], bmax[3];
    int32_t tri = -1;
    int64_t begin = 0, end = 0;
};

}  // namespace

extern "C" {

// Returns 0 on success; 1 bad arguments; 2 index out of range; 3 degenerate
// split (reference would not terminate); 4 out of host memory.  out must hold 9*(2T-1) floats
// (T = nface/10); *out_nodes receives the node count actually written.
static int bvh_build(const int32_t* face, int64_t nface, const float* vp, int64_t nvp, float* out,
                     int64_t* out_nodes);

// No C++ exception leaves the C ABI: 4 = out of host memory.
int rt_bvh_build(const int32_t* face, int64_t nface, const float* vp, int64_t nvp,
                 float* out, int64_t* out_nodes) {
    try {
        return bvh_build(face, nface, vp, nvp, out, out_nodes);
    } catch (const std::bad_alloc&) {
        return 4;
    }
}

static int bvh_build(const int32_t* face, int64_t nface, const float* vp, int64_t nvp, float* out,
                     int64_t* out_nodes) {
    if (!face || !vp || !out || !out_nodes || nface < 0 || nface % 10 != 0 || nvp % 3 != 0)
        return 1;
    const int64_t T = nface / 10;
    *out_nodes = 0;
    if (T == 0) return 0;
    const int64_t NV = nvp / 3;
    for (int64_t t = 0; t < T; ++t)
        for (int j = 7; j < 10; ++j) {
            const int32_t id = face[10 * t + j];
            if (id < 0 || id >= NV) return 2;
        }

    // Centroids in float64, ((a+b)+c)/3 per axis like numpy on (3,1) arrays.
    std::vector<double> cen(3 * T);
    for (int64_t t = 0; t < T; ++t) {
        const float* a = vp + 3 * (int64_t)face[10 * t + 7];
        const float* b = vp + 3 * (int64_t)face[10 * t + 8];
        const float* c = vp + 3 * (int64_t)face[10 * t + 9];
        for (int x = 0; x < 3; ++x)
            cen[3 * t + x] = (((double)a[x] + (double)b[x]) + (double)c[x]) / 3.0;
    }

    std::vector<int64_t> idx(T), tmp(T);
    for (int64_t t = 0; t < T; ++t) idx[t] = t;

    std::vector<BuildNode> nodes;
    nodes.reserve(2 * T);

    auto make_node = [&](int64_t b, int64_t e) {
        BuildNode n;
        n.begin = b; n.end = e;
        for (int x = 0; x < 3; ++x) { n.bmin[x] = INFINITY; n.bmax[x] = -INFINITY; }
        for (int64_t i = b; i < e; ++i) {
            const int64_t t = idx[i];
            for (int j = 7; j < 10; ++j) {
                const float* p = vp + 3 * (int64_t)face[10 * t + j];
                for (int x = 0; x < 3; ++x) {
                    n.bmin[x] = std::min(n.bmin[x], p[x]);
                    n.bmax[x] = std::max(n.bmax[x], p[x]);
                }
            }
        }
        return n;
    };

    nodes.push_back(make_node(0, T));
    // Explicit stack of node ids reproducing build()'s left-first recursion.
    std::vector<int32_t> stack;
    stack.push_back(0);
    while (!stack.empty()) {
        const int32_t id = stack.back();
        stack.pop_back();
        const int64_t b = nodes[id].begin, e = nodes[id].end;
        const int64_t n = e - b;
        if (n <= 1) {
            nodes[id].tri = (int32_t)idx[b];
            continue;
        }
        double mean[3] = {0, 0, 0}, var[3] = {0, 0, 0};
        for (int64_t i = b; i < e; ++i)
            for (int x = 0; x < 3; ++x) mean[x] += cen[3 * idx[i] + x];
        for (int x = 0; x < 3; ++x) mean[x] = mean[x] / (double)n;
        for (int64_t i = b; i < e; ++i)
            for (int x = 0; x < 3; ++x) {
                const double d = cen[3 * idx[i] + x] - mean[x];
                var[x] += d * d;
            }
        for (int x = 0; x < 3; ++x) var[x] = var[x] / (double)n;
        int axis = 0;
        for (int x = 1; x < 3; ++x)
            if (var[x] > var[axis]) axis = x;  // np.argmax: first maximum
        const double pivot = mean[axis];
        int64_t nl = 0, nr = 0;
        for (int64_t i = b; i < e; ++i)
            if (cen[3 * idx[i] + axis] < pivot) tmp[b + nl++] = idx[i];
        for (int64_t i = b; i < e; ++i)
            if (!(cen[3 * idx[i] + axis] < pivot)) tmp[b + nl + nr++] = idx[i];
        if (nl == 0 || nr == 0) return 3;
        std::memcpy(&idx[b], &tmp[b], sizeof(int64_t) * n);
        const int32_t l = (int32_t)nodes.size();
        nodes.push_back(make_node(b, b + nl));
        nodes.push_back(make_node(b + nl, e));
        nodes[id].left = l;
        nodes[id].right = l + 1;
        // recurse left first: push right, then left
        stack.push_back(l + 1);
        stack.push_back(l);
    }

    for (size_t i = 0; i < nodes.size(); ++i) {
        float* r = out + 9 * i;
        r[0] = (float)nodes[i].left;
        r[1] = (float)nodes[i].right;
        for (int x = 0; x < 3; ++x) { r[2 + x] = nodes[i].bmin[x]; r[5 + x] = nodes[i].bmax[x]; }
        r[8] = (float)nodes[i].tri;
    }
    *out_nodes = (int64_t)nodes.size();
    return 0;
}

}  // extern "C"
