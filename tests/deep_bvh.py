"""A scene whose BVH is deeper than the reference's 20-slot traversal stack (stack.cl:4, 23-24).

``caterpillar_scene(n)``: n parallel triangles facing the camera (normal -y) at increasing
distance, in a BVH shaped as a caterpillar: internal node 2i has the leaf of triangle i as its
left child and internal node 2i+2 as its right child; the last internal node's right child is
the leaf of triangle n-1, the NEAREST triangle.  The reference's pre-order DFS (MathLib.cl:
234-288) pushes left then right, so every level leaves one leaf on the stack: from level 19 on
the pushes are dropped and the nearest triangle is never tested.  Boxes are exact (leaf = the
triangle's bounds, internal = the union below), as BVH.py exports them.
"""
import numpy as np


def caterpillar_scene(n: int = 40) -> dict:
    vp, face, boxes = [], [], []
    for k in range(n):
        y = 1.0 + 0.05 * (n - 1 - k)   # triangle n-1 is the nearest to a camera at y = -3.5
        tri = [(-1.5, y, -1.5), (1.5, y, -1.5), (0.0, y, 1.5)]
        vp += tri
        face += [0, 0, 0, 0, 0, 0, 0, 3 * k, 3 * k + 1, 3 * k + 2]
        t = np.array(tri, np.float32)
        boxes.append(np.concatenate([t.min(0), t.max(0)]))
    boxes = np.array(boxes, np.float32)
    nodes = np.zeros((2 * n - 1, 9), np.float32)
    for i in range(n - 1):
        u = boxes[i:]
        nodes[2 * i] = [2 * i + 1, 2 * i + 2, *u[:, :3].min(0), *u[:, 3:].max(0), -1]
        nodes[2 * i + 1] = [-1, -1, *boxes[i], i]
    nodes[2 * n - 2] = [-1, -1, *boxes[n - 1], n - 1]
    return {"V_p": np.array(vp, np.float32).reshape(-1), "V_n": np.array([0, -1, 0], np.float32),
            "V_uv": np.array([0, 0], np.float32), "faceData": np.array(face, np.int32),
            "materialData": np.array([1, 0.8, 0.6, 0.4, 0, 0], np.float32), "bvh": nodes.reshape(-1)}
