// Traversal BVH for the GPU (gpu_bvh.cpp): binned-SAH binary tree in the kernels' node layout.
#pragma once
#include <cstdint>
#include <vector>

namespace nh {

struct GpuLeaf {
    int start, count;  // range in GpuBvh::order
};

struct GpuBvh {
    std::vector<float> nodes;     // 16 floats per inner node (nh_traverse.h layout), DFS order, root = 0
    std::vector<GpuLeaf> leaves;
    std::vector<uint32_t> order;  // leaf-order slot -> input primitive index
    int root_kind = 0;            // 0 empty, 1 inner root, 2 leaf root (leaves[0])
    int depth = 0;                // levels (root = 1)
    float root_box[6] = {0, 0, 0, 0, 0, 0};
};

// boxes: 6 floats (min xyz, max xyz) per primitive; centroids: 3 floats per primitive
int build_gpu_bvh(const float *boxes, const float *centroids, uint32_t n, GpuBvh &out);

}  // namespace nh
