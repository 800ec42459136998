// Traversal BVH for the GPU (NH_TRAVERSAL_SAH): a binned-SAH binary tree over the scene's
// primitives, built for the gfx950 traversal kernels rather than for parity with BVH::build.
//
// The reference itself renders its GPU path from a different acceleration structure than its CPU
// BVH (the OptiX backend builds an OptiX GAS, include/nori/optix/OptixState.as.cpp:47-248). What
// the image depends on is the closest-hit contract, not the tree: smallest t, and among equal t
// the primitive the reference's left-first traversal meets last, i.e. the largest position k in
// the reference BVH's m_indices order. Every primitive record therefore carries that k, and the
// kernels break ties on it whichever tree they traverse.
//
// Build: 32 bins on each of the three axes of the centroid bounds, SAH with equal traversal and
// intersection cost, leaves of at most kMaxLeaf primitives; subtrees above kParallelCut
// primitives are built on their own threads.
#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <future>
#include <mutex>
#include <thread>
#include <vector>

#include "gpu_bvh.h"

namespace nh {

namespace {

constexpr int kBins = 32;
constexpr int kMaxLeaf = 4;
constexpr uint32_t kParallelCut = 1u << 15;

struct Box {
    float mn[3], mx[3];
    void reset() {
        for (int i = 0; i < 3; ++i) { mn[i] = FLT_MAX; mx[i] = -FLT_MAX; }
    }
    void grow(const Box &b) {
        for (int i = 0; i < 3; ++i) { mn[i] = std::min(mn[i], b.mn[i]); mx[i] = std::max(mx[i], b.mx[i]); }
    }
    void grow(const float *p) {
        for (int i = 0; i < 3; ++i) { mn[i] = std::min(mn[i], p[i]); mx[i] = std::max(mx[i], p[i]); }
    }
    double area() const {
        const double dx = (double)mx[0] - mn[0], dy = (double)mx[1] - mn[1], dz = (double)mx[2] - mn[2];
        if (dx < 0 || dy < 0 || dz < 0) return 0.0;
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
};

struct BuildNode {
    Box box;
    uint32_t begin = 0, count = 0;  // leaf: primitive range in `order`
    int left = -1, right = -1;      // children (indices into the node pool), -1 for a leaf
};

struct Builder {
    const float *boxes, *cent;  // 6 and 3 floats per primitive
    std::vector<uint32_t> &order;
    std::vector<BuildNode> nodes;
    std::mutex mu;
    std::atomic<int> depth{0};

    Builder(const float *b, const float *c, std::vector<uint32_t> &o) : boxes(b), cent(c), order(o) {}

    int alloc() {
        std::lock_guard<std::mutex> g(mu);
        nodes.emplace_back();
        return (int)nodes.size() - 1;
    }
    void set(int id, const BuildNode &n) {
        std::lock_guard<std::mutex> g(mu);
        nodes[id] = n;
    }

    Box prim_box(uint32_t p) const {
        Box b;
        for (int i = 0; i < 3; ++i) { b.mn[i] = boxes[6 * (size_t)p + i]; b.mx[i] = boxes[6 * (size_t)p + 3 + i]; }
        return b;
    }

    // builds the subtree of order[begin, begin + count) into node `id`
    void build(int id, uint32_t begin, uint32_t count, int level) {
        BuildNode n;
        n.box.reset();
        Box cb;
        cb.reset();
        for (uint32_t i = begin; i < begin + count; ++i) {
            n.box.grow(prim_box(order[i]));
            cb.grow(&cent[3 * (size_t)order[i]]);
        }
        int d = depth.load();
        while (level > d && !depth.compare_exchange_weak(d, level)) {}
        n.begin = begin;
        n.count = count;
        if (count <= 1) return set(id, n);
        // best split over 3 axes x kBins bins
        int best_axis = -1, best_bin = -1;
        double best_cost = (double)count;  // leaf cost (intersection cost 1 per primitive)
        const double inv_area = 1.0 / std::max(n.box.area(), 1e-30);
        for (int axis = 0; axis < 3; ++axis) {
            const float lo = cb.mn[axis], ext = cb.mx[axis] - cb.mn[axis];
            if (!(ext > 0.f)) continue;
            const float scale = kBins / ext;
            Box bb[kBins];
            uint32_t bc[kBins] = {0};
            for (auto &b : bb) b.reset();
            for (uint32_t i = begin; i < begin + count; ++i) {
                const uint32_t p = order[i];
                int bin = (int)((cent[3 * (size_t)p + axis] - lo) * scale);
                bin = std::min(std::max(bin, 0), kBins - 1);
                bc[bin]++;
                bb[bin].grow(prim_box(p));
            }
            double right_area[kBins];
            uint32_t right_cnt[kBins];
            Box acc;
            acc.reset();
            uint32_t cnt = 0;
            for (int b = kBins - 1; b > 0; --b) {
                acc.grow(bb[b]);
                cnt += bc[b];
                right_area[b] = acc.area();
                right_cnt[b] = cnt;
            }
            acc.reset();
            cnt = 0;
            for (int b = 0; b < kBins - 1; ++b) {
                acc.grow(bb[b]);
                cnt += bc[b];
                if (cnt == 0 || right_cnt[b + 1] == 0) continue;
                const double cost = 1.0 + inv_area * (acc.area() * cnt + right_area[b + 1] * right_cnt[b + 1]);
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = axis;
                    best_bin = b;
                }
            }
        }
        uint32_t mid;
        if (best_axis < 0) {
            if (count <= (uint32_t)kMaxLeaf) return set(id, n);
            // no useful split (coincident centroids or the leaf is cheaper): halve by position
            mid = begin + count / 2;
        } else {
            if (count <= (uint32_t)kMaxLeaf && best_cost >= (double)count) return set(id, n);
            const float lo = cb.mn[best_axis], scale = kBins / (cb.mx[best_axis] - cb.mn[best_axis]);
            auto it = std::partition(order.begin() + begin, order.begin() + begin + count, [&](uint32_t p) {
                int bin = (int)((cent[3 * (size_t)p + best_axis] - lo) * scale);
                return std::min(std::max(bin, 0), kBins - 1) <= best_bin;
            });
            mid = (uint32_t)(it - order.begin());
            if (mid == begin || mid == begin + count) mid = begin + count / 2;
        }
        n.left = alloc();
        n.right = alloc();
        set(id, n);
        const uint32_t nl = mid - begin, nr = count - nl;
        if (count > kParallelCut) {
            auto f = std::async(std::launch::async, [&, l = n.left] { build(l, begin, nl, level + 1); });
            build(n.right, mid, nr, level + 1);
            f.get();
        } else {
            build(n.left, begin, nl, level + 1);
            build(n.right, mid, nr, level + 1);
        }
    }
};

void put_box(float *dst, const Box &b) {
    for (int i = 0; i < 3; ++i) { dst[i] = b.mn[i]; dst[3 + i] = b.mx[i]; }
}

}  // namespace

int build_gpu_bvh(const float *boxes, const float *centroids, uint32_t n, GpuBvh &out) {
    out = GpuBvh{};
    if (n == 0) return 0;
    out.order.resize(n);
    for (uint32_t i = 0; i < n; ++i) out.order[i] = i;
    Builder b(boxes, centroids, out.order);
    b.nodes.reserve(2 * (size_t)n);
    const int root = b.alloc();
    b.build(root, 0, n, 0);
    out.depth = b.depth.load() + 1;
    const auto &N = b.nodes;
    put_box(out.root_box, N[root].box);
    if (N[root].left < 0) {
        out.root_kind = 2;
        out.leaves.push_back({(int)N[root].begin, (int)N[root].count});
        return 0;
    }
    out.root_kind = 1;
    // inner nodes in left-first DFS order; child boxes stored in the parent
    std::vector<int> gid(N.size(), -1), stack{root};
    std::vector<int> inner;
    while (!stack.empty()) {
        const int i = stack.back();
        stack.pop_back();
        if (N[i].left < 0) continue;
        gid[i] = (int)inner.size();
        inner.push_back(i);
        stack.push_back(N[i].right);
        stack.push_back(N[i].left);
    }
    out.nodes.assign(16 * inner.size(), 0.f);
    auto ref = [&](int ch) -> int {
        if (N[ch].left < 0) {
            out.leaves.push_back({(int)N[ch].begin, (int)N[ch].count});
            return ~(int)(out.leaves.size() - 1);
        }
        return gid[ch];
    };
    for (size_t g = 0; g < inner.size(); ++g) {
        const BuildNode &p = N[inner[g]];
        float *dst = &out.nodes[16 * g];
        float lb[6], rb[6];
        put_box(lb, N[p.left].box);
        put_box(rb, N[p.right].box);
        // n0 = (L.min.xyz, L.max.x)  n1 = (L.max.yz, R.min.xy)  n2 = (R.min.z, R.max.xyz)  n3 = refs
        dst[0] = lb[0]; dst[1] = lb[1]; dst[2] = lb[2]; dst[3] = lb[3];
        dst[4] = lb[4]; dst[5] = lb[5]; dst[6] = rb[0]; dst[7] = rb[1];
        dst[8] = rb[2]; dst[9] = rb[3]; dst[10] = rb[4]; dst[11] = rb[5];
        const int lr = ref(p.left), rr = ref(p.right);
        std::memcpy(&dst[12], &lr, 4);
        std::memcpy(&dst[13], &rr, 4);
    }
    return 0;
}

}  // namespace nh
