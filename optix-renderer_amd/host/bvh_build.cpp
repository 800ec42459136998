// Host SAH BVH builder producing the reference's node array bit for bit.
//
// Algorithm = BVH::build / BVHBuildTask (src/utils/bvh.cpp:54-380): 16-bin SAH on the
// largest axis above 32 primitives (:100-233), full-sort SAH below it or when binning
// finds no split (:236-305), leaves when no split lowers the cost, node placement
// left = node+1 / right = node + 2*left_count, then the compaction pass (:356-379).
// The reference partitions with TBB atomics (order of equal-bin primitives depends on
// thread timing); this builder partitions stably, which is the serial-schedule result.
// Differences from the reference's implementation that do not change the output:
// centroids and primitive boxes are computed once up front (the reference recomputes
// them from the vertices inside every comparator, 46% of its build time), binning is
// a parallel exact reduction, and independent subtrees are built on worker threads.
#include <algorithm>
#include <atomic>
#include <climits>
#include <cmath>
#include <cstring>
#include <future>
#include <memory>
#include <thread>
#include <vector>

#include "nh_host.h"
#include "nori_hip.h"

namespace nh {
namespace {

struct Box {
    float mn[3], mx[3];
    Box() { reset(); }
    void reset() {
        for (int i = 0; i < 3; ++i) { mn[i] = INFINITY; mx[i] = -INFINITY; }
    }
    void expand(const Box &b) {
        // Eigen cwiseMin/cwiseMax: std::min(a,b) = (b < a) ? b : a
        for (int i = 0; i < 3; ++i) {
            mn[i] = (b.mn[i] < mn[i]) ? b.mn[i] : mn[i];
            mx[i] = (mx[i] < b.mx[i]) ? b.mx[i] : mx[i];
        }
    }
    static Box merge(const Box &a, const Box &b) {
        Box r = a;
        r.expand(b);
        return r;
    }
    float area() const {  // BoundingBox::getSurfaceArea (bbox.h:87-100)
        float d[3] = {mx[0] - mn[0], mx[1] - mn[1], mx[2] - mn[2]};
        float result = 0.0f;
        for (int i = 0; i < 3; ++i) {
            float term = 1.0f;
            for (int j = 0; j < 3; ++j) {
                if (i == j) continue;
                term *= d[j];
            }
            result += term;
        }
        return 2.0f * result;
    }
    int largest_axis() const {  // bbox.h:308-317
        float e0 = mx[0] - mn[0], e1 = mx[1] - mn[1], e2 = mx[2] - mn[2];
        if (e0 >= e1 && e0 >= e2) return 0;
        if (e1 >= e0 && e1 >= e2) return 1;
        return 2;
    }
};

// x86 cvttss2si semantics for (int)float: NaN / out of range -> INT_MIN
inline int f2i(float x) {
    if (!(x > -2147483904.0f && x < 2147483648.0f)) return INT_MIN;
    return (int)x;
}

struct Node {
    uint32_t word0, word1;
    Box box;
};

constexpr int BIN_COUNT = 16;
constexpr uint32_t SERIAL_THRESHOLD = 32;
constexpr uint32_t GRAIN = 1000;

struct Builder {
    std::vector<float> cx[3];  // centroids per axis
    std::vector<Box> pbox;
    std::vector<Node> nodes;
    std::vector<uint32_t> indices;
    int n_threads = 1;
    std::atomic<int> live_tasks{0};

    void set_leaf(Node &n, uint32_t start, uint32_t size) {
        n.word0 = 1u | (size << 1);
        n.word1 = start;
    }
    void set_inner(Node &n, uint32_t axis, uint32_t right) {
        n.word0 = 0u | (axis << 1);
        n.word1 = right;
    }

    // BVHBuildTask::execute_serially (bvh.cpp:236-305)
    void serial(uint32_t node_idx, uint32_t *start, uint32_t *end, uint32_t *temp) {
        Node &node = nodes[node_idx];
        uint32_t size = (uint32_t)(end - start);
        float best_cost = (float)1 * size;
        int64_t best_index = -1, best_axis = -1;
        float *left_areas = (float *)temp;
        for (int axis = 0; axis < 3; ++axis) {
            const float *c = cx[axis].data();
            std::sort(start, end, [c](uint32_t f1, uint32_t f2) { return c[f1] < c[f2]; });
            Box bbox;
            for (uint32_t i = 0; i < size; ++i) {
                bbox.expand(pbox[start[i]]);
                left_areas[i] = (float)bbox.area();
            }
            if (axis == 0) node.box = bbox;
            bbox.reset();
            float tri_factor = 1 / node.box.area();
            for (uint32_t i = size - 1; i >= 1; --i) {
                bbox.expand(pbox[start[i]]);
                float left_area = left_areas[i - 1];
                float right_area = bbox.area();
                uint32_t prims_left = i, prims_right = size - i;
                float sah_cost = 2.0f * 1 + tri_factor * (prims_left * left_area + prims_right * right_area);
                if (sah_cost < best_cost) {
                    best_cost = sah_cost;
                    best_index = i;
                    best_axis = axis;
                }
            }
        }
        if (best_index == -1) {
            set_leaf(node, (uint32_t)(start - indices.data()), size);
            return;
        }
        const float *c = cx[best_axis].data();
        std::sort(start, end, [c](uint32_t f1, uint32_t f2) { return c[f1] < c[f2]; });
        uint32_t left_count = (uint32_t)best_index;
        uint32_t left_idx = node_idx + 1, right_idx = node_idx + 2 * left_count;
        set_inner(node, (uint32_t)best_axis, right_idx);
        serial(left_idx, start, start + left_count, temp);
        serial(right_idx, start + left_count, end, temp + left_count);
    }

    struct Bins {
        uint32_t counts[BIN_COUNT];
        Box bbox[BIN_COUNT];
        Bins() { std::memset(counts, 0, sizeof(counts)); }
    };

    void bin_range(const uint32_t *start, uint32_t b, uint32_t e, int axis, float mn, float inv, Bins &r) {
        const float *c = cx[axis].data();
        for (uint32_t i = b; i < e; ++i) {
            uint32_t f = start[i];
            int index = std::min(std::max(f2i((c[f] - mn) * inv), 0), BIN_COUNT - 1);
            r.counts[index]++;
            r.bbox[index].expand(pbox[f]);
        }
    }

    // BVHBuildTask::execute (bvh.cpp:100-233)
    void task(uint32_t node_idx, uint32_t *start, uint32_t *end, uint32_t *temp) {
        for (;;) {
            uint32_t size = (uint32_t)(end - start);
            Node &node = nodes[node_idx];
            if (size < SERIAL_THRESHOLD) {
                serial(node_idx, start, end, temp);
                return;
            }
            int axis = node.box.largest_axis();
            float mn = node.box.mn[axis], mx = node.box.mx[axis];
            float inv = BIN_COUNT / (mx - mn);
            Bins bins;
            // exact reduction: counts add, boxes merge by min/max -> order independent
            const uint32_t par_chunks = (size >= 200000 && n_threads > 1) ? (uint32_t)n_threads : 1;
            if (par_chunks > 1) {
                std::vector<Bins> partial(par_chunks);
                std::vector<std::thread> th;
                uint32_t step = (size + par_chunks - 1) / par_chunks;
                for (uint32_t k = 0; k < par_chunks; ++k) {
                    uint32_t b = k * step, e = std::min(size, b + step);
                    th.emplace_back([&, k, b, e] { bin_range(start, b, e, axis, mn, inv, partial[k]); });
                }
                for (auto &t : th) t.join();
                for (auto &p : partial)
                    for (int i = 0; i < BIN_COUNT; ++i) {
                        bins.counts[i] += p.counts[i];
                        bins.bbox[i] = Box::merge(bins.bbox[i], p.bbox[i]);
                    }
            } else {
                bin_range(start, 0, size, axis, mn, inv, bins);
            }
            Box bbox_left[BIN_COUNT];
            bbox_left[0] = bins.bbox[0];
            for (int i = 1; i < BIN_COUNT; ++i) {
                bins.counts[i] += bins.counts[i - 1];
                bbox_left[i] = Box::merge(bbox_left[i - 1], bins.bbox[i]);
            }
            Box bbox_right = bins.bbox[BIN_COUNT - 1], best_bbox_right;
            int64_t best_index = -1;
            float best_cost = (float)1 * size;
            float tri_factor = (float)1 / node.box.area();
            for (int i = BIN_COUNT - 2; i >= 0; --i) {
                uint32_t prims_left = bins.counts[i], prims_right = size - bins.counts[i];
                float sah_cost = 2.0f * 1 + tri_factor * (prims_left * bbox_left[i].area() + prims_right * bbox_right.area());
                if (sah_cost < best_cost) {
                    best_cost = sah_cost;
                    best_index = i;
                    best_bbox_right = bbox_right;
                }
                bbox_right = Box::merge(bbox_right, bins.bbox[i]);
            }
            if (best_index == -1) {
                serial(node_idx, start, end, temp);
                return;
            }
            uint32_t left_count = bins.counts[best_index];
            uint32_t left_idx = node_idx + 1, right_idx = node_idx + 2 * left_count;
            nodes[left_idx].box = bbox_left[best_index];
            nodes[right_idx].box = best_bbox_right;
            set_inner(node, (uint32_t)axis, right_idx);
            // stable partition == the TBB partition run serially in grain order
            const float *c = cx[axis].data();
            uint32_t il = 0, ir = left_count;
            for (uint32_t i = 0; i < size; ++i) {
                uint32_t f = start[i];
                int index = f2i((c[f] - mn) * inv);
                if (index <= best_index) temp[il++] = f;
                else temp[ir++] = f;
            }
            std::memcpy(start, temp, size * sizeof(uint32_t));
            (void)GRAIN;
            // right subtree: on a worker thread when large, else inline after the left one
            uint32_t *rs = start + left_count, *re = end, *rt = temp + left_count;
            std::future<void> fut;
            bool spawned = false;
            if (n_threads > 1 && (re - rs) > 20000 && live_tasks.load() < n_threads - 1) {
                live_tasks++;
                fut = std::async(std::launch::async, [this, right_idx, rs, re, rt] {
                    task(right_idx, rs, re, rt);
                    live_tasks--;
                });
                spawned = true;
            }
            // continue with the left subtree in this thread (recycle_as_child_of)
            if (!spawned) {
                task(left_idx, start, start + left_count, temp);
                node_idx = right_idx;
                start = rs;
                end = re;
                temp = rt;
                continue;
            }
            task(left_idx, start, start + left_count, temp);
            fut.get();
            return;
        }
    }

    std::pair<float, uint32_t> statistics(uint32_t idx) const {
        const Node &n = nodes[idx];
        if (n.word0 & 1u) return {(float)1 * (n.word0 >> 1), 1u};
        auto l = statistics(idx + 1), r = statistics(n.word1);
        float sl = nodes[idx + 1].box.area(), sr = nodes[n.word1].box.area(), sc = n.box.area();
        return {2 * 1 + (sl * l.first + sr * r.first) / sc, l.second + r.second + 1u};
    }
};

uint32_t max_depth(const std::vector<nh_bvh_node> &nodes) {
    if (nodes.empty()) return 0;
    uint32_t best = 0;
    std::vector<std::pair<uint32_t, uint32_t>> st{{0u, 0u}};
    while (!st.empty()) {
        auto [i, d] = st.back();
        st.pop_back();
        best = std::max(best, d);
        if (!(nodes[i].word0 & 1u)) {
            st.push_back({i + 1, d + 1});
            st.push_back({nodes[i].word1, d + 1});
        }
    }
    return best;
}

}  // namespace
}  // namespace nh

struct nh_bvh {
    std::vector<nh_bvh_node> nodes;
    std::vector<uint32_t> indices;
    std::vector<uint32_t> shape_offset;
    float bmin[3], bmax[3];
    uint32_t depth = 0;
};

extern "C" {

int nh_bvh_build(const nh_scene_desc *sc, int32_t n_threads, nh_bvh **out) {
    using namespace nh;
    if (!sc || !out) { set_host_error("null argument"); return NH_ERR_INVALID; }
    try {
        auto bvh = std::make_unique<nh_bvh>();
        bvh->shape_offset.push_back(0u);
        Box scene_box;
        for (uint32_t s = 0; s < sc->n_shapes; ++s) {
            const nh_shape &sh = sc->shapes[s];
            uint32_t cnt = sh.type == NH_SHAPE_MESH ? sh.n_faces : 1u;
            bvh->shape_offset.push_back(bvh->shape_offset.back() + cnt);
            Box b;
            for (int i = 0; i < 3; ++i) { b.mn[i] = sh.bbox_min[i]; b.mx[i] = sh.bbox_max[i]; }
            scene_box.expand(b);  // BVH::addShape: m_bbox.expandBy(shape->getBoundingBox())
        }
        const uint32_t size = bvh->shape_offset.back();
        for (int i = 0; i < 3; ++i) { bvh->bmin[i] = scene_box.mn[i]; bvh->bmax[i] = scene_box.mx[i]; }
        if (size == 0) { *out = bvh.release(); return NH_OK; }

        Builder b;
        b.n_threads = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
        for (int a = 0; a < 3; ++a) b.cx[a].resize(size);
        b.pbox.resize(size);
        uint32_t p = 0;
        for (uint32_t s = 0; s < sc->n_shapes; ++s) {
            const nh_shape &sh = sc->shapes[s];
            if (sh.type == NH_SHAPE_SPHERE) {
                Box bb;
                for (int i = 0; i < 3; ++i) { bb.mn[i] = sh.bbox_min[i]; bb.mx[i] = sh.bbox_max[i]; }
                b.pbox[p] = bb;
                for (int a = 0; a < 3; ++a) b.cx[a][p] = sh.center[a];
                ++p;
                continue;
            }
            const float *V = sc->V + 3 * (size_t)sh.v_offset;
            const uint32_t *F = sc->F + 3 * (size_t)sh.f_offset;
            for (uint32_t f = 0; f < sh.n_faces; ++f, ++p) {
                const float *v0 = V + 3 * F[3 * f], *v1 = V + 3 * F[3 * f + 1], *v2 = V + 3 * F[3 * f + 2];
                Box bb;
                for (int i = 0; i < 3; ++i) {
                    bb.mn[i] = bb.mx[i] = v0[i];
                }
                for (const float *v : {v1, v2})
                    for (int i = 0; i < 3; ++i) {
                        bb.mn[i] = (v[i] < bb.mn[i]) ? v[i] : bb.mn[i];
                        bb.mx[i] = (bb.mx[i] < v[i]) ? v[i] : bb.mx[i];
                    }
                b.pbox[p] = bb;
                // Mesh::getCentroid: (1/3) * ((v0 + v1) + v2)
                for (int a = 0; a < 3; ++a) b.cx[a][p] = (1.0f / 3.0f) * ((v0[a] + v1[a]) + v2[a]);
            }
        }
        b.nodes.assign(2 * (size_t)size, Node{0u, 0u, Box()});
        for (auto &n : b.nodes) {  // memset(0) of the reference's node array
            n.word0 = n.word1 = 0;
            for (int i = 0; i < 3; ++i) n.box.mn[i] = n.box.mx[i] = 0.0f;
        }
        b.nodes[0].box = scene_box;
        b.indices.resize(size);
        for (uint32_t i = 0; i < size; ++i) b.indices[i] = i;
        std::vector<uint32_t> temp(size);
        b.task(0u, b.indices.data(), b.indices.data() + size, temp.data());

        auto stats = b.statistics(0);
        // compaction (bvh.cpp:356-379)
        std::vector<Node> compact(stats.second);
        std::vector<uint32_t> skipped_accum(b.nodes.size());
        for (int64_t i = (int64_t)stats.second - 1, j = (int64_t)b.nodes.size(), skipped = 0; i >= 0; --i) {
            while (b.nodes[--j].word0 == 0 && b.nodes[j].word1 == 0) skipped++;
            Node &nn = compact[i];
            nn = b.nodes[j];
            skipped_accum[j] = (uint32_t)skipped;
            if (!(nn.word0 & 1u))
                nn.word1 = (uint32_t)(i + nn.word1 - j - (skipped - skipped_accum[nn.word1]));
        }
        bvh->nodes.resize(compact.size());
        for (size_t i = 0; i < compact.size(); ++i) {
            bvh->nodes[i].word0 = compact[i].word0;
            bvh->nodes[i].word1 = compact[i].word1;
            for (int a = 0; a < 3; ++a) {
                bvh->nodes[i].bbox_min[a] = compact[i].box.mn[a];
                bvh->nodes[i].bbox_max[a] = compact[i].box.mx[a];
            }
        }
        bvh->indices = std::move(b.indices);
        bvh->depth = max_depth(bvh->nodes);
        *out = bvh.release();
        return NH_OK;
    } catch (const std::exception &e) {
        set_host_error(e.what());
        return NH_ERR_INVALID;
    }
}

int nh_bvh_get_desc(const nh_bvh *bvh, nh_bvh_desc *out) {
    if (!bvh || !out) { nh::set_host_error("null argument"); return NH_ERR_INVALID; }
    std::memset(out, 0, sizeof(*out));
    out->n_nodes = (uint32_t)bvh->nodes.size();
    out->nodes = bvh->nodes.data();
    out->n_indices = (uint32_t)bvh->indices.size();
    out->indices = bvh->indices.data();
    out->n_shapes = (uint32_t)bvh->shape_offset.size() - 1;
    out->shape_offset = bvh->shape_offset.data();
    for (int i = 0; i < 3; ++i) { out->bbox_min[i] = bvh->bmin[i]; out->bbox_max[i] = bvh->bmax[i]; }
    out->max_depth = bvh->depth;
    return NH_OK;
}

void nh_bvh_free(nh_bvh *bvh) { delete bvh; }

}  // extern "C"
