// rtw_bvh.hip -- host-side BVH builder + flattener (the "Zig host builds a
// flattened BVH" half of the boundary).
//
// RTW_BVH_REFERENCE restates BVHTree.constructTree (src/bvh.zig:43-71):
//   * one axis draw per constructTree call, randomIntRange(0,2) (biased,
//     returns 0..3; 3 falls into the z branch), drawn before the span switch;
//   * span 1 -> leaf; span 2 -> two leaves ordered by boxComparator;
//   * else std.sort.heap of the slice by box min on the axis, median split.
// The tree is emitted directly in pre-order with skip links (rtw_layout.h),
// so the kernel's stackless walk replays the reference traversal order.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/rtw_gpu.h"
#include "rtw_internal.h"
#include "rtw_layout.h"
#include "rtw_rng.h"

namespace {

struct Box {
    float mn[3], mx[3];
};

struct Obj {
    Box box;
    uint32_t sphere;
};

// Aabb.fromPoints (src/aabb.zig:18-26)
Box box_from_points(const float a[3], const float b[3]) {
    Box r;
    for (int i = 0; i < 3; i++) {
        r.mn[i] = a[i] < b[i] ? a[i] : b[i];
        r.mx[i] = a[i] > b[i] ? a[i] : b[i];
    }
    return r;
}

// Aabb.fromBoxes + interval.fromIntervals (src/aabb.zig:28-34, src/interval.zig:42-44)
Box box_union(const Box& a, const Box& b) {
    Box r;
    for (int i = 0; i < 3; i++) {
        r.mn[i] = a.mn[i] < b.mn[i] ? a.mn[i] : b.mn[i];
        r.mx[i] = a.mx[i] > b.mx[i] ? a.mx[i] : b.mx[i];
    }
    return r;
}

// Sphere.init / initMoving bounding boxes (src/objects.zig:80-92)
Box sphere_box(const rtw_sphere& s) {
    const float r = s.radius;
    float lo[3], hi[3];
    for (int i = 0; i < 3; i++) { lo[i] = s.center1[i] - r; hi[i] = s.center1[i] + r; }
    Box b1 = box_from_points(lo, hi);
    if (!s.is_moving) return b1;
    for (int i = 0; i < 3; i++) { lo[i] = s.center2[i] - r; hi[i] = s.center2[i] + r; }
    return box_union(b1, box_from_points(lo, hi));
}

class RefBuilder {
public:
    RefBuilder(const rtw_scene_desc& d, std::vector<rtw_node>& out, std::vector<float>& cvec)
        : desc_(d), nodes_(out), cvec_(cvec), rng_(rtw_rng_stream(d.bvh_seed, 2, 0, 0)) {
        objs_.resize(d.n_spheres);
        for (uint32_t i = 0; i < d.n_spheres; i++) {
            objs_[i].box = sphere_box(d.spheres[i]);
            objs_[i].sphere = i;
        }
        cvec_.assign(4 * (size_t)d.n_spheres, 0.0f);
        for (uint32_t i = 0; i < d.n_spheres; i++) {
            const rtw_sphere& s = d.spheres[i];
            if (s.is_moving)
                for (int k = 0; k < 3; k++) cvec_[4 * i + k] = s.center2[k] - s.center1[k];
        }
    }

    void build() {
        nodes_.clear();
        nodes_.reserve(2 * objs_.size());
        depth_ = 0;
        emit(0, objs_.size(), 1);
    }

    uint32_t depth() const { return depth_; }
    uint32_t axis_draws() const { return draws_; }

private:
    // rtweekend.randomIntRange(0, 2) (src/rtweekend.zig:23-27)
    uint32_t draw_axis() {
        draws_++;
        const float mn = 0.0f, mx = 3.0f;
        return (uint32_t)std::round(rtw_rng_range(rng_, mn, mx));
    }

    // boxComparator (src/bvh.zig:95-103)
    static bool less(uint32_t axis, const Obj& a, const Obj& b) {
        const int ax = axis == 0 ? 0 : (axis == 1 ? 1 : 2);
        return a.box.mn[ax] < b.box.mn[ax];
    }

    // Zig std.sort.heap (0.12): heapContext/siftDown restated
    void sift_down(size_t a, size_t target, size_t b, uint32_t axis) {
        size_t cur = target;
        for (;;) {
            size_t child = (cur - a) * 2 + a + 1;
            if (!(child < b)) break;
            size_t next = child + 1;
            if (next < b && less(axis, objs_[child], objs_[next])) child = next;
            if (less(axis, objs_[child], objs_[cur])) break;
            std::swap(objs_[cur], objs_[child]);
            cur = child;
        }
    }
    void heap_sort(size_t a, size_t b, uint32_t axis) {
        size_t i = a + (b - a) / 2;
        while (i > a) { i -= 1; sift_down(a, i, b, axis); }
        i = b;
        while (i > a) {
            i -= 1;
            std::swap(objs_[a], objs_[i]);
            sift_down(a, a, i, axis);
        }
    }

    Box emit_leaf(const Obj& o) {
        const rtw_sphere& s = desc_.spheres[o.sphere];
        rtw_node n;
        uint32_t skip = (uint32_t)nodes_.size() + 1;
        n.a[0] = s.center1[0]; n.a[1] = s.center1[1]; n.a[2] = s.center1[2];
        uint32_t w = skip | RTW_LEAF_BIT;
        std::memcpy(&n.a[3], &w, 4);
        n.b[0] = s.radius;
        std::memcpy(&n.b[1], &s.material, 4);
        std::memcpy(&n.b[2], &o.sphere, 4);
        uint32_t mv = s.is_moving ? 1u : 0u;
        std::memcpy(&n.b[3], &mv, 4);
        nodes_.push_back(n);
        return o.box;
    }

    Box emit(size_t start, size_t end, uint32_t level) {
        depth_ = std::max(depth_, level);
        const uint32_t axis = draw_axis();
        const size_t span = end - start;
        if (span == 1) return emit_leaf(objs_[start]);
        const size_t me = nodes_.size();
        nodes_.push_back(rtw_node{});
        Box lb, rb;
        if (span == 2) {
            depth_ = std::max(depth_, level + 1);
            if (less(axis, objs_[start], objs_[start + 1])) {
                lb = emit_leaf(objs_[start]);
                rb = emit_leaf(objs_[start + 1]);
            } else {
                lb = emit_leaf(objs_[start + 1]);
                rb = emit_leaf(objs_[start]);
            }
        } else {
            heap_sort(start, end, axis);
            const size_t mid = start + span / 2;
            lb = emit(start, mid, level + 1);
            rb = emit(mid, end, level + 1);
        }
        Box bb = box_union(lb, rb);
        rtw_node& n = nodes_[me];
        uint32_t skip = (uint32_t)nodes_.size();
        for (int i = 0; i < 3; i++) { n.a[i] = bb.mn[i]; n.b[i] = bb.mx[i]; }
        std::memcpy(&n.a[3], &skip, 4);
        n.b[3] = 0.0f;
        return bb;
    }

    const rtw_scene_desc& desc_;
    std::vector<rtw_node>& nodes_;
    std::vector<float>& cvec_;
    std::vector<Obj> objs_;
    rtw_rng rng_;
    uint32_t depth_ = 0;
    uint32_t draws_ = 0;
};

// Binned-SAH BVH2 with single-sphere leaves, emitted in the same pre-order
// skip-link format (so the traversal kernel is unchanged).  Deterministic (no
// RNG).  The reference builds a *random* tree every run (axis from
// std.crypto.random), so topology is not observable; only closest-hit
// semantics are, and they are topology-independent.
// Child order: the child whose box centre comes first along `order_dir`
// (a typical ray direction supplied by the caller, default -y) is emitted
// first, so front-most geometry shrinks `closest` early in the fixed walk.
class SahBuilder {
public:
    SahBuilder(const rtw_scene_desc& d, std::vector<rtw_node>& out, std::vector<float>& cvec)
        : desc_(d), nodes_(out), cvec_(cvec) {
        const uint32_t n = d.n_spheres;
        objs_.resize(n);
        cent_.resize(n);
        for (uint32_t i = 0; i < n; i++) {
            objs_[i].box = sphere_box(d.spheres[i]);
            objs_[i].sphere = i;
            for (int k = 0; k < 3; k++) cent_[i][k] = 0.5f * (objs_[i].box.mn[k] + objs_[i].box.mx[k]);
        }
        idx_.resize(n);
        for (uint32_t i = 0; i < n; i++) idx_[i] = i;
        cvec_.assign(4 * (size_t)n, 0.0f);
        for (uint32_t i = 0; i < n; i++) {
            const rtw_sphere& s = d.spheres[i];
            if (s.is_moving)
                for (int k = 0; k < 3; k++) cvec_[4 * i + k] = s.center2[k] - s.center1[k];
        }
        for (int k = 0; k < 3; k++) dir_[k] = d.order_dir[k];
        if (dir_[0] == 0 && dir_[1] == 0 && dir_[2] == 0) dir_[1] = -1;
    }
    void build() {
        nodes_.clear();
        nodes_.reserve(2 * objs_.size());
        depth_ = 0;
        emit(0, idx_.size(), 1);
    }
    uint32_t depth() const { return depth_; }

private:
    static float area(const Box& b) {
        const float dx = b.mx[0] - b.mn[0], dy = b.mx[1] - b.mn[1], dz = b.mx[2] - b.mn[2];
        return 2.0f * (dx * dy + dy * dz + dz * dx);
    }
    Box bounds(size_t a, size_t b) const {
        Box r = objs_[idx_[a]].box;
        for (size_t i = a + 1; i < b; i++) r = box_union(r, objs_[idx_[i]].box);
        return r;
    }
    Box emit_leaf(uint32_t oi) {
        const Obj& o = objs_[oi];
        const rtw_sphere& s = desc_.spheres[o.sphere];
        rtw_node n;
        uint32_t skip = (uint32_t)nodes_.size() + 1;
        n.a[0] = s.center1[0]; n.a[1] = s.center1[1]; n.a[2] = s.center1[2];
        uint32_t w = skip | RTW_LEAF_BIT;
        std::memcpy(&n.a[3], &w, 4);
        n.b[0] = s.radius;
        std::memcpy(&n.b[1], &s.material, 4);
        std::memcpy(&n.b[2], &o.sphere, 4);
        uint32_t mv = s.is_moving ? 1u : 0u;
        std::memcpy(&n.b[3], &mv, 4);
        nodes_.push_back(n);
        return o.box;
    }
    // returns split position (index) after partitioning idx_[a, b)
    size_t split(size_t a, size_t b) {
        const size_t n = b - a;
        float cmn[3] = {1e30f, 1e30f, 1e30f}, cmx[3] = {-1e30f, -1e30f, -1e30f};
        for (size_t i = a; i < b; i++)
            for (int k = 0; k < 3; k++) {
                cmn[k] = std::min(cmn[k], cent_[idx_[i]][k]);
                cmx[k] = std::max(cmx[k], cent_[idx_[i]][k]);
            }
        constexpr int NB = 32;
        float best = 1e38f;
        int best_axis = -1, best_bin = 0;
        for (int ax = 0; ax < 3; ax++) {
            const float ext = cmx[ax] - cmn[ax];
            if (!(ext > 0)) continue;
            Box bb[NB];
            int cnt[NB] = {0};
            bool init[NB] = {false};
            for (size_t i = a; i < b; i++) {
                const uint32_t o = idx_[i];
                int bin = (int)((cent_[o][ax] - cmn[ax]) / ext * NB);
                bin = bin < 0 ? 0 : (bin >= NB ? NB - 1 : bin);
                bb[bin] = init[bin] ? box_union(bb[bin], objs_[o].box) : objs_[o].box;
                init[bin] = true;
                cnt[bin]++;
            }
            float rarea[NB];
            int rcnt[NB];
            Box acc{};
            bool ai = false;
            int c = 0;
            for (int k = NB - 1; k > 0; k--) {
                if (init[k]) { acc = ai ? box_union(acc, bb[k]) : bb[k]; ai = true; }
                c += cnt[k];
                rarea[k] = ai ? area(acc) : 0.0f;
                rcnt[k] = c;
            }
            Box lacc{};
            bool li = false;
            int lc = 0;
            for (int k = 0; k < NB - 1; k++) {
                if (init[k]) { lacc = li ? box_union(lacc, bb[k]) : bb[k]; li = true; }
                lc += cnt[k];
                if (lc == 0 || rcnt[k + 1] == 0) continue;
                const float cost = area(lacc) * (float)lc + rarea[k + 1] * (float)rcnt[k + 1];
                if (cost < best) { best = cost; best_axis = ax; best_bin = k; }
            }
        }
        size_t mid;
        if (best_axis < 0) {
            mid = a + n / 2;  // all centroids coincide: median
        } else {
            const float ext = cmx[best_axis] - cmn[best_axis];
            auto it = std::partition(idx_.begin() + a, idx_.begin() + b, [&](uint32_t o) {
                int bin = (int)((cent_[o][best_axis] - cmn[best_axis]) / ext * NB);
                bin = bin < 0 ? 0 : (bin >= NB ? NB - 1 : bin);
                return bin <= best_bin;
            });
            mid = (size_t)(it - idx_.begin());
            if (mid == a || mid == b) mid = a + n / 2;
        }
        return mid;
    }
    Box emit(size_t a, size_t b, uint32_t level) {
        depth_ = std::max(depth_, level);
        if (b - a == 1) return emit_leaf(idx_[a]);
        const size_t mid = split(a, b);
        // front-to-back child order along dir_
        const Box lb0 = bounds(a, mid), rb0 = bounds(mid, b);
        float pl = 0, pr = 0;
        for (int k = 0; k < 3; k++) {
            pl += dir_[k] * (lb0.mn[k] + lb0.mx[k]);
            pr += dir_[k] * (rb0.mn[k] + rb0.mx[k]);
        }
        const size_t me = nodes_.size();
        nodes_.push_back(rtw_node{});
        Box l, r;
        if (pr < pl) {  // right child is nearer along dir_: emit it first
            l = emit(mid, b, level + 1);
            r = emit(a, mid, level + 1);
        } else {
            l = emit(a, mid, level + 1);
            r = emit(mid, b, level + 1);
        }
        Box bb = box_union(l, r);
        rtw_node& n = nodes_[me];
        uint32_t skip = (uint32_t)nodes_.size();
        for (int i = 0; i < 3; i++) { n.a[i] = bb.mn[i]; n.b[i] = bb.mx[i]; }
        std::memcpy(&n.a[3], &skip, 4);
        n.b[3] = 0.0f;
        return bb;
    }

    const rtw_scene_desc& desc_;
    std::vector<rtw_node>& nodes_;
    std::vector<float>& cvec_;
    std::vector<Obj> objs_;
    std::vector<std::array<float, 3>> cent_;
    std::vector<uint32_t> idx_;
    float dir_[3];
    uint32_t depth_ = 0;
};

}  // namespace

int rtw_build_bvh(const rtw_scene_desc& desc, std::vector<rtw_node>& nodes, std::vector<float>& cvec,
                  uint32_t* depth, uint32_t* axis_draws, float* box_pad, float* extent) {
    if (box_pad) *box_pad = 0;
    if (extent) *extent = 0;
    if (desc.bvh_mode == RTW_BVH_SAH) {
        SahBuilder b(desc, nodes, cvec);
        b.build();
        if (depth) *depth = b.depth();
        if (axis_draws) *axis_draws = 0;
        // Pad the inner boxes for the FMA slab test: its t error for a plane P and
        // origin o is < 4 ulp of (|P| + |o|) in space, so a pad of E * 2^-19
        // (E = max |coordinate| of the scene) keeps the test conservative for
        // every origin with |o| <= 7E (checked per launch, else the exact test runs).
        // A superset of boxes is visited; sphere tests decide the hit.
        float e = 0;
        for (const rtw_node& n : nodes) {
            uint32_t w;
            std::memcpy(&w, &n.a[3], 4);
            if (w & RTW_LEAF_BIT) continue;
            for (int k = 0; k < 3; k++) e = std::max(e, std::max(std::fabs(n.a[k]), std::fabs(n.b[k])));
        }
        const float pad = e * 1.9073486e-06f;  // 2^-19
        for (rtw_node& n : nodes) {
            uint32_t w;
            std::memcpy(&w, &n.a[3], 4);
            if (w & RTW_LEAF_BIT) continue;
            for (int k = 0; k < 3; k++) {
                n.a[k] -= pad;
                n.b[k] += pad;
            }
        }
        if (box_pad) *box_pad = pad;
        if (extent) *extent = e;
        return RTW_OK;
    }
    if (desc.bvh_mode != RTW_BVH_REFERENCE) return RTW_E_INVALID;
    RefBuilder b(desc, nodes, cvec);
    b.build();
    if (depth) *depth = b.depth();
    if (axis_draws) *axis_draws = b.axis_draws();
    return RTW_OK;
}
