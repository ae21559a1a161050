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
//
// The leaves are the world objects (spheres, quads, Translate/RotateY instances
// of a HittableList, ConstantMedium); their boxes are restated from Sphere.init,
// Quad.init, HittableList.add, Translate.init, RotateY.init and
// ConstantMedium.boundingBox (src/objects.zig:80-92, 201-210, 273-276, 299-304,
// 340-388, 462-464), because the reference orders and splits by them.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdlib>
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

// a world object: kind (RTW_OBJ_*) + index into its array, and its box
struct Obj {
    Box box;
    uint32_t kind, index;
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

// Aabb.pad (aabb.zig:36-43), Interval.expand (interval.zig:26-29)
Box box_pad(Box b) {
    const float delta = 0.0001f;
    for (int k = 0; k < 3; k++) {
        if (!(b.mx[k] - b.mn[k] >= delta)) {
            const float padding = delta / 2.0f;
            b.mn[k] = b.mn[k] - padding;
            b.mx[k] = b.mx[k] + padding;
        }
    }
    return b;
}

// Validated object graph + device geometry records + per-object boxes.
class Geometry {
public:
    Geometry(const rtw_scene_desc& d, rtw_geometry& g) : d_(d), g_(g) {}

    int build() {
        const rtw_scene_desc& d = d_;
        if (d.n_quads && !d.quads) return RTW_E_INVALID;
        if (d.n_members && !d.members) return RTW_E_INVALID;
        if (d.n_instances && !d.instances) return RTW_E_INVALID;
        if (d.n_media && !d.media) return RTW_E_INVALID;
        g_.feat = 0;
        // spheres: device records + center_vec
        g_.spheres.assign(d.n_spheres, rtw_dev_sphere{});
        g_.cvec.assign(4 * (size_t)d.n_spheres, 0.0f);
        sbox_.resize(d.n_spheres);
        for (uint32_t i = 0; i < d.n_spheres; i++) {
            const rtw_sphere& s = d.spheres[i];
            rtw_dev_sphere& o = g_.spheres[i];
            for (int k = 0; k < 3; k++) o.c1[k] = s.center1[k];
            o.radius = s.radius;
            o.mat = s.material;
            o.moving = s.is_moving ? 1u : 0u;
            if (s.is_moving)
                for (int k = 0; k < 3; k++) g_.cvec[4 * i + k] = s.center2[k] - s.center1[k];
            sbox_[i] = sphere_box(s);
        }
        // quads: Quad.init (objects.zig:201-210)
        g_.quads.assign(d.n_quads, rtw_dev_quad{});
        qbox_.resize(d.n_quads);
        qtrue_.resize(d.n_quads);
        for (uint32_t i = 0; i < d.n_quads; i++) {
            const rtw_quad& q = d.quads[i];
            if (q.material >= d.n_materials) return RTW_E_INVALID;
            rtw_dev_quad& o = g_.quads[i];
            float n[3], nn[3];
            n[0] = q.u[1] * q.v[2] - q.u[2] * q.v[1];
            n[1] = q.u[2] * q.v[0] - q.u[0] * q.v[2];
            n[2] = q.u[0] * q.v[1] - q.u[1] * q.v[0];
            const float len = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
            for (int k = 0; k < 3; k++) nn[k] = n[k] / len;
            const float nd = n[0] * n[0] + n[1] * n[1] + n[2] * n[2];
            o.d = nn[0] * q.q[0] + nn[1] * q.q[1] + nn[2] * q.q[2];
            float far[3];
            for (int k = 0; k < 3; k++) {
                o.q[k] = q.q[k];
                o.n[k] = nn[k];
                o.u[k] = q.u[k];
                o.v[k] = q.v[k];
                o.w[k] = n[k] / nd;
                far[k] = (q.q[k] + q.u[k]) + q.v[k];
            }
            o.mat = q.material;
            qbox_[i] = box_pad(box_from_points(q.q, far));
            // the reference's box spans one diagonal only (objects.zig:210): a quad whose u, v are not
            // axis-aligned can reach outside it.  qtrue_: the box of all four corners.
            float qu[3], qv[3];
            for (int k = 0; k < 3; k++) { qu[k] = q.q[k] + q.u[k]; qv[k] = q.q[k] + q.v[k]; }
            qtrue_[i] = box_union(box_from_points(q.q, far), box_from_points(qu, qv));
            for (int k = 0; k < 3; k++)
                if (qtrue_[i].mn[k] < qbox_[i].mn[k] || qtrue_[i].mx[k] > qbox_[i].mx[k]) loose_ = true;
        }
        if (d.n_quads) g_.feat |= RTW_F_GEOM;
        // instance members
        g_.members.resize(d.n_members);
        for (uint32_t i = 0; i < d.n_members; i++) {
            const rtw_object& m = d.members[i];
            if (m.kind == RTW_OBJ_SPHERE ? m.index >= d.n_spheres : (m.kind != RTW_OBJ_QUAD || m.index >= d.n_quads))
                return RTW_E_INVALID;
            g_.members[i] = RTW_REF(m.kind, m.index);
        }
        // instances: HittableList box then the transform chain (innermost first)
        g_.insts.assign(d.n_instances, rtw_dev_instance{});
        ibox_.resize(d.n_instances);
        itrue_.resize(d.n_instances);
        for (uint32_t i = 0; i < d.n_instances; i++) {
            const rtw_instance& in = d.instances[i];
            if (in.count == 0 || in.count > 127 || in.first > d.n_members || in.count > d.n_members - in.first ||
                in.n_xf > RTW_MAX_XF)
                return RTW_E_INVALID;
            rtw_dev_instance& o = g_.insts[i];
            o.first = in.first;
            o.count = in.count;
            o.n_xf = in.n_xf;
            for (int k = 0; k < 3; k++) {  // no culling unless rtw_build_bvh pads the box (SAH trees)
                o.box[0][k] = -__builtin_inff();
                o.box[1][k] = __builtin_inff();
            }
            Box b, tb;  // the reference's box; a true bound of the members (for the leaf's own box test)
            if (in.flags & RTW_INST_LIST) {  // HittableList: bounding_box starts as Aabb{} = [0,0]^3
                for (int k = 0; k < 3; k++) b.mn[k] = b.mx[k] = 0.0f;
                for (uint32_t m = 0; m < in.count; m++) b = box_union(b, member_box(d.members[in.first + m]));
            } else {
                b = member_box(d.members[in.first]);
            }
            tb = member_true_box(d.members[in.first]);
            for (uint32_t m = 1; m < in.count; m++) tb = box_union(tb, member_true_box(d.members[in.first + m]));
            for (uint32_t k = 0; k < in.n_xf; k++) {
                const rtw_transform& x = in.xf[k];
                uint32_t kind = x.kind;
                std::memcpy(&o.xf[k][0], &kind, 4);
                if (x.kind == RTW_XF_TRANSLATE) {  // Translate.init: box.add(offset)
                    for (int c = 0; c < 3; c++) {
                        o.xf[k][1 + c] = x.v[c];
                        b.mn[c] = b.mn[c] + x.v[c];
                        b.mx[c] = b.mx[c] + x.v[c];
                        tb.mn[c] = tb.mn[c] + x.v[c];
                        tb.mx[c] = tb.mx[c] + x.v[c];
                    }
                } else if (x.kind == RTW_XF_ROTATE_Y) {  // RotateY.init
                    const float pi = 3.1415926535897932385f;
                    const float radians = x.v[0] * pi / 180.0f;  // degreesToRadians (rtweekend.zig:10-12)
                    const float sn = std::sin(radians), cs = std::cos(radians);
                    o.xf[k][1] = sn;
                    o.xf[k][2] = cs;
                    o.xf[k][3] = 0.0f;
                    b = rotate_y_box(b, sn, cs);
                    tb = rotate_y_box(tb, sn, cs);
                } else {
                    return RTW_E_INVALID;
                }
            }
            ibox_[i] = b;
            itrue_[i] = tb;
        }
        if (d.n_instances) g_.feat |= RTW_F_GEOM;
        // media: ConstantMedium (objects.zig:445-464)
        g_.media.assign(d.n_media, rtw_dev_medium{});
        mbox_.resize(d.n_media);
        for (uint32_t i = 0; i < d.n_media; i++) {
            const rtw_medium& m = d.media[i];
            const rtw_object& bd = m.boundary;
            const bool ok = (bd.kind == RTW_OBJ_SPHERE && bd.index < d.n_spheres) ||
                            (bd.kind == RTW_OBJ_QUAD && bd.index < d.n_quads) ||
                            (bd.kind == RTW_OBJ_INSTANCE && bd.index < d.n_instances);
            if (!ok || m.material >= d.n_materials) return RTW_E_INVALID;
            g_.media[i].boundary = RTW_REF(bd.kind, bd.index);
            g_.media[i].neg_inv_density = -1.0f / m.density;  // objects.zig:451
            g_.media[i].mat = m.material;
            mbox_[i] = object_box(bd);
        }
        if (d.n_media) g_.feat |= RTW_F_MEDIUM | RTW_F_GEOM;
        // world objects
        const uint32_t n = d.objects ? d.n_objects : d.n_spheres;
        if (n == 0) return RTW_E_INVALID;
        objs_.resize(n);
        for (uint32_t i = 0; i < n; i++) {
            const rtw_object ref = d.objects ? d.objects[i] : rtw_object{RTW_OBJ_SPHERE, i};
            const uint32_t cap = ref.kind == RTW_OBJ_SPHERE     ? d.n_spheres
                                 : ref.kind == RTW_OBJ_QUAD     ? d.n_quads
                                 : ref.kind == RTW_OBJ_INSTANCE ? d.n_instances
                                 : ref.kind == RTW_OBJ_MEDIUM   ? d.n_media
                                                                : 0;
            if (ref.index >= cap) return RTW_E_INVALID;
            objs_[i].kind = ref.kind;
            objs_[i].index = ref.index;
            objs_[i].box = object_box(ref);
        }
        return RTW_OK;
    }

    const std::vector<Obj>& objects() const { return objs_; }
    // a bound of every point of instance i's members in world space (up to rounding)
    const Box& instance_true_box(uint32_t i) const { return itrue_[i]; }
    // some quad reaches outside its reference box (objects.zig:210): boxes are then not bounds, and a walk
    // that skips inner nodes (object_tree flattening) could find hits the plain tree's boxes cull
    bool loose_boxes() const { return loose_; }

    // leaf record of a world object (rtw_layout.h)
    rtw_node leaf(const Obj& o, uint32_t skip) const {
        rtw_node n{};
        const uint32_t w = skip | RTW_LEAF_BIT;
        std::memcpy(&n.a[3], &w, 4);
        if (o.kind == RTW_OBJ_SPHERE) {
            const rtw_sphere& s = d_.spheres[o.index];
            n.a[0] = s.center1[0]; n.a[1] = s.center1[1]; n.a[2] = s.center1[2];
            n.b[0] = s.radius;
            std::memcpy(&n.b[1], &s.material, 4);
            std::memcpy(&n.b[2], &o.index, 4);
            const uint32_t mv = s.is_moving ? 1u : 0u;
            std::memcpy(&n.b[3], &mv, 4);
            return n;
        }
        const uint32_t mat = o.kind == RTW_OBJ_QUAD ? d_.quads[o.index].material
                             : o.kind == RTW_OBJ_MEDIUM ? d_.media[o.index].material : 0u;
        const uint32_t kind = o.kind << 8;
        std::memcpy(&n.b[1], &mat, 4);
        std::memcpy(&n.b[2], &o.index, 4);
        std::memcpy(&n.b[3], &kind, 4);
        return n;
    }

private:
    Box member_box(const rtw_object& m) const { return m.kind == RTW_OBJ_SPHERE ? sbox_[m.index] : qbox_[m.index]; }
    Box member_true_box(const rtw_object& m) const { return m.kind == RTW_OBJ_SPHERE ? sbox_[m.index] : qtrue_[m.index]; }
    Box object_box(const rtw_object& r) const {
        switch (r.kind) {
        case RTW_OBJ_SPHERE: return sbox_[r.index];
        case RTW_OBJ_QUAD: return qbox_[r.index];
        case RTW_OBJ_INSTANCE: return ibox_[r.index];
        default: return mbox_[r.index];
        }
    }
    // RotateY.init box (objects.zig:353-386)
    static Box rotate_y_box(const Box& bb, float sn, float cs) {
        const float inf = __builtin_inff();
        float mn[3] = {inf, inf, inf}, mx[3] = {-inf, -inf, -inf};
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 2; j++)
                for (int k = 0; k < 2; k++) {
                    const float i_f = (float)i, j_f = (float)j, k_f = (float)k;
                    const float x = i_f * bb.mx[0] + (1 - i_f) * bb.mn[0];
                    const float y = j_f * bb.mx[1] + (1 - j_f) * bb.mn[1];
                    const float z = k_f * bb.mx[2] + (1 - k_f) * bb.mn[2];
                    const float newx = cs * x + sn * z;
                    const float newz = -sn * x + cs * z;
                    const float t[3] = {newx, y, newz};
                    for (int c = 0; c < 3; c++) {
                        mn[c] = std::fmin(mn[c], t[c]);
                        mx[c] = std::fmax(mx[c], t[c]);
                    }
                }
        return box_from_points(mn, mx);
    }

    const rtw_scene_desc& d_;
    rtw_geometry& g_;
    std::vector<Box> sbox_, qbox_, ibox_, mbox_, qtrue_, itrue_;
    bool loose_ = false;
    std::vector<Obj> objs_;
};

class RefBuilder {
public:
    RefBuilder(const rtw_scene_desc& d, const Geometry& g, std::vector<rtw_node>& out)
        : geo_(g), nodes_(out), objs_(g.objects()), rng_(rtw_rng_stream(d.bvh_seed, 2, 0, 0)) {}

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
        nodes_.push_back(geo_.leaf(o, (uint32_t)nodes_.size() + 1));
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

    const Geometry& geo_;
    std::vector<rtw_node>& nodes_;
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
    SahBuilder(const rtw_scene_desc& d, const Geometry& g, std::vector<rtw_node>& out, uint32_t max_leaf,
               bool hoist = false, float flatten = 0.0f)
        : geo_(g), nodes_(out), objs_(g.objects()), hoist_(hoist), flatten_(flatten) {
        const size_t n = objs_.size();
        cent_.resize(n);
        for (size_t i = 0; i < n; i++)
            for (int k = 0; k < 3; k++) cent_[i][k] = 0.5f * (objs_[i].box.mn[k] + objs_[i].box.mx[k]);
        idx_.resize(n);
        for (size_t i = 0; i < n; i++) idx_[i] = (uint32_t)i;
        for (int k = 0; k < 3; k++) dir_[k] = d.order_dir[k];
        if (dir_[0] == 0 && dir_[1] == 0 && dir_[2] == 0) dir_[1] = -1;
        max_leaf_ = std::max<size_t>(1, max_leaf);
    }
    // orders = 1: one pre-order with children front-to-back along order_dir;
    // orders = 8: one pre-order per ray-direction octant (bit k set = negative
    // component k), children ordered front-to-back along that octant's diagonal,
    // concatenated.  The walk of a ray uses the array of its own octant, so the
    // child nearer along the ray is visited first and shrinks `closest` early.
    //
    // Hoisted spheres (hoist_): a sphere whose box dwarfs everything else (Book-1's and the stress
    // scene's ground, r = 1000) sits at the top of any tree, where rays of different octants test
    // it at different steps of their walks -- every such test a divergent sphere step of its wave.
    // Such spheres are emitted FIRST in every copy, as leaves with skip = i + 1, followed by the
    // tree of the other objects: each walk starts at node 0, so every lane of a wave tests them at
    // the same steps (0 .. h-1), with no box step interleaved, and the stackless format, the walks
    // and the skip links are unchanged (a "forest" of h leaves and one tree).  Same closest hit:
    // each ray still tests every hoisted sphere and walks the rest of the scene.
    void build(uint32_t orders) {
        nodes_.clear();
        tree_.clear();
        tree_.reserve(2 * objs_.size());
        depth_ = 0;
        const size_t h = hoist_ ? select_hoisted() : 0;
        const int root = build_tree(h, idx_.size(), 1);
        nodes_.reserve(orders * (tree_.size() + h));
        for (uint32_t o = 0; o < orders; o++) {
            float dir[3];
            for (int k = 0; k < 3; k++) dir[k] = orders == 1 ? dir_[k] : ((o >> k) & 1 ? -1.0f : 1.0f);
            if (orders == 4) {  // copies by the x and z signs (order_of): diagonals in the xz plane
                dir[0] = (o & 1u) ? -1.0f : 1.0f;
                dir[1] = 0.0f;
                dir[2] = (o & 2u) ? -1.0f : 1.0f;
            }
            base_ = (uint32_t)nodes_.size();
            for (size_t k = 0; k < h; k++)
                nodes_.push_back(geo_.leaf(objs_[idx_[k]], (uint32_t)nodes_.size() + 1 - base_));
            emit_tree(root, dir, -1.0f);
        }
        n_hoisted_ = (uint32_t)h;
    }
    uint32_t depth() const { return depth_; }
    uint32_t hoisted() const { return n_hoisted_; }

private:
    struct TNode {
        Box box;
        int left = -1, right = -1;
        uint32_t first = 0, count = 0;  // leaf: idx_[first, first + count)
    };

    int build_tree(size_t a, size_t b, uint32_t level) {
        depth_ = std::max(depth_, level);
        const int me = (int)tree_.size();
        tree_.push_back(TNode{});
        Box box = objs_[idx_[a]].box;
        for (size_t i = a + 1; i < b; i++) box = box_union(box, objs_[idx_[i]].box);
        tree_[me].box = box;
        tree_[me].first = (uint32_t)a;
        tree_[me].count = (uint32_t)(b - a);
        if (b - a == 1) return me;
        float sc;
        const size_t mid = split(a, b, &sc);
        // SAH termination: a leaf of up to max_leaf_ objects is a run of leaf records
        // the walk tests one after the other with no box (cost n * ci_); a split costs
        // one box test per child plus the area-weighted tests below it
        if (b - a <= max_leaf_ && (float)(b - a) * ci_ <= 2.0f + ci_ * sc / area(box)) return me;
        tree_[me].count = 0;
        const int l = build_tree(a, mid, level + 1);
        const int r = build_tree(mid, b, level + 1);
        tree_[me].left = l;
        tree_[me].right = r;
        return me;
    }

    // pre-order with skip links (relative to the array start base_).  parent_area: the area of the
    // emitted inner node above (< 0 at the root).  Object scenes (flatten_ > 0): an inner node whose box
    // has >= flatten_ of the area of the emitted node above is not emitted -- its children follow in its
    // place, in the same order, and the skip link of the node above still ends past them.  A ray then
    // visits a superset of the plain tree's leaves in the same order, and every box is conservative, so
    // the closest hit (ties included) is the plain tree's.  (Cornell: the walls' thin boxes make every
    // union of two of them the whole room, so four inner nodes under the root tested the room again on
    // every ray.)
    void emit_tree(int t, const float dir[3], float parent_area) {
        const TNode& n = tree_[t];
        if (n.left < 0) {
            for (uint32_t i = 0; i < n.count; i++) {
                const Obj& o = objs_[idx_[n.first + i]];
                nodes_.push_back(geo_.leaf(o, (uint32_t)nodes_.size() + 1 - base_));
            }
            return;
        }
        const Box& lb = tree_[n.left].box;
        const Box& rb = tree_[n.right].box;
        float pl = 0, pr = 0;
        for (int k = 0; k < 3; k++) {
            pl += dir[k] * (lb.mn[k] + lb.mx[k]);
            pr += dir[k] * (rb.mn[k] + rb.mx[k]);
        }
        const float a = area(n.box);
        const bool emit = !(flatten_ > 0 && parent_area >= 0 && a >= flatten_ * parent_area);
        const size_t me = nodes_.size();
        if (emit) nodes_.push_back(rtw_node{});
        const float below = emit ? a : parent_area;
        if (pr < pl) {  // right child is nearer along dir: walk it first
            emit_tree(n.right, dir, below);
            emit_tree(n.left, dir, below);
        } else {
            emit_tree(n.left, dir, below);
            emit_tree(n.right, dir, below);
        }
        if (!emit) return;
        rtw_node& o = nodes_[me];
        const uint32_t skip = (uint32_t)nodes_.size() - base_;
        for (int i = 0; i < 3; i++) { o.a[i] = n.box.mn[i]; o.b[i] = n.box.mx[i]; }
        std::memcpy(&o.a[3], &skip, 4);
        o.b[3] = 0.0f;
    }

    // Moves the hoisted spheres to idx_[0, h): repeatedly the sphere with the largest box, while its box
    // area exceeds 4x that of the union of all remaining objects' boxes (at most 4; a tree must remain).
    size_t select_hoisted() {
        size_t h = 0;
        while (h < 4 && idx_.size() - h > 2) {
            size_t best = idx_.size();
            float best_a = -1.0f;
            for (size_t i = h; i < idx_.size(); i++) {
                const Obj& o = objs_[idx_[i]];
                if (o.kind != RTW_OBJ_SPHERE) continue;
                const float a = area(o.box);
                if (a > best_a) { best_a = a; best = i; }
            }
            if (best == idx_.size()) break;
            bool any = false;
            Box rest{};
            for (size_t i = h; i < idx_.size(); i++) {
                if (i == best) continue;
                rest = any ? box_union(rest, objs_[idx_[i]].box) : objs_[idx_[i]].box;
                any = true;
            }
            if (!(best_a > 4.0f * area(rest))) break;
            std::swap(idx_[h], idx_[best]);
            h++;
        }
        return h;
    }

    static float area(const Box& b) {
        const float dx = b.mx[0] - b.mn[0], dy = b.mx[1] - b.mn[1], dz = b.mx[2] - b.mn[2];
        return 2.0f * (dx * dy + dy * dz + dz * dx);
    }
    // returns split position (index) after partitioning idx_[a, b)
    // binned SAH split of idx_[a, b); *cost = sum over the two sides of area x count
    size_t split(size_t a, size_t b, float* cost) {
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
        *cost = best_axis < 0 ? 1e38f : best;
        return mid;
    }
    const Geometry& geo_;
    std::vector<rtw_node>& nodes_;
    std::vector<Obj> objs_;
    std::vector<TNode> tree_;
    uint32_t base_ = 0;
    std::vector<std::array<float, 3>> cent_;
    std::vector<uint32_t> idx_;
    float dir_[3];
    uint32_t depth_ = 0;
    size_t max_leaf_ = 1;  // objects per leaf run
    float ci_ = 2.0f;      // cost of one leaf test relative to one box test
    bool hoist_ = false;   // emit dominant spheres first, ahead of the tree (build)
    float flatten_ = 0.0f;  // > 0: inner nodes with >= this fraction of the area above are not emitted (emit_tree)
    uint32_t n_hoisted_ = 0;
};

}  // namespace

int rtw_build_bvh(const rtw_scene_desc& desc, std::vector<rtw_node>& nodes, rtw_geometry& geom,
                  uint32_t* depth, uint32_t* axis_draws, float* box_pad, float* extent, uint32_t orders,
                  uint32_t sah_max_leaf, uint32_t hoist, uint32_t* n_hoisted, uint32_t flatten_pct) {
    if (box_pad) *box_pad = 0;
    if (extent) *extent = 0;
    if (n_hoisted) *n_hoisted = 0;
    Geometry geo(desc, geom);
    if (int rc = geo.build()) return rc;
    if (desc.bvh_mode == RTW_BVH_SAH) {
        SahBuilder b(desc, geo, nodes, sah_max_leaf, hoist != 0, geo.loose_boxes() ? 0.0f : (float)flatten_pct / 100.0f);
        b.build(orders);
        if (n_hoisted) *n_hoisted = b.hoisted();
        if (depth) *depth = b.depth();
        if (axis_draws) *axis_draws = 0;
        // Pad the inner boxes for the FMA slab test: its t error for a plane P and
        // origin o is < 4 ulp of (|P| + |o|) in space, so a pad of E * 2^-19
        // (E = max |coordinate| of the scene) keeps the test conservative for
        // every origin with |o| <= 7E (checked per launch, else the exact test runs).
        // A superset of boxes is visited; sphere tests decide the hit.
        // E spans every object's box, not only the inner nodes: hoisted spheres (Book-1's r = 1000
        // ground) are leaves outside the tree, and secondary rays start anywhere on them -- ground
        // hits near the horizon lie hundreds of units out, so an E of the tree alone would not
        // cover their origins.
        float e = 0;
        for (const rtw_node& n : nodes) {
            uint32_t w;
            std::memcpy(&w, &n.a[3], 4);
            if (w & RTW_LEAF_BIT) continue;
            for (int k = 0; k < 3; k++) e = std::max(e, std::max(std::fabs(n.a[k]), std::fabs(n.b[k])));
        }
        for (const Obj& o : geo.objects())
            for (int k = 0; k < 3; k++) e = std::max(e, std::max(std::fabs(o.box.mn[k]), std::fabs(o.box.mx[k])));
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
        // Instance leaves test their own world box before the transforms and member tests (object_leaf):
        // a hit the leaf accepts at t in [0.001, closest] is a point computed through the transform chain
        // (Translate / RotateY, objects.zig:314-326, 401-435) and the member tests -- or, for a medium whose
        // boundary is the instance, a point between two boundary hits (objects.zig:470-507) -- so it lies
        // within a few ulp of (|o| + t|d|) <= 15E of the box, not exactly inside it.  E * 2^-12 on top of the
        // slab test's pad covers 273 ulp of 15E for every origin the fast test admits (|o| <= 7E); the
        // exact test (far origins, tuning.fast_box = 0) never culls.
        const float ipad = pad + e * 2.4414062e-04f;  // + 2^-12
        for (uint32_t i = 0; i < (uint32_t)geom.insts.size(); i++) {
            const Box& b = geo.instance_true_box(i);
            for (int k = 0; k < 3; k++) {
                geom.insts[i].box[0][k] = b.mn[k] - ipad;
                geom.insts[i].box[1][k] = b.mx[k] + ipad;
            }
        }
        if (box_pad) *box_pad = pad;
        if (extent) *extent = e;
        return RTW_OK;
    }
    if (desc.bvh_mode != RTW_BVH_REFERENCE) return RTW_E_INVALID;
    RefBuilder b(desc, geo, nodes);
    b.build();
    if (depth) *depth = b.depth();
    if (axis_draws) *axis_draws = b.axis_draws();
    return RTW_OK;
}

// ---------------------------------------------------------------------------
// Compact 16-B nodes for the wavefront walk of static sphere SAH trees: one
// dwordx4 per step instead of two (the walk is bound by the vector-memory
// gather rate, not by arithmetic).  Same indices and skip links as the 32-B
// array (hit ids and shading keep using it):
//   inner: x = minx | miny << 16, y = minz | maxx << 16, z = maxy | maxz << 16
//          (fp16, min rounded down and max up: a superset of the padded box,
//          read by v_fma_mix_f32 at no conversion cost), w = the skip target's byte
//          offset from the start of the array (all 8 copies)
//   leaf:  center.xyz (fp32), w = bits(radius * radius) | RTW_LEAF_BIT (the
//          reference's `radius * radius`, objects.zig:126, evaluated once here
//          with the same fp32 rounding); a leaf's successor is always i + 1
namespace {

uint16_t h_bits(_Float16 h) {
    uint16_t b;
    std::memcpy(&b, &h, 2);
    return b;
}
float h_val(uint16_t b) {
    _Float16 h;
    std::memcpy(&h, &b, 2);
    return (float)h;
}
// one fp16 ulp toward -inf / +inf (finite inputs)
uint16_t h_prev(uint16_t b) { return (b & 0x8000) ? (uint16_t)(b + 1) : (b == 0 ? (uint16_t)0x8001 : (uint16_t)(b - 1)); }
uint16_t h_next(uint16_t b) { return (b & 0x8000) ? (b == 0x8000 ? (uint16_t)0x0001 : (uint16_t)(b - 1)) : (uint16_t)(b + 1); }
bool h_subnormal(uint16_t b) { return (b & 0x7C00) == 0 && (b & 0x03FF) != 0; }
// largest fp16 <= x that is zero or normal (a subnormal could be flushed by the hardware)
uint16_t h_down(float x) {
    uint16_t b = h_bits((_Float16)x);
    if (h_val(b) > x) b = h_prev(b);
    if (h_subnormal(b)) b = (b & 0x8000) ? (uint16_t)0x8400 : (uint16_t)0x0000;
    return b;
}
uint16_t h_up(float x) {
    uint16_t b = h_bits((_Float16)x);
    if (h_val(b) < x) b = h_next(b);
    if (h_subnormal(b)) b = (b & 0x8000) ? (uint16_t)0x8000 : (uint16_t)0x0400;
    return b;
}

}  // namespace

// The 32-B fp32 form (fp32 = true, 4 copies only; rtw_tuning.compact_nodes 2): two uint4 per node, the
// padded fp32 box of the 32-B array itself (the box_next fast test's operands: no rounding outward needed)
// laid out for packed FMAs -- v_pk_fma_f32 does two of the slab test's FMAs in the time v_fma_mix_f32 does one:
//   inner: (near x, min y, far x, max y), (near z, far z, skip, 0)   near / far by the copy's x and z signs;
//          skip = the target's byte offset from the array start (32 B per node)
//   leaf:  (center.xyz, bits(radius * radius)), (0, 0, RTW_LEAF_BIT, 0)
bool rtw_compact_nodes(const std::vector<rtw_node>& nodes, uint32_t orders, std::vector<rtw_cnode>& out, bool fp32) {
    // one copy per ray-direction octant, or (orders = 4) per sign pair of x and z
    if ((orders != 8 && orders != 4) || nodes.size() % orders || (fp32 && orders != 4)) return false;
    const size_t per = nodes.size() / orders;
    if (fp32) {
        out.assign(2 * nodes.size(), rtw_cnode{});
        auto fb = [](float f) {
            uint32_t b;
            std::memcpy(&b, &f, 4);
            return b;
        };
        for (size_t i = 0; i < nodes.size(); i++) {
            const uint32_t oct = (uint32_t)(i / per);
            const rtw_node& n = nodes[i];
            rtw_cnode& c0 = out[2 * i];
            rtw_cnode& c1 = out[2 * i + 1];
            uint32_t w;
            std::memcpy(&w, &n.a[3], 4);
            if (w & RTW_LEAF_BIT) {
                const float rr = n.b[0] * n.b[0];  // objects.zig:126, as the 16-B form
                if (!(rr >= 0) || !std::isfinite(rr)) return false;
                std::memcpy(&c0.v[0], &n.a[0], 12);
                c0.v[3] = fb(rr);
                c1.v[2] = RTW_LEAF_BIT;
                continue;
            }
            for (int k = 0; k < 3; k++)
                if (!std::isfinite(n.a[k]) || !std::isfinite(n.b[k])) return false;
            const bool nx = oct & 1u, nz = (oct >> 1) & 1u;
            c0.v[0] = fb(nx ? n.b[0] : n.a[0]);
            c0.v[1] = fb(n.a[1]);
            c0.v[2] = fb(nx ? n.a[0] : n.b[0]);
            c0.v[3] = fb(n.b[1]);
            c1.v[0] = fb(nz ? n.b[2] : n.a[2]);
            c1.v[1] = fb(nz ? n.a[2] : n.b[2]);
            const uint64_t skip_bytes = ((uint64_t)oct * per + (w & RTW_SKIP_MASK)) * 32u;
            if (skip_bytes >= RTW_LEAF_BIT) return false;
            c1.v[2] = (uint32_t)skip_bytes;
        }
        return true;
    }
    out.resize(nodes.size());
    for (size_t i = 0; i < nodes.size(); i++) {
        const uint32_t oct = (uint32_t)(i / per);  // order_of: bit k set = negative direction on axis k
        const rtw_node& n = nodes[i];
        rtw_cnode& c = out[i];
        uint32_t w;
        std::memcpy(&w, &n.a[3], 4);
        if (w & RTW_LEAF_BIT) {
            const float rr = n.b[0] * n.b[0];
            uint32_t rb;
            std::memcpy(&rb, &rr, 4);
            if (!(rr >= 0) || !std::isfinite(rr) || (rb & RTW_LEAF_BIT)) return false;
            std::memcpy(&c.v[0], &n.a[0], 12);
            c.v[3] = rb | RTW_LEAF_BIT;
            continue;
        }
        // per axis the slab the copy's rays enter first (near) and leave last (far):
        // min/max for a non-negative direction component, swapped for a negative one
        // (orders = 4: x and z by the copy's signs, y as min / max -- traverse_compact<.., Y4> takes the
        // median of three, which needs no order between the two y slabs)
        uint16_t h[6];
        for (int k = 0; k < 3; k++) {
            if (!(std::fabs(n.a[k]) <= 60000.0f) || !(std::fabs(n.b[k]) <= 60000.0f)) return false;
            const uint16_t lo = h_down(n.a[k]), hi = h_up(n.b[k]);
            const bool neg = orders == 4 ? (k == 1 ? false : ((oct >> (k / 2)) & 1u)) : ((oct >> k) & 1u);
            h[k] = neg ? hi : lo;
            h[3 + k] = neg ? lo : hi;
        }
        c.v[0] = (uint32_t)h[0] | ((uint32_t)h[1] << 16);
        c.v[1] = (uint32_t)h[2] | ((uint32_t)h[3] << 16);
        c.v[2] = (uint32_t)h[4] | ((uint32_t)h[5] << 16);
        // the skip target as the BYTE offset of its node from the start of the whole array (all copies):
        // the walk steps through byte addresses, with no index -> address multiply per step
        const uint64_t skip_bytes = ((uint64_t)oct * per + (w & RTW_SKIP_MASK)) * 16u;
        if (skip_bytes >= RTW_LEAF_BIT) return false;
        c.v[3] = (uint32_t)skip_bytes;
    }
    return true;
}

// ---------------------------------------------------------------------------
// Two-wide nodes for the stack walk of large static sphere SAH trees (trees the
// kernels read through L1/L2, e.g. the 100 k-sphere stress scene).  One 32-B
// record per inner node of ordering 0 holds BOTH children, so a walk step tests
// two children after one dependent load, and the near inner child is chosen per
// ray at run time instead of by 8 octant-ordered copies: 1/8 of the footprint in
// L1/L2 and about half the dependent loads per ray.
//   slot k (v[4k .. 4k+3]) of an inner child: box per axis min | max << 16 (fp16
//           rounded outward, a superset of the padded box), then the child's record
//           index (pre-order over the inner nodes, root 0)
//   slot k of a leaf child: the sphere in place -- center.xyz (fp32), bits(r * r) |
//           RTW_LEAF_BIT (as the compact nodes), tested with no box (bvh.zig:123-125)
// leaf_id[2 * record + k] = the leaf's index in ordering 0: the hit id the shading
// reads (looked up once per ray, after the walk).
// *max_stack = the most entries the walk can push (the max inner depth).
bool rtw_wide2_nodes(const std::vector<rtw_node>& nodes, uint32_t n_per, std::vector<rtw_cnode>& out,
                     std::vector<uint32_t>& leaf_id, uint32_t* max_stack) {
    auto word = [&](uint32_t i) {
        uint32_t w;
        std::memcpy(&w, &nodes[i].a[3], 4);
        return w;
    };
    // a forest: h hoisted leaves (SahBuilder::build) ahead of the tree's root at node h.  Record k < h is
    // a virtual inner node: slot 0 the hoisted sphere k, slot 1 record k + 1 (or the tree's root), whose
    // box encloses everything after it -- the walk tests the hoisted spheres first, as the pre-order does.
    uint32_t h = 0;
    while (h < n_per && (word(h) & RTW_LEAF_BIT)) h++;
    if (n_per < h + 3 || nodes.size() < n_per) return false;
    std::vector<uint32_t> widx(n_per, 0), depth(n_per, 0);
    uint32_t n_inner = h;
    for (uint32_t i = h; i < n_per; i++)
        if (!(word(i) & RTW_LEAF_BIT)) widx[i] = n_inner++;
    out.assign(2 * (size_t)n_inner, rtw_cnode{});
    leaf_id.assign(2 * (size_t)n_inner, 0u);
    auto sphere_slot = [&](uint32_t j, size_t slot) {
        const rtw_node& n = nodes[j];
        uint32_t mv;
        std::memcpy(&mv, &n.b[3], 4);
        const float rr = n.b[0] * n.b[0];
        uint32_t rb;
        std::memcpy(&rb, &rr, 4);
        if (mv || !(rr >= 0) || !std::isfinite(rr) || (rb & RTW_LEAF_BIT)) return false;
        std::memcpy(&out[slot].v[0], &n.a[0], 12);
        out[slot].v[3] = rb | RTW_LEAF_BIT;
        leaf_id[slot] = j;
        return true;
    };
    auto box_slot = [&](const float* mn, const float* mx, uint32_t rec, size_t slot) {
        for (int a = 0; a < 3; a++) {
            if (!(std::fabs(mn[a]) <= 60000.0f) || !(std::fabs(mx[a]) <= 60000.0f)) return false;
            out[slot].v[a] = (uint32_t)h_down(mn[a]) | ((uint32_t)h_up(mx[a]) << 16);
        }
        out[slot].v[3] = rec;
        return true;
    };
    {   // the virtual records, from the last (its slot 1 is the tree's root) to the first
        float mn[3], mx[3];
        for (int a = 0; a < 3; a++) {
            mn[a] = nodes[h].a[a];
            mx[a] = nodes[h].b[a];
        }
        for (uint32_t k = h; k-- > 0;) {
            if (!sphere_slot(k, 2 * (size_t)k) || !box_slot(mn, mx, k + 1 < h ? k + 1 : widx[h], 2 * (size_t)k + 1))
                return false;
            const float r = std::fabs(nodes[k].b[0]), pad = 1e-3f * (r + 1.0f);
            for (int a = 0; a < 3; a++) {  // + sphere k: the box of record k's subtree, for record k - 1
                mn[a] = std::min(mn[a], nodes[k].a[a] - r - pad);
                mx[a] = std::max(mx[a], nodes[k].a[a] + r + pad);
            }
            depth[k] = k + 1;
        }
    }
    depth[h] = h + 1;
    uint32_t dmax = h + 1;
    auto next = [&](uint32_t j) { return (word(j) & RTW_LEAF_BIT) ? j + 1 : (word(j) & RTW_SKIP_MASK); };
    for (uint32_t i = h; i < n_per; i++) {
        if (word(i) & RTW_LEAF_BIT) continue;
        const uint32_t c[2] = {i + 1, next(i + 1)};
        if (c[1] >= n_per || next(c[1]) != (word(i) & RTW_SKIP_MASK)) return false;  // not a binary tree
        for (int k = 0; k < 2; k++) {
            const uint32_t j = c[k];
            const rtw_node& n = nodes[j];
            const size_t slot = 2 * (size_t)widx[i] + k;
            rtw_cnode& o = out[slot];
            (void)o;
            if (word(j) & RTW_LEAF_BIT) {
                if (!sphere_slot(j, slot)) return false;
                continue;
            }
            if (!box_slot(n.a, n.b, widx[j], slot)) return false;  // padded by rtw_build_bvh
            depth[j] = depth[i] + 1;
            dmax = std::max(dmax, depth[j]);
        }
    }
    if (max_stack) *max_stack = dmax;
    return true;
}
