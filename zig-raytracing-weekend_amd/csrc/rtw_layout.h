// rtw_layout.h -- device-resident scene layout (HBM), shared by the host-side
// builder (rtw_bvh.cpp / rtw_host.hip) and the gfx950 kernels (rtw_kernels.hip).
//
// Node (32 B = two 16-B loads).  Nodes are stored in
// depth-first pre-order of the reference BVHTree (src/bvh.zig:43-89) with a
// skip link = index of the first node after the subtree.  A stackless
// traversal (hit -> i+1, miss -> skip) therefore visits nodes in exactly the
// order of the reference's recursive BVHNode.hit (src/bvh.zig:122-136):
// left subtree first, right subtree with the interval shrunk to the closest
// hit so far, leaves tested without a box test.
//
//   inner: a = (bmin.x, bmin.y, bmin.z, bits(skip))            b = (bmax.x, bmax.y, bmax.z, 0)
//   leaf : a = (c1.x,   c1.y,   c1.z,   bits(skip | LEAF_BIT)) b = (radius, bits(mat), bits(sphere), bits(moving))
//
// Moving spheres keep center_vec = center2 - center1 in a side array indexed by
// sphere id (only read when the moving flag is set).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RTW_LEAF_BIT 0x80000000u
#define RTW_SKIP_MASK 0x7FFFFFFFu

struct rtw_node {
    float a[4];
    float b[4];
};
static_assert(sizeof(rtw_node) == 32, "node must be 32 bytes");

// Leaf b.w: bit 0 = moving sphere, bits 8..15 = object kind (RTW_OBJ_*).  Non-sphere
// leaves: a = (0, 0, 0, bits(skip | LEAF_BIT)), b = (0, bits(mat), bits(index), bits(kind << 8)).
#define RTW_LEAF_KIND(bw) (((bw) >> 8) & 0xFFu)
// object reference inside the device arrays: kind in the top 4 bits
#define RTW_REF(kind, idx) (((uint32_t)(kind) << 28) | (uint32_t)(idx))
#define RTW_REF_KIND(r) ((r) >> 28)
#define RTW_REF_INDEX(r) ((r) & 0x0FFFFFFFu)
// hit id of a closest hit: leaf node | instance member << 24
#define RTW_HIT_NODE_BITS 24

// 32 B: every sphere (instance members read these; world-object spheres are inlined in their leaf)
struct rtw_dev_sphere {
    float c1[3];
    float radius;
    uint32_t mat, moving, _p0, _p1;
};
static_assert(sizeof(rtw_dev_sphere) == 32, "sphere record must be 32 bytes");

// 80 B: Quad.init derived fields (objects.zig:201-210)
struct rtw_dev_quad {
    float q[3];
    float d;
    float n[3];
    uint32_t mat;
    float u[4];
    float v[4];
    float w[4];
};
static_assert(sizeof(rtw_dev_quad) == 80, "quad record must be 80 bytes");

// 96 B: members[first .. first+count) (RTW_REF), xf[k] = {bits(kind), a, b, c}:
// translate (a, b, c) = offset; rotate_y a = sin, b = cos.  xf[0] innermost.
// box: the instance's world box (RotateY/Translate.init) padded for the leaf's own FMA slab test
// (rtw_build_bvh; SAH trees only, else +-inf): box[0] = min.xyz, box[1] = max.xyz
struct rtw_dev_instance {
    uint32_t first, count, n_xf, _p;
    float xf[3][4];
    float box[2][4];
};
static_assert(sizeof(rtw_dev_instance) == 96, "instance record must be 96 bytes");

// 16 B: ConstantMedium
struct rtw_dev_medium {
    uint32_t boundary;       // RTW_REF
    float neg_inv_density;
    uint32_t mat;
    uint32_t _p;
};

// 32 B: {kind, texture, fuzz, ir} {albedo.xyz, 0}
struct rtw_dev_material {
    uint32_t kind;
    uint32_t texture;
    float fuzz;
    float ir;
    float albedo[4];
};
static_assert(sizeof(rtw_dev_material) == 32, "material must be 32 bytes");

// 48 B, same field order as rtw_texture (image/perlin are indices)
struct rtw_dev_texture {
    uint32_t kind;
    uint32_t image;
    uint32_t perlin;
    float scale;
    float even[4];
    float odd[4];
};
static_assert(sizeof(rtw_dev_texture) == 48, "texture must be 48 bytes");

struct rtw_dev_image {
    uint64_t offset;          // byte offset into the image blob
    uint32_t width, height, bytes_per_row, _pad;
};

// Per perlin table: ranvec as float4[256] (4 KiB) then perm_x|perm_y|perm_z as uint32[3][256]
#define RTW_PERLIN_BYTES (256 * 16 + 3 * 256 * 4)

// Row-interleaved shards (multi-GPU): row r of shard `shard`'s compact
// tile is image row ((r / rpb) * n_shards + shard) * rpb + r % rpb (>= H: padding).
// One definition for the render kernels (map_row), the multi-GPU pack/unpack and the
// host (rtw_shard_image_row).
__host__ __device__ inline uint32_t rtw_tile_row_image(uint32_t rpb, uint32_t n_shards, uint32_t shard, uint32_t r) {
    return ((r / rpb) * n_shards + shard) * rpb + r % rpb;
}
