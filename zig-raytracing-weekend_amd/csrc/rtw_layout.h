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

// Balanced shards (rows_per_block | RTW_ROWS_BALANCED, include/rtw_gpu.h):
//  * rounds of n blocks are dealt in alternating order -- round k gives its block k * n + s to shard s when k is
//    even and to shard n - 1 - s when k is odd -- so no shard always takes the lowest block of a round (the
//    plain order gives shard n - 1 the bottom rpb rows of every n * rpb: where the image's cost grows downwards,
//    as Book-1's ground does, C2's shard 7 at 8 ranks rendered 7 % more than shard 0);
//  * the rows left over after the whole rounds (H mod (rpb * n)) are split evenly -- `sub` = ceil(rest / n)
//    consecutive rows each, in one more block slot of the tile -- so every shard renders the same number of rows
//    (+- sub) instead of one block more for the first rest / rpb shards (C2 at 8: 100 rows each, not 104 / 96).
// The tiles keep rpb-row blocks, so a shard's 8x8 pixel tiles still cover adjacent image rows.  Needs the image
// height; every function below takes it.
#define RTW_ROWS_FLAGS 0x80000000u
__host__ __device__ inline uint32_t rtw_shard_row(uint32_t H, uint32_t rpbf, uint32_t n, uint32_t s, uint32_t r) {
    const uint32_t rpb = rpbf & ~RTW_ROWS_FLAGS;
    if (!(rpbf & RTW_ROWS_FLAGS)) return rtw_tile_row_image(rpb, n, s, r);
    const uint32_t full = H / (rpb * n), fr = full * rpb;  // whole rounds; a shard's tile rows in them
    const uint32_t k = r / rpb, pos = (k & 1u) ? n - 1u - s : s;  // round k, the shard's block in it
    if (r < fr) return (k * n + pos) * rpb + r % rpb;
    const uint32_t y0 = full * rpb * n, sub = (H - y0 + n - 1) / n, i = r - fr;
    return i < sub ? y0 + pos * sub + i : 0xFFFFFFFFu;  // (>= H: padding)
}
// tile rows of shard s (padded: whole blocks), and the largest over the shards (every tile's capacity)
__host__ __device__ inline uint32_t rtw_shard_tile_rows(uint32_t H, uint32_t rpbf, uint32_t n, uint32_t s) {
    const uint32_t rpb = rpbf & ~RTW_ROWS_FLAGS;
    if (!(rpbf & RTW_ROWS_FLAGS)) {
        const uint32_t nblk = (H + rpb - 1) / rpb;
        return nblk > s ? (nblk - s + n - 1) / n * rpb : 0u;
    }
    const uint32_t full = H / (rpb * n), y0 = full * rpb * n, sub = (H - y0 + n - 1) / n;
    const uint32_t pos = (full & 1u) ? n - 1u - s : s;  // the shard's place in the last (partial) round
    return full * rpb + (pos * sub < H - y0 ? rpb : 0u);
}
__host__ __device__ inline uint32_t rtw_shard_capacity(uint32_t H, uint32_t rpbf, uint32_t n) {
    const uint32_t rpb = rpbf & ~RTW_ROWS_FLAGS;
    if (!(rpbf & RTW_ROWS_FLAGS)) return rtw_shard_tile_rows(H, rpbf, n, 0);
    const uint32_t full = H / (rpb * n);
    return full * rpb + (H > full * rpb * n ? rpb : 0u);
}
