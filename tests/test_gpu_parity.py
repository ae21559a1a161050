"""GPU parity: the gfx950 kernels (through the C ABI) against the C oracle.

Tolerance contract: every ray, hit, normal and scatter
direction is computed with the same fp32 operations as the oracle
(-ffp-contract=off, correctly rounded div/sqrt, restated Zig pow), so paths are
identical; only the radiance product is re-associated (iterative L += T*e vs
the reference's recursive e + a*(...)), bounded by max_depth * 2^-24 relative
per sample.  Tests assert |gpu - oracle| <= 1e-5 * max(1, |oracle|) per
channel for every pixel, textured scenes included: the sphere UV's acos/atan2 and
the noise's sin are the Zig toolchain's algorithms restated on both sides
(csrc/rtw_libm.h, oracle/zig_libm.h; tests/test_libm.py), so texel indices and
noise values are bit-identical too.
"""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

REL = 1e-5


@pytest.fixture(scope="module", params=["sah", "reference"])
def book1(rtw, request):
    """Book-1 world in both BVH modes: the SAH tree (product default) and the
    reference's random-axis median topology (exact traversal replay)."""
    mode = {"sah": rtw._abi.RTW_BVH_SAH, "reference": rtw._abi.RTW_BVH_REFERENCE}[request.param]
    arr = rtw.flatten(rtw.worlds.generate_world(0, "book1"), bvh_mode=mode)
    return arr, rtw.World(arr)


@pytest.fixture(scope="module")
def oracle_book1(oracle):
    sp, mt, tx = oracle.gen_book1(0, 0)
    return oracle.World(sp, mt, tx)


def close(gpu, ref, rel=REL):
    return np.abs(gpu - ref) <= rel * np.maximum(1.0, np.abs(ref))


def render_rows(rtw, world, cam, y0, y1, spp_begin, spp_end, seed, buf=None):
    """rtw_render over full rows [y0, y1) (host buffer API)."""
    W = cam.derived.image_width
    if buf is None:
        buf = np.zeros((cam.size, 4), np.float32)
        buf[:, 3] = 1
    rc = rtw.lib().rtw_render(world.handle, C.byref(cam.derived), y0 * W, y1 * W, spp_begin, spp_end, seed,
                              buf.ctypes.data, None, rtw._abi.PROGRESS_FN(0), None)
    rtw._abi.check(rc, "rtw_render")
    return buf


def test_device_count(rtw):
    n = C.c_int()
    rtw.lib().rtw_device_count(C.byref(n))
    assert n.value >= 1


def test_device_rng_bit_exact(rtw, oracle, book1):
    _, world = book1
    out = np.zeros(64, np.float32)
    for seed, pix, s in ((0, 0, 0), (1, 959999, 499), (12345, 77, 3)):
        rtw._abi.check(rtw.lib().rtw_debug_rng(world.handle, seed, pix, s, 64, out.ctypes.data), "rtw_debug_rng")
        assert np.array_equal(out, oracle.path_floats(seed, pix, s, 64))


def test_per_sample_radiance(rtw, oracle, book1, oracle_book1):
    """One sample at a time: GPU device function vs oracle recursion."""
    _, world = book1
    cam = rtw.book1_camera().init()
    ocam = oracle.camera(image_width=1200, aspect_ratio=1.5, samples_per_pixel=500, max_depth=50, background_mode=1)
    rng = np.random.default_rng(3)
    out = np.zeros(3, np.float32)
    n_exact = 0
    pairs = list(zip(rng.integers(0, cam.size, 300), rng.integers(0, 500, 300)))
    for pix, s in pairs:
        rtw._abi.check(rtw.lib().rtw_debug_sample(world.handle, C.byref(cam.derived), 0, int(pix), int(s),
                                                  out.ctypes.data), "rtw_debug_sample")
        ref = oracle_book1.sample(ocam, 0, int(pix), int(s))
        assert close(out, ref).all(), (pix, s, out, ref)
        n_exact += int(np.array_equal(out, ref))
    assert n_exact >= len(pairs) // 2   # most paths have <= 2 bounces: bit-exact


@pytest.mark.parametrize("name", ["book1_c2_center", "book1_c2_ground", "book1_c2_glass"])
def test_golden_crops_book1(rtw, book1, name):
    """Committed oracle float4 crops (tests/golden/crops.npz) vs rtw_render."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    crop = {c[0]: c for c in mg.CROPS}[name]
    _, _, camkw, (x0, y0, w, h), spp, seed = crop
    with np.load(os.path.join(GOLDEN, "crops.npz"), allow_pickle=False) as z:
        ref, pix = z[name], z[name + "_pix"]
    _, world = book1
    cam = rtw.book1_camera(image_width=camkw["image_width"], aspect_ratio=camkw["aspect_ratio"],
                           spp=camkw["samples_per_pixel"], max_depth=camkw["max_depth"]).init()
    buf = np.zeros((cam.size, 4), np.float32)
    render_rows(rtw, world, cam, y0, y0 + h, 0, spp, seed, buf)
    got = buf[pix]
    assert np.array_equal(got[:, 3], ref[:, 3])
    ok = close(got[:, :3], ref[:, :3])
    assert ok.all(), (np.argwhere(~ok)[:5], np.abs(got[:, :3] - ref[:, :3]).max())


def test_golden_crop_ref_head_moving(rtw, earth_rgba):
    """HEAD scene: moving spheres (initMoving), checker ground, earth texture."""
    with np.load(os.path.join(GOLDEN, "crops.npz"), allow_pickle=False) as z:
        ref = z["head_small"]
    imgs = [rtw.Image(earth_rgba)]
    world = rtw.World(rtw.flatten(rtw.worlds.generate_world(0, "ref_head", imgs)))
    cam = rtw.book1_camera(image_width=320, aspect_ratio=16 / 9, spp=8, max_depth=50).init()
    buf = render_rows(rtw, world, cam, 0, 180, 0, 8, 3)
    ok = close(buf[:, :3], ref[:, :3])
    assert ok.all(), (ok.all(axis=1).mean(), np.abs(buf[:, :3] - ref[:, :3]).max())


def test_sky_rows_vs_reference_image2(rtw, book1):
    """GPU reproduces the reference's own image2.ppm sky rows (+-1 LSB, round-256)."""
    with np.load(os.path.join(GOLDEN, "sky_rows.npz"), allow_pickle=False) as z:
        rows = z["image2_rows"].astype(np.int32)
    _, world = book1
    cam = rtw.book1_camera(image_width=400, aspect_ratio=16 / 9, spp=64, max_depth=50)
    cam.pixel_offset = 0
    cam.init()
    buf = render_rows(rtw, world, cam, 0, 15, 0, 64, 0)[:15 * 400]
    g = np.sqrt(buf[:, :3] / buf[:, 3:4])
    got = np.round(256 * np.clip(g, 0, 0.999)).astype(np.int32).reshape(15, 400, 3)
    assert np.abs(got - rows).max() <= 1


def test_c2_full_size_properties(rtw, oracle, book1, oracle_book1):
    """BASELINE config 2 geometry (1200x800) at 8 spp: batch invariance, shard
    invariance, determinism, no NaN, and oracle agreement on 3000 random pixels."""
    _, world = book1
    cam = rtw.book1_camera().init()
    a = render_rows(rtw, world, cam, 0, 800, 0, 8, 0)
    b = render_rows(rtw, world, cam, 0, 800, 0, 3, 0)
    b = render_rows(rtw, world, cam, 0, 800, 3, 8, 0, b)
    assert np.array_equal(a, b)                        # progressive batches == one pass
    c = render_rows(rtw, world, cam, 0, 800, 0, 8, 0)
    assert np.array_equal(a, c)                        # deterministic
    assert np.isfinite(a).all() and (a[:, 3] == 8).all()
    pix = np.random.default_rng(0).choice(cam.size, 3000, replace=False).astype(np.uint32)
    ocam = oracle.camera(image_width=1200, aspect_ratio=1.5, samples_per_pixel=500, max_depth=50, background_mode=1)
    ref = oracle_book1.render_pixels(ocam, 0, pix, 0, 8, threads=os.cpu_count() or 1)
    assert close(a[pix, :3], ref[:, :3]).all()


def test_four_copy_stage_full_c2(rtw, book1):
    """BASELINE config 2 at its geometry (1200x800, 6 spp): the 4-copy compact stage at two blocks per CU
    (tuning.bvh_orders 4: copies by the x and z signs, y's slabs by med3) renders the 8-copy image bit for bit,
    as do its one-block and split-kernel forms."""
    arr, world = book1
    cam = rtw.book1_camera().init()
    ref = render_rows(rtw, world, cam, 0, 800, 0, 6, 2)
    for tu in ({"bvh_orders": 4}, {"bvh_orders": 4, "clds_shape": 1},
               {"bvh_orders": 4, "clds_shape": 4}, {"bvh_orders": 4, "fuse": 0}, {"bvh_orders": 4, "compact_nodes": 2},
               {"bvh_orders": 4, "compact_nodes": 2, "fuse": 0}):
        w = rtw.World(arr, tuning=tu)
        got = render_rows(rtw, w, cam, 0, 800, 0, 6, 2)
        w.close()
        assert np.array_equal(ref, got), tu


def test_shard_rows_reassemble(rtw, book1):
    """rtw_render_rows_device (the multi-GPU unit) reassembles to the 1-GPU image."""
    import torch
    _, world = book1
    cam = rtw.book1_camera(image_width=600, aspect_ratio=1.5, spp=4).init()
    H, W = cam.derived.image_height, cam.derived.image_width
    full = render_rows(rtw, world, cam, 0, H, 0, 4, 9)
    BAL = rtw._abi.RTW_ROWS_BALANCED
    for n_shards, rpb in ((3, 8), (8, 16), (2, 1), (8, 8 | BAL), (3, 8 | BAL), (7, 16 | BAL)):
        img = np.zeros((H, W, 4), np.float32)
        d = rtw.distributed
        for s in range(n_shards):
            rows = rtw.lib().rtw_shard_rows(H, rpb, n_shards, s)
            tr = d.shard_tile_rows(H, rpb, n_shards, s)
            tile = torch.zeros((max(1, tr) * W, 4), dtype=torch.float32, device="cuda")
            rc = rtw.lib().rtw_render_rows_device(world.handle, C.byref(cam.derived), rpb, n_shards, s, 0, 4, 9,
                                                  tile.data_ptr(), None, None)
            rtw._abi.check(rc, "rtw_render_rows_device")
            t = tile.cpu().numpy().reshape(-1, W, 4)
            ys = [d.shard_row(H, rpb, n_shards, s, r) for r in range(tr)]
            k = 0
            for r, y in enumerate(ys):
                if y < H:
                    img[y] = t[r]
                    k += 1
            assert k == rows
        assert np.array_equal(img.reshape(-1, 4)[:, :3], full[:, :3])


def test_reference_task_chunks(rtw, oracle, book1, oracle_book1):
    """start_render: 8 Tasks of size/8 (main.zig:314-326) == oracle threads render;
    trailing size % 8 pixels untouched; texture = toGamma2 of the buffer."""
    arr, world = book1
    cam = rtw.book1_camera(image_width=203, aspect_ratio=16 / 9, spp=4, max_depth=50)
    cam.init()
    writer = rtw.SharedStateImageWriter(cam.image_width, cam.image_height)
    state = rtw.RayTraceState(cam, writer, world, seed=11)
    rtw.start_render(state, 8)
    ocam = oracle.camera(image_width=203, aspect_ratio=16 / 9, samples_per_pixel=4, max_depth=50, background_mode=1)
    obuf, otex = oracle_book1.render_threads(ocam, 11, 8)
    chunk = cam.size // 8
    assert close(writer.buffer[:, :3], obuf[:, :3]).all()
    assert np.array_equal(writer.buffer[:, 3], obuf[:, 3])
    assert (writer.buffer[chunk * 8:] == np.array([0, 0, 0, 1], np.float32)).all()
    same = (writer.buffer == obuf).all(axis=1)
    assert np.array_equal(writer.texture_buffer[same][:chunk * 8], otex[same][:chunk * 8])


def test_cancel_between_batches(rtw, book1):
    _, world = book1
    cam = rtw.book1_camera(image_width=300, aspect_ratio=1.5, spp=64).init()
    writer = rtw.SharedStateImageWriter(cam.image_width, cam.image_height)
    state = rtw.RayTraceState(cam, writer, world)
    state.stop()
    with pytest.raises(rtw.RtwError) as e:
        cam.render(state, rtw.Task(0, cam.size))
    assert e.value.code == rtw._abi.RTW_E_CANCELLED


def test_textured_c5_crop(rtw, oracle, earth_rgba):
    """Config 5 (earthmap image texture + Perlin noise) on a 1920x1080 crop."""
    imgs = [rtw.Image(earth_rgba)]
    arr = rtw.flatten(rtw.worlds.earth_perlin_world(0, imgs))
    world = rtw.World(arr)
    cam = rtw.earth_perlin_camera(image_width=1920, spp=4).init()
    y0, y1 = 400, 464
    buf = render_rows(rtw, world, cam, y0, y1, 0, 4, 1)
    ow = oracle.World(arr.spheres, arr.materials, arr.textures, arr.perlins, [earth_rgba])
    ocam = oracle.camera(aspect_ratio=16 / 9, image_width=1920, samples_per_pixel=4, max_depth=50,
                         background=(0.7, 0.8, 1.0), background_mode=0, vfov=30.0, lookat=(0.0, 1.0, 0.0),
                         defocus_angle=0.0)
    pix = np.arange(y0 * 1920, y1 * 1920, dtype=np.uint32)
    ref = ow.render_pixels(ocam, 1, pix, 0, 4, threads=os.cpu_count() or 1)
    got = buf[pix]
    ok = close(got[:, :3], ref[:, :3]).all(axis=1)
    assert ok.all(), (ok.mean(), np.abs(got[:, :3] - ref[:, :3]).max())


def test_stress_100k_crop(rtw, oracle):
    """Config 4 (100k spheres): deep reference-topology BVH, GPU vs oracle on a strip."""
    arr = rtw.flatten(rtw.worlds.stress_world(100_000, 0), bvh_mode=rtw._abi.RTW_BVH_REFERENCE)
    world = rtw.World(arr)
    arr_sah = rtw.flatten(rtw.worlds.stress_world(100_000, 0))
    world_sah = rtw.World(arr_sah)
    st = world.stats()
    assert st["n_nodes"] == 2 * len(arr.spheres) - 1
    cam = rtw.book1_camera(image_width=1920, aspect_ratio=16 / 9, spp=2).init()
    y0, y1 = 500, 516
    buf = render_rows(rtw, world, cam, y0, y1, 0, 2, 0)
    ow = oracle.World(arr.spheres, arr.materials, arr.textures)
    ocam = oracle.camera(image_width=1920, aspect_ratio=16 / 9, samples_per_pixel=256, max_depth=50,
                         background_mode=1)
    pix = np.arange(y0 * 1920, y1 * 1920, dtype=np.uint32)
    ref = ow.render_pixels(ocam, 0, pix, 0, 2, threads=os.cpu_count() or 1)
    assert close(buf[pix, :3], ref[:, :3]).all()
    buf2 = render_rows(rtw, world_sah, cam, y0, y1, 0, 2, 0)
    assert close(buf2[pix, :3], ref[:, :3]).all()


def test_device_counters_equal_reference_traversal(rtw, oracle, book1, oracle_book1):
    """The stackless walk visits exactly the reference's nodes: device ray/node/leaf
    counters == oracle's instrumented recursion on the same pixels."""
    import torch
    arr, world = book1
    if arr.bvh_mode != rtw._abi.RTW_BVH_REFERENCE:
        pytest.skip("traversal-count identity holds for the reference topology")
    cam = rtw.book1_camera(image_width=1200, aspect_ratio=1.5, spp=2).init()
    y0, y1 = 300, 332
    acc = torch.zeros((cam.size, 4), dtype=torch.float32, device="cuda")
    cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
    opts = rtw._abi.RtwRenderOpts(0, 0, cnt.data_ptr())
    rc = rtw.lib().rtw_render_device(world.handle, C.byref(cam.derived), y0 * 1200, y1 * 1200, 0, 2, 0,
                                     acc.data_ptr(), None, C.byref(opts))
    rtw._abi.check(rc, "rtw_render_device")
    g = cnt.cpu().numpy()
    ocam = oracle.camera(image_width=1200, aspect_ratio=1.5, samples_per_pixel=500, max_depth=50, background_mode=1)
    pix = np.arange(y0 * 1200, y1 * 1200, dtype=np.uint32)
    with oracle.counters() as oc:
        oracle_book1.render_pixels(ocam, 0, pix, 0, 2, threads=1)
    assert g[rtw._abi.RTW_STAT_SAMPLES] == oc.samples
    assert g[rtw._abi.RTW_STAT_RAYS] == oc.rays
    assert g[rtw._abi.RTW_STAT_NODES] == oc.nodes
    assert g[rtw._abi.RTW_STAT_LEAVES] == oc.leaves


@pytest.mark.parametrize("scene", ["book1", "ref_head"])
def test_persistent_v1_bit_identical_to_v0(rtw, earth_rgba, scene):
    """The persistent megakernel (dynamic pixel queue, path regeneration, LDS BVH,
    feature-specialised) and the simple per-pixel kernel perform the same fp32
    operations per pixel in the same order: outputs are bit-identical."""
    imgs = [rtw.Image(earth_rgba)]
    arr = rtw.flatten(rtw.worlds.generate_world(0, scene, imgs))
    cam = rtw.book1_camera(image_width=480, aspect_ratio=1.5, spp=6).init()
    outs = {}
    for k in ("v0", "v1", "wf"):
        world = rtw.World(arr, tuning={"kernel": KERNELS[k]})
        outs[k] = render_rows(rtw, world, cam, 0, cam.derived.image_height, 0, 6, 21)
        world.close()
    assert np.array_equal(outs["v0"], outs["v1"])
    assert np.array_equal(outs["v0"], outs["wf"])


KERNELS = {"wf": 0, "v1": 1, "v0": 2}   # rtw_kernel_kind


@pytest.mark.parametrize("knob", [{"mega_shade_min": 1}, {"mega_shade_min": 64}, {"mega_tile_order": 0},
                                  {"mega_waves": 8}, {"lds": 127 & ~64}])
def test_v1_knobs_invariant(rtw, book1, knob):
    """Megakernel scheduling (rtw_tuning: ballot threshold, tile order, launch
    bounds, LDS staging) only moves work between lanes: outputs are bit-identical."""
    arr, _ = book1
    cam = rtw.book1_camera(image_width=300, aspect_ratio=1.5, spp=3).init()
    w1 = rtw.World(arr, tuning={"kernel": 1})
    ref = render_rows(rtw, w1, cam, 0, 200, 0, 3, 4)
    w1.close()
    w2 = rtw.World(arr, tuning={"kernel": 1, **knob})
    got = render_rows(rtw, w2, cam, 0, 200, 0, 3, 4)
    w2.close()
    assert np.array_equal(ref, got)


@pytest.mark.parametrize("knob", [{"wf_iters": 1}, {"wf_iters": 9}, {"wf_iters": 50}, {"wf_paths": 4096}, {"fast_box": 0},
                                  {"lds": 127 & ~1}, {"sah_max_leaf": 4}, {"compact_nodes": 0}, {"lds": 127 & ~2},
                                  {"fuse": 0}, {"fuse": 1}, {"lds": 127 & ~4}, {"bvh_orders": 1}, {"tile_lists": 0}, {"tile_lists": 2}, {"tile_lists": 64},
                                  {"lds": 127 & ~2, "wide_walk": 0}, {"fuse": 5}, {"lds": 127 & ~2, "fuse": 5},
                                  {"lds": 127 & ~2, "fuse": 5, "wide_walk": 0}, {"hoist": 0}, {"hoist": 0, "fuse": 0},
                                  {"sort_iters": 0}, {"sort_iters": 50}, {"sort_iters_split": 50, "fuse": 0}, {"sort_iters_split": 0, "fuse": 0},
                                  {"sort_iters": 2, "wf_iters": 1}, {"sort_bits": 0}, {"sort_bits": 2, "fuse": 0}, {"wf_iters": 3, "fuse": 0},
                                  {"bvh_orders": 4}, {"bvh_orders": 4, "clds_shape": 1}, {"bvh_orders": 4, "fuse": 0},
                                  {"bvh_orders": 4, "lds": 127 & ~2}, {"bvh_orders": 4, "wide_walk": 0, "lds": 127 & ~2},
                                  {"bvh_orders": 4, "compact_nodes": 0}, {"bvh_orders": 4, "kernel": 1},
                                  {"bvh_orders": 4, "kernel": 2}, {"bvh_orders": 4, "compact_nodes": 2},
                                  {"bvh_orders": 4, "compact_nodes": 2, "fuse": 0},
                                  {"bvh_orders": 4, "compact_nodes": 2, "lds": 127 & ~2},
                                  {"bvh_orders": 4, "compact_nodes": 2, "tile_lists": 0},
                                  {"bvh_orders": 8, "compact_nodes": 2}, {"deal": 9}, {"deal": 9, "fuse": 0},
                                  {"deal": 9, "lds": 127 & ~2}, {"deal": 9, "wf_paths": 4096},
                                  {"deal": 0}, {"deal": 0, "fuse": 0}, {"deal": 0, "lds": 127 & ~2, "fuse": 5},
                                  {"deal": 9, "wf_iters": 1}, {"deal": 9, "fuse": 0, "wf_iters": 2},
                                  {"deal": 9, "lds": 127 & ~2, "fuse": 5}, {"deal": 9, "fuse": 1},
                                  {"deal": 10}, {"deal": 11, "wf_iters": 1}, {"deal": 11}, {"deal": 11, "fuse": 0},
                                  {"deal": 11, "wf_paths": 4096}, {"deal": 11, "wf_paths": 65536, "fuse": 0},
                                  {"deal": 59}, {"deal": 27, "lds": 127 & ~2, "fuse": 5}, {"deal": 57, "wf_iters": 9}, {"deal": 51},
                                  {"deal": 59, "fuse": 0}, {"deal": 59, "lds": 127 & ~2, "fuse": 0}, {"deal": 51, "fuse": 0, "wf_iters": 3},
                                  # deal 128 (RTW_DEAL_SMALL_SORT): the direction-bucketed queues of the large benched
                                  # batches on this small image -- fused compact-LDS step (4- and 8-copy stages, one and
                                  # two blocks per CU, fp32 nodes), fused step through L1/L2, split trace / shade, all
                                  # iterations bucketed, fewer key bits, many batches, the static deal
                                  {"deal": 187}, {"deal": 187, "sort_iters": 50}, {"deal": 187, "sort_iters": 50, "wf_iters": 9},
                                  {"deal": 187, "bvh_orders": 8}, {"deal": 187, "clds_shape": 1}, {"deal": 187, "compact_nodes": 2},
                                  {"deal": 187, "lds": 127 & ~2, "fuse": 5}, {"deal": 187, "lds": 127 & ~2, "fuse": 5, "sort_iters": 50},
                                  {"deal": 187, "fuse": 0}, {"deal": 187, "fuse": 0, "sort_iters_split": 50},
                                  {"deal": 187, "fuse": 0, "sort_iters_split": 3, "wf_iters": 9}, {"deal": 187, "sort_bits": 2},
                                  {"deal": 187, "fuse": 0, "sort_bits": 1}, {"deal": 187, "wf_paths": 65536},
                                  {"deal": 187, "fuse": 0, "wf_paths": 65536}, {"deal": 128}, {"deal": 128, "fuse": 0},
                                  {"deal": 187, "lds": 127 & ~2, "fuse": 0, "wide_walk": 0}])
def test_wavefront_knobs_invariant(rtw, book1, knob):
    """Wavefront tuning (rtw_tuning: bounces before the tail kernel, batch size ->
    many batches, FMA vs reference slab test, LDS-staged nodes, SAH leaf runs of up
    to 4 spheres, 16-B fp16-box nodes vs 32-B nodes, compact nodes in LDS, fused
    gen+trace+shade kernel vs separate kernels, LDS vs L1/L2 tail, materials in LDS,
    one node ordering instead of 8, camera rays against per-tile candidate lists vs
    the walk, the two-wide stack walk through L1/L2 vs the
    octant-ordered compact walk, the fused step through L1/L2, dominant spheres hoisted ahead of the
    tree or not, survivors filed into direction-bucketed blocks or appended -- forced on at this size by deal bit
    128, as the benched batches run them --; the dynamic and static deals; the fused path's packed 48-B path
    state and the split path's 60-B one, each with its tail) never changes a pixel."""
    arr, world = book1
    cam = rtw.book1_camera(image_width=300, aspect_ratio=1.5, spp=5).init()
    ref = render_rows(rtw, world, cam, 0, 200, 0, 5, 4)
    w2 = rtw.World(arr, tuning=knob)
    got = render_rows(rtw, w2, cam, 0, 200, 0, 5, 4)
    w2.close()
    assert np.array_equal(ref, got)


@pytest.mark.parametrize("n,seed", [(20000, 3), (100000, 0)])
def test_compact_nodes_are_exact(rtw, n, seed):
    """The 16-B node walk (fp16 inner boxes rounded outward, leaves with radius^2)
    and the two-wide stack walk (fp16 child boxes, leaf boxes padded like inner ones)
    visit a superset of the 32-B walk's boxes: identical images on dense stress
    worlds (small spheres far from the origin: the coarsest fp16 boxes), at the
    BASELINE config-4 camera."""
    arr = rtw.flatten(rtw.worlds.stress_world(n, seed), bvh_mode=rtw._abi.RTW_BVH_SAH)
    cam = rtw.book1_camera(image_width=480, aspect_ratio=16 / 9, spp=4).init()
    outs = []
    for tu in ({"compact_nodes": 0, "tile_lists": 0, "hoist": 0}, {"compact_nodes": 1, "wide_walk": 0},
               {"compact_nodes": 1, "wide_walk": 1}, {"compact_nodes": 1, "wide_walk": 0, "hoist": 0},
               {"compact_nodes": 1, "wide_walk": 0, "bvh_orders": 4}, {"compact_nodes": 2, "bvh_orders": 4}):
        w = rtw.World(arr, tuning=tu)
        outs.append(render_rows(rtw, w, cam, 0, cam.derived.image_height, 0, 4, 6))
        w.close()
    assert np.isfinite(outs[1]).all()
    assert np.array_equal(outs[0], outs[1])
    assert np.array_equal(outs[0], outs[2])  # the two-wide stack walk (rtw_wide2_nodes): same hits
    assert np.array_equal(outs[0], outs[3])  # the ground sphere inside the tree (no hoisting)
    assert np.array_equal(outs[0], outs[4])  # 4 (x, z)-sign copies, y near/far by med3 (traverse_compact<.., Y4>)
    assert np.array_equal(outs[0], outs[5])  # their 32-B fp32-box form, packed FMAs (traverse_compact<.., F32>)
    # (the defaults also give camera rays the frustum-walked tile lists of large trees: same hits)


@pytest.mark.parametrize("scene", ["ref_head", "book1"])
def test_hoisted_ground_to_the_horizon(rtw, scene):
    """The FMA slab test's pad covers secondary-ray origins on the hoisted r = 1000 ground, hundreds of units
    out at the horizon (rtw_bvh.hip: the pad's extent spans every object box, hoisted ones included): the
    ground hoisted ahead of the tree or inside it, and the exact slab test, give the same image.  ref_head has
    moving spheres (the padded 32-B fp32 walk); the camera looks up so the horizon crosses the frame."""
    arr = rtw.flatten(rtw.worlds.generate_world(0, scene))
    cam = rtw.Camera(aspect_ratio=1.5, image_width=360, samples_per_pixel=4, max_depth=50,
                     background_mode=rtw._abi.RTW_BG_GRADIENT, vfov=40.0, lookfrom=(13.0, 2.0, 3.0),
                     lookat=(0.0, 2.0, 0.0), defocus_angle=0.0, focus_dist=10.0).init()
    outs = []
    for tu in ({"hoist": 1}, {"hoist": 0}, {"hoist": 1, "fast_box": 0}, {"hoist": 0, "fast_box": 0}):
        w = rtw.World(arr, tuning=tu)
        assert w.stats()["n_hoisted"] == tu["hoist"]
        outs.append(render_rows(rtw, w, cam, 0, cam.derived.image_height, 0, 4, 11))
        w.close()
    assert np.isfinite(outs[0]).all()
    for o in outs[1:]:
        assert np.array_equal(outs[0], o)


@pytest.mark.parametrize("scene", ["book1", "stress"])
def test_fast_reject_is_exact(rtw, scene):
    """The sphere fast-reject (hardware sqrt/rcp estimate + error margin) never
    changes a result: bit-identical to the always-IEEE path."""
    objs = rtw.worlds.generate_world(0, "book1") if scene == "book1" else rtw.worlds.stress_world(20000, 3)
    arr = rtw.flatten(objs)
    cam = rtw.book1_camera(image_width=600, aspect_ratio=1.5, spp=4).init()
    outs = []
    for fr in (0, 1):
        w = rtw.World(arr, tuning={"fast_reject": fr})
        outs.append(render_rows(rtw, w, cam, 0, cam.derived.image_height, 0, 4, 5))
        w.close()
    assert np.array_equal(outs[0], outs[1])


def test_texture_from_accum_device_matches_host(rtw):
    """Device texel update (rtw_texture_from_accum_device) == host toGamma2 texels."""
    import torch
    rng = np.random.default_rng(1)
    acc = np.concatenate([rng.random((5000, 3), np.float32) * 30, rng.integers(1, 64, (5000, 1)).astype(np.float32)], 1)
    acc[:4, :3] = 0
    acc[4:8, :3] = 1e7
    host = np.zeros((5000, 4), np.uint8)
    rtw.lib().rtw_texture_from_accum(acc.ctypes.data, 5000, host.ctypes.data)
    d_acc = torch.from_numpy(acc).cuda()
    d_out = torch.zeros((5000, 4), dtype=torch.uint8, device="cuda")
    rtw._abi.check(rtw.lib().rtw_texture_from_accum_device(d_acc.data_ptr(), 5000, d_out.data_ptr(), None), "tex")
    torch.cuda.synchronize()
    assert np.array_equal(d_out.cpu().numpy(), host)


def test_progressive_and_resume_bit_identical(rtw, book1, tmp_path):
    """progressive batches (the interactive UI loop) and a
    checkpoint -> new process state -> resume are bit-identical to one render;
    countSamples reaches spp * n; a checkpoint of another scene is refused."""
    arr, world = book1
    cam = rtw.book1_camera(image_width=160, aspect_ratio=1.5, spp=7).init()
    one = rtw.RayTraceState(cam, rtw.SharedStateImageWriter(160, cam.derived.image_height), world, seed=5)
    one.writer.buffer[:, 3] = 0
    cam.render_range(one, 0, cam.size, 0, 7)
    prog = rtw.RayTraceState(cam, rtw.SharedStateImageWriter(160, cam.derived.image_height), world, seed=5)
    prog.writer.buffer[:, 3] = 0
    seen = []
    done = rtw.progressive_render(prog, 0, 2, lambda s, n: seen.append((s, n)) or s >= 4)
    assert done == 4 and [s for s, _ in seen] == [2, 4] and seen[-1][1] == 4 * cam.size
    prog.checkpoint(str(tmp_path / "c.ckpt"), done)
    fresh = rtw.RayTraceState(cam, rtw.SharedStateImageWriter(160, cam.derived.image_height), world, seed=5)
    start = fresh.resume(str(tmp_path / "c.ckpt"))
    assert start == 4
    assert rtw.progressive_render(fresh, start, 2) == 7
    assert np.array_equal(fresh.writer.buffer, one.writer.buffer)
    assert fresh.count_samples() == 7 * cam.size
    other = rtw.World(rtw.flatten(rtw.worlds.two_spheres_world()))
    bad = rtw.RayTraceState(cam, rtw.SharedStateImageWriter(160, cam.derived.image_height), other, seed=5)
    with pytest.raises(rtw.RtwError):
        bad.resume(str(tmp_path / "c.ckpt"))
    other.close()


def test_c3_geometry_multi_batch_and_shards(rtw, oracle, book1, oracle_book1):
    """BASELINE config 3 (3840x2160, the 8-GPU config) at its own geometry.
    (1) samples [0, 72) of the full image cross the wavefront batch split: at 8.3 M
    pixels a 2^29-path batch holds 64 samples, so the render runs as 2 batches (counted
    by the reduce launches) -- a full-width row strip and 1500 random pixels match the
    oracle at 1e-5 and every w = 72; (2) 8 row-interleaved shards of 8-row blocks
    (the C3 sharding, rtw_render_rows_device) reassemble bit-identically to the 1-GPU
    image (camera.zig:93-116 semantics on every pixel)."""
    import torch
    _, world = book1
    cam = rtw.book1_camera(image_width=3840, aspect_ratio=16 / 9, spp=1024).init()
    W, H = cam.derived.image_width, cam.derived.image_height
    assert (W, H) == (3840, 2160)
    acc = torch.zeros((cam.size, 4), dtype=torch.float32, device="cuda")
    timing = rtw._abi.RtwKernelTiming()
    opts = rtw._abi.RtwRenderOpts(0, 0, None, C.pointer(timing))
    rtw._abi.check(rtw.lib().rtw_render_device(world.handle, C.byref(cam.derived), 0, cam.size, 0, 72, 0,
                                               acc.data_ptr(), None, C.byref(opts)), "rtw_render_device")
    assert timing.launches[rtw._abi.RTW_K_REDUCE] >= 2, "expected the render to span several batches"
    got = acc.cpu().numpy()
    assert np.isfinite(got).all() and (got[:, 3] == 72).all()
    rng = np.random.default_rng(33)
    pix = np.unique(np.concatenate([np.arange(1200 * W, 1201 * W),
                                    rng.choice(cam.size, 1500, replace=False)])).astype(np.uint32)
    ocam = oracle.camera(image_width=3840, aspect_ratio=16 / 9, samples_per_pixel=1024, max_depth=50,
                         background_mode=1)
    ref = oracle_book1.render_pixels(ocam, 0, pix, 0, 72, threads=os.cpu_count() or 1)
    ok = close(got[pix, :3], ref[:, :3])
    assert ok.all(), (pix[np.argwhere(~ok)[:5, 0]], np.abs(got[pix, :3] - ref[:, :3]).max())
    del acc

    full = torch.zeros((cam.size, 4), dtype=torch.float32, device="cuda")
    rtw._abi.check(rtw.lib().rtw_render_device(world.handle, C.byref(cam.derived), 0, cam.size, 0, 2, 5,
                                               full.data_ptr(), None, None), "rtw_render_device")
    n, rpb = 8, 8
    d = rtw.distributed
    cap = d.tile_rows_capacity(H, rpb, n)
    tiles = torch.zeros((n, cap * W, 4), dtype=torch.float32, device="cuda")
    for s in range(n):
        rtw._abi.check(rtw.lib().rtw_render_rows_device(world.handle, C.byref(cam.derived), rpb, n, s, 0, 2, 5,
                                                        tiles[s].data_ptr(), None, None), "rtw_render_rows_device")
    src, dst = d.reassembly_index(H, rpb, n)
    img = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    img.index_copy_(0, torch.tensor(dst, device="cuda"),
                    tiles.view(-1, W, 4).index_select(0, torch.tensor(src, device="cuda")))
    assert torch.equal(img.view(-1, 4), full)


@pytest.mark.parametrize("cam_seed", range(6))
def test_tile_lists_random_cameras(rtw, book1, cam_seed):
    """The camera-ray candidate lists (wf_tile_lists: a conservative superset of the
    spheres a tile's jittered, defocused rays can reach) never change a pixel, for
    random cameras: inside and around the sphere field, wide and narrow fields of
    view, strong defocus, near focus planes, the +1 pixel quirk -- bit-identical to
    the walk."""
    arr, _ = book1
    g = np.random.default_rng(100 + cam_seed)
    lookfrom = tuple(float(v) for v in g.uniform([-14, 0.3, -14], [14, 6, 14]))
    lookat = tuple(float(v) for v in g.uniform([-4, 0, -4], [4, 1.5, 4]))
    cam = rtw.Camera(aspect_ratio=float(g.uniform(0.6, 2.0)), image_width=int(g.integers(96, 200)),
                     samples_per_pixel=3, max_depth=8, background_mode=rtw._abi.RTW_BG_GRADIENT,
                     vfov=float(g.uniform(8, 100)), lookfrom=lookfrom, lookat=lookat,
                     defocus_angle=float(g.choice([0.0, 0.6, 4.0, 12.0])),
                     focus_dist=float(g.uniform(0.5, 20))).init()
    outs = []
    for tl in (0, 1):
        w = rtw.World(arr, tuning={"tile_lists": tl})
        outs.append(render_rows(rtw, w, cam, 0, cam.derived.image_height, 0, 3, cam_seed))
        w.close()
    assert np.isfinite(outs[1]).all()
    assert np.array_equal(outs[0], outs[1])
