"""The host backend of the C ABI (rtw_scene_create(desc, RTW_DEVICE_CPU, ...), csrc/rtw_cpu.hip):
Camera.render (src/camera.zig:93-116) on host threads with the GPU's per-sample code, here on
CPU only (no GPU needed), against the oracle under the GPU parity contract -- every channel of
every pixel within 1e-5 (5e-5 at depth 200) relative -- for every scene class: Book-1 (both
BVH modes), HEAD's moving spheres + checker + earth texture, BASELINE config 5 (image + Perlin),
quads, Cornell box, Cornell smoke (ConstantMedium), simple_light.  Also BASELINE config 1
(400x225, 10 spp) through the reference's 8-Task split (src/main.zig:314-326), cancel, and
that the device-buffer / multi-GPU entry points refuse a host context."""
import ctypes as C
import os

import numpy as np
import pytest

CPU = -1


def close(got, ref, rel=1e-5):
    return np.abs(got - ref) <= rel * np.maximum(1.0, np.abs(ref))


def host_render(rtw, arr, cam, spp, seed, threads=0, s0=0, buf=None):
    world = rtw.World(arr, device=CPU, tuning={"cpu_threads": threads} if threads else None)
    if buf is None:
        buf = np.zeros((cam.size, 4), np.float32)
    rc = rtw.lib().rtw_render(world.handle, C.byref(cam.derived), 0, cam.size, s0, spp, seed, buf.ctypes.data, None,
                              rtw._abi.PROGRESS_FN(0), None)
    rtw._abi.check(rc, "rtw_render (host context)")
    world.close()
    return buf


@pytest.mark.parametrize("mode", ["sah", "reference"])
def test_book1_vs_oracle(rtw, oracle, mode):
    m = {"sah": rtw._abi.RTW_BVH_SAH, "reference": rtw._abi.RTW_BVH_REFERENCE}[mode]
    arr = rtw.flatten(rtw.worlds.generate_world(0, "book1"), bvh_mode=m)
    cam = rtw.book1_camera(image_width=160, aspect_ratio=1.5, spp=4, max_depth=50).init()
    got = host_render(rtw, arr, cam, 4, 7)
    ow = oracle.World(arr.spheres, arr.materials, arr.textures)
    ocam = oracle.camera(image_width=160, aspect_ratio=1.5, samples_per_pixel=4, max_depth=50, background_mode=1)
    ref = ow.render_pixels(ocam, 7, np.arange(cam.size, dtype=np.uint32), 0, 4, threads=os.cpu_count() or 1)
    assert (got[:, 3] == 4).all()
    assert close(got[:, :3], ref[:, :3]).all(), np.abs(got[:, :3] - ref[:, :3]).max()
    assert (got[:, :3] == ref[:, :3]).all(axis=1).mean() > 0.5   # most paths: bit-exact


def test_textured_head_and_c5_vs_oracle(rtw, oracle, earth_rgba):
    imgs = [rtw.Image(earth_rgba)]
    arr = rtw.flatten(rtw.worlds.generate_world(0, "ref_head", imgs))
    cam = rtw.book1_camera(image_width=160, aspect_ratio=16 / 9, spp=3, max_depth=50).init()
    got = host_render(rtw, arr, cam, 3, 3)
    ow = oracle.World(arr.spheres, arr.materials, arr.textures, arr.perlins, [earth_rgba])
    ocam = oracle.camera(image_width=160, aspect_ratio=16 / 9, samples_per_pixel=3, max_depth=50, background_mode=1)
    ref = ow.render_pixels(ocam, 3, np.arange(cam.size, dtype=np.uint32), 0, 3, threads=os.cpu_count() or 1)
    assert close(got[:, :3], ref[:, :3]).all()

    arr = rtw.flatten(rtw.worlds.earth_perlin_world(0, imgs))
    cam = rtw.earth_perlin_camera(image_width=192, spp=3).init()
    got = host_render(rtw, arr, cam, 3, 1)
    ow = oracle.World(arr.spheres, arr.materials, arr.textures, arr.perlins, [earth_rgba])
    ocam = oracle.camera(aspect_ratio=16 / 9, image_width=192, samples_per_pixel=3, max_depth=50,
                         background=(0.7, 0.8, 1.0), background_mode=0, vfov=30.0, lookat=(0.0, 1.0, 0.0),
                         defocus_angle=0.0)
    ref = ow.render_pixels(ocam, 1, np.arange(cam.size, dtype=np.uint32), 0, 3, threads=os.cpu_count() or 1)
    assert close(got[:, :3], ref[:, :3]).all(), np.abs(got[:, :3] - ref[:, :3]).max()


OBJECT_SCENES = {
    "quads": (lambda w: w.quads_world()[:4], dict(aspect_ratio=1.0, vfov=80.0, lookfrom=(0.0, 0.0, 9.0),
                                                  lookat=(0.0, 0.0, 0.0), defocus_angle=0.0,
                                                  background=(0.7, 0.8, 1.0)), 64, 50),
    "cornell": (lambda w: w.cornell_box(), dict(aspect_ratio=1.0, vfov=40.0, lookfrom=(278.0, 278.0, -800.0),
                                                lookat=(278.0, 278.0, 0.0), defocus_angle=0.0), 48, 200),
    "cornell_smoke": (lambda w: w.cornell_smoke(), dict(aspect_ratio=1.0, vfov=40.0, lookfrom=(278.0, 278.0, -800.0),
                                                        lookat=(278.0, 278.0, 0.0), defocus_angle=0.0), 48, 50),
    "simple_light": (lambda w: w.simple_light_world(0), dict(aspect_ratio=16 / 9, vfov=20.0, lookfrom=(26.0, 3.0, 6.0),
                                                             lookat=(0.0, 2.0, 0.0), defocus_angle=0.0), 64, 50),
}


@pytest.mark.parametrize("name", list(OBJECT_SCENES))
def test_object_scenes_vs_oracle(rtw, oracle, name):
    """Reference topology: the host walk replays the oracle's tree, so ties resolve alike."""
    build, kw, W, depth = OBJECT_SCENES[name]
    arr = rtw.flatten(build(rtw.worlds), bvh_mode=rtw._abi.RTW_BVH_REFERENCE)
    cam = rtw.Camera(image_width=W, samples_per_pixel=4, max_depth=depth, **kw).init()
    ocam = oracle.camera(image_width=W, samples_per_pixel=4, max_depth=depth, **kw)
    got = host_render(rtw, arr, cam, 4, 5)
    ref = oracle.World.from_arrays(arr).render_pixels(ocam, 5, np.arange(cam.size, dtype=np.uint32), 0, 4,
                                                     threads=os.cpu_count() or 1)
    assert close(got[:, :3], ref[:, :3], 5e-5).all(), np.abs(got[:, :3] - ref[:, :3]).max()


def test_c1_reference_tasks(rtw, oracle):
    """BASELINE config 1 (400x225, 10 spp, depth 50): the reference's 8 Tasks of size/8
    (start_render over a host context) == the oracle's 8-thread render; progressive split
    [0,4) + [4,10) == one call; thread count does not change a bit."""
    arr = rtw.flatten(rtw.worlds.generate_world(0, "book1"))
    world = rtw.World(arr, device=CPU)
    cam = rtw.book1_camera(image_width=400, aspect_ratio=16 / 9, spp=10, max_depth=50)
    cam.init()
    writer = rtw.SharedStateImageWriter(cam.image_width, cam.image_height)
    state = rtw.RayTraceState(cam, writer, world, seed=0)
    rtw.start_render(state, 8)
    ow = oracle.World(arr.spheres, arr.materials, arr.textures)
    ocam = oracle.camera(image_width=400, aspect_ratio=16 / 9, samples_per_pixel=10, max_depth=50, background_mode=1)
    obuf, _ = ow.render_threads(ocam, 0, 8)
    assert close(writer.buffer[:, :3], obuf[:, :3]).all()
    assert np.array_equal(writer.buffer[:, 3], obuf[:, 3])
    world.close()
    one = host_render(rtw, arr, cam, 10, 0, threads=3)
    two = host_render(rtw, arr, cam, 4, 0, threads=5)
    two = host_render(rtw, arr, cam, 10, 0, threads=2, s0=4, buf=two)
    assert np.array_equal(one, two)


def test_host_context_cancel_and_refusals(rtw):
    arr = rtw.flatten(rtw.worlds.generate_world(0, "book1"))
    world = rtw.World(arr, device=CPU)
    cam = rtw.book1_camera(image_width=64, aspect_ratio=1.5, spp=2).init()
    buf = np.zeros((cam.size, 4), np.float32)
    flag = C.c_int32(1)
    rc = rtw.lib().rtw_render(world.handle, C.byref(cam.derived), 0, cam.size, 0, 2, 0, buf.ctypes.data,
                              C.byref(flag), rtw._abi.PROGRESS_FN(0), None)
    assert rc == rtw._abi.RTW_E_CANCELLED
    L = rtw.lib()
    assert L.rtw_render_device(world.handle, C.byref(cam.derived), 0, cam.size, 0, 2, 0, buf.ctypes.data, None,
                               None) == rtw._abi.RTW_E_INVALID
    assert L.rtw_render_rows_device(world.handle, C.byref(cam.derived), 8, 1, 0, 0, 2, 0, buf.ctypes.data, None,
                                    None) == rtw._abi.RTW_E_INVALID
    h = C.c_void_p()
    ctxs = (C.c_void_p * 1)(world.handle.value)
    assert L.rtw_multi_create(ctxs, 1, C.byref(h)) == rtw._abi.RTW_E_INVALID
    world.close()


def test_host_render_rows_shards_reassemble(rtw):
    """rtw_render_rows on a host context (ABI 5): every shard of a row-interleaved split, rendered into its
    own host tile, reassembles to the single-call host render bit for bit (rows past H never written)."""
    arr = rtw.flatten(rtw.worlds.generate_world(0, "book1"))
    world = rtw.World(arr, device=CPU)
    cam = rtw.book1_camera(image_width=72, aspect_ratio=1.5, spp=3).init()
    W, H = cam.derived.image_width, cam.derived.image_height
    full = host_render(rtw, arr, cam, 3, 4)
    for n, rpb in ((3, 8), (2, 5), (4, 1)):
        image = np.zeros((H, W, 4), np.float32)
        for k in range(n):
            rows = rtw.distributed.shard_rows(H, rpb, n, k)
            tile = np.full((len(rows) * W + W, 4), -7.0, np.float32)   # one guard row past the shard
            tile[:len(rows) * W] = 0
            rtw.distributed.render_rows_host(world, cam, rpb, n, k, 0, 3, tile, seed=4)
            assert (tile[len(rows) * W:] == -7.0).all()
            image[rows] = tile[:len(rows) * W].reshape(len(rows), W, 4)
        assert np.array_equal(image.reshape(-1, 4), full), (n, rpb)
    world.close()


def test_host_render_ex_stop_and_progress(rtw):
    """ABI-5 stop/progress on a host context: a cleared `running` byte (RenderThread.running) stops before
    anything is rendered; progress after every spp batch, and a stop from it keeps the finished batches
    (w = their end); resuming the range completes the image bit-identically."""
    arr = rtw.flatten(rtw.worlds.generate_world(0, "book1"))
    world = rtw.World(arr, device=CPU)
    cam = rtw.book1_camera(image_width=48, aspect_ratio=1.5, spp=6).init()
    L = rtw.lib()
    buf = np.zeros((cam.size, 4), np.float32)
    running = C.c_uint8(0)
    o = rtw._abi.render_opts(running=running)
    assert L.rtw_render_ex(world.handle, C.byref(cam.derived), 0, cam.size, 0, 6, 2, buf.ctypes.data,
                           C.byref(o)) == rtw._abi.RTW_E_CANCELLED
    assert not buf.any()
    running.value = 1
    seen = []
    o = rtw._abi.render_opts(spp_batch=2, running=running,
                             progress=lambda d, t: seen.append((d, t)) or len(seen) == 1)
    assert L.rtw_render_ex(world.handle, C.byref(cam.derived), 0, cam.size, 0, 6, 2, buf.ctypes.data,
                           C.byref(o)) == rtw._abi.RTW_E_CANCELLED
    assert seen == [(cam.size * 2, cam.size * 6)]
    assert (buf[:, 3] == 2).all()
    o = rtw._abi.render_opts(running=running)
    rtw._abi.check(L.rtw_render_ex(world.handle, C.byref(cam.derived), 0, cam.size, 2, 6, 2, buf.ctypes.data,
                                   C.byref(o)), "rtw_render_ex")
    assert np.array_equal(buf, host_render(rtw, arr, cam, 6, 2))
    world.close()


def test_scene_hash_independent_of_tree_layout(rtw):
    """rtw_scene_hash (the checkpoint's scene key) names the scene, not the node layout the tuning
    picks: equal under orderings, hoisting and object-tree flattening; different for another tree
    kind, another reference-topology seed and another scene."""
    def h(arr, tu=None):
        world = rtw.World(arr, device=CPU, tuning=tu)
        out = C.c_uint64()
        rtw._abi.check(rtw.lib().rtw_scene_hash(world.handle, C.byref(out)), "rtw_scene_hash")
        world.close()
        return out.value

    book = rtw.flatten(rtw.worlds.generate_world(0, "book1"))
    base = h(book)
    assert h(book, {"bvh_orders": 1}) == base and h(book, {"hoist": 0}) == base
    assert h(rtw.flatten(rtw.worlds.generate_world(0, "book1"), bvh_mode=rtw._abi.RTW_BVH_REFERENCE)) != base
    assert h(rtw.flatten(rtw.worlds.generate_world(1, "book1"))) != base
    cornell = rtw.flatten(rtw.worlds.cornell_box())
    assert h(cornell, {"object_tree": 0}) == h(cornell) == h(cornell, {"object_tree": 50})
