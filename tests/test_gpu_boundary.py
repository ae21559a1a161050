"""The drop-in boundary on the GPU (ABI 5): BASELINE config 1 at its own geometry through the
reference's 8 Tasks, and the stop / progress contract of Camera.render's `running` poll
(src/camera.zig:107; RenderThread.running, src/main.zig:50,58-60; the UI's progress and POWER,
main.zig:470-514) for one context, a host-buffer shard and the multi-device frame.

Every comparison with the oracle uses the parity tolerance of test_gpu_parity.py (1e-5 relative,
every pixel); every comparison between two renders of this library is bit-exact."""
import ctypes as C
import os

import numpy as np
import pytest

from test_gpu_parity import close, render_rows

pytestmark = pytest.mark.gpu

CPU = -1


def to_gamma2(buf):
    """SharedStateImageWriter.writeColor's texel (camera.zig:58-65, color.zig:43-62) in fp32."""
    b = buf.astype(np.float32)
    scale = (np.float32(1.0) / b[:, 3]).astype(np.float32)
    x = np.sqrt((b[:, :3] * scale[:, None]).astype(np.float32))
    x = np.clip(x, np.float32(0.0), np.float32(0.999)).astype(np.float32)
    out = np.zeros((b.shape[0], 4), np.uint8)
    out[:, :3] = (np.float32(256.0) * x).astype(np.uint8)
    out[:, 3] = 255
    return out


@pytest.fixture(scope="module")
def c1(rtw, oracle):
    """BASELINE config 1: Book-1, 400x225, 10 spp, depth 50; the oracle's 8-thread render."""
    arr = rtw.flatten(rtw.worlds.generate_world(0, "book1"))
    ow = oracle.World(arr.spheres, arr.materials, arr.textures)
    ocam = oracle.camera(image_width=400, aspect_ratio=16 / 9, samples_per_pixel=10, max_depth=50,
                         background_mode=1)
    obuf, otex = ow.render_threads(ocam, 0, 8)
    return arr, obuf, otex


@pytest.mark.parametrize("device", [0, CPU], ids=["hip", "host"])
def test_c1_full_geometry_eight_tasks(rtw, c1, device):
    """startRender's 8 Tasks of size/8 (main.zig:314-326 -> camera.zig:93-116) over the whole 400x225 x
    10 spp image, on the HIP path and on the host backend: every pixel within 1e-5 of the oracle, w = 10,
    the trailing size % 8 pixels untouched ({0,0,0,1} from scrub), texels = toGamma2 of the buffer and
    equal to the oracle's wherever the buffers agree bit for bit."""
    arr, obuf, otex = c1
    world = rtw.World(arr, device=device)
    cam = rtw.book1_camera(image_width=400, aspect_ratio=16 / 9, spp=10, max_depth=50)
    cam.init()
    assert (cam.derived.image_width, cam.derived.image_height) == (400, 225)
    writer = rtw.SharedStateImageWriter(400, 225)
    state = rtw.RayTraceState(cam, writer, world, seed=0)
    rtw.start_render(state, 8)
    world.close()
    chunk = cam.size // 8
    buf = writer.buffer
    assert close(buf[:, :3], obuf[:, :3]).all(), np.abs(buf[:, :3] - obuf[:, :3]).max()
    assert np.array_equal(buf[:, 3], obuf[:, 3])
    assert (buf[:chunk * 8, 3] == 10).all()
    assert (buf[chunk * 8:] == np.array([0, 0, 0, 1], np.float32)).all()
    assert np.array_equal(writer.texture_buffer[:chunk * 8], to_gamma2(buf[:chunk * 8]))
    same = (buf == obuf).all(axis=1)
    assert same.mean() > 0.3
    assert np.array_equal(writer.texture_buffer[same], otex[same])


def test_c1_hip_equals_host_backend(rtw, c1):
    """The two backends of the boundary render C1 bit-identically (same per-sample code)."""
    arr, _, _ = c1
    cam = rtw.book1_camera(image_width=400, aspect_ratio=16 / 9, spp=10, max_depth=50).init()
    outs = []
    for device in (0, CPU):
        world = rtw.World(arr, device=device)
        outs.append(render_rows(rtw, world, cam, 0, 225, 0, 10, 0))
        world.close()
    assert np.array_equal(outs[0], outs[1])


@pytest.fixture(scope="module")
def book1_world(rtw):
    arr = rtw.flatten(rtw.worlds.generate_world(0, "book1"))
    w = rtw.World(arr)
    yield arr, w
    w.close()


def test_render_ex_progress_stops_after_a_batch(rtw, book1_world):
    """rtw_render_ex: spp_batch 2, progress returns True after the second batch -> RTW_E_CANCELLED, the
    buffer holds exactly samples [0, 4) (== a 4-spp render, bit for bit) with w = 4."""
    arr, world = book1_world
    cam = rtw.book1_camera(image_width=240, aspect_ratio=1.5, spp=10).init()
    ref = render_rows(rtw, world, cam, 0, cam.derived.image_height, 0, 4, 9)
    writer = rtw.SharedStateImageWriter(240, 160)
    state = rtw.RayTraceState(cam, writer, world, seed=9)
    seen = []

    def progress(done, total):
        seen.append((done, total))
        return len(seen) == 2

    with pytest.raises(rtw.RtwError) as e:
        cam.render_range(state, 0, cam.size, 0, 10, progress=progress, spp_batch=2)
    assert e.value.code == rtw._abi.RTW_E_CANCELLED
    assert seen == [(cam.size * 2, cam.size * 10), (cam.size * 4, cam.size * 10)]
    assert np.array_equal(writer.buffer, ref)
    assert np.array_equal(writer.texture_buffer, to_gamma2(ref))


def test_render_ex_running_flag(rtw, book1_world):
    """RenderThread.running as a Zig bool (u8): 0 before the call -> cancelled, nothing rendered; the
    flag cleared by the progress callback (the UI thread's stop(), main.zig:58-60) ends the render after
    the batch that saw it; a non-zero flag renders everything."""
    arr, world = book1_world
    cam = rtw.book1_camera(image_width=120, aspect_ratio=1.5, spp=6).init()
    L = rtw.lib()
    buf = np.zeros((cam.size, 4), np.float32)
    running = C.c_uint8(0)
    o = rtw._abi.render_opts(spp_batch=1, running=running)
    assert L.rtw_render_ex(world.handle, C.byref(cam.derived), 0, cam.size, 0, 6, 1, buf.ctypes.data,
                           C.byref(o)) == rtw._abi.RTW_E_CANCELLED
    assert not buf.any()
    running.value = 1

    def stop_at_3(done, total):
        if done == 3 * cam.size:
            running.value = 0
        return False

    o = rtw._abi.render_opts(spp_batch=1, running=running, progress=stop_at_3)
    assert L.rtw_render_ex(world.handle, C.byref(cam.derived), 0, cam.size, 0, 6, 1, buf.ctypes.data,
                           C.byref(o)) == rtw._abi.RTW_E_CANCELLED
    ref = render_rows(rtw, world, cam, 0, cam.derived.image_height, 0, 3, 1)
    assert np.array_equal(buf[:, :3], ref[:, :3]) and (buf[:, 3] == 3).all()
    running.value = 1
    o = rtw._abi.render_opts(running=running)
    rtw._abi.check(L.rtw_render_ex(world.handle, C.byref(cam.derived), 0, cam.size, 3, 6, 1, buf.ctypes.data,
                                   C.byref(o)), "rtw_render_ex")
    ref6 = render_rows(rtw, world, cam, 0, cam.derived.image_height, 0, 6, 1)
    assert np.array_equal(buf[:, :3], ref6[:, :3]) and (buf[:, 3] == 6).all()
    # device-buffer options are refused on the host-buffer entry point
    bad = rtw._abi.render_opts(flags=rtw._abi.RTW_RENDER_NO_SYNC)
    assert L.rtw_render_ex(world.handle, C.byref(cam.derived), 0, cam.size, 0, 1, 1, buf.ctypes.data,
                           C.byref(bad)) == rtw._abi.RTW_E_INVALID


@pytest.mark.parametrize("n_shards,rpb", [(3, 8), (2, 5)])
def test_render_rows_host_tile_matches_device_tile(rtw, book1_world, n_shards, rpb):
    """rtw_render_rows (host tile, ABI 5) == rtw_render_rows_device (HBM tile) on a GPU context, and the
    tiles reassemble to the single-context frame."""
    import torch
    arr, world = book1_world
    cam = rtw.book1_camera(image_width=160, aspect_ratio=1.5, spp=3).init()
    W, H = cam.derived.image_width, cam.derived.image_height
    full = render_rows(rtw, world, cam, 0, H, 0, 3, 5)
    image = np.zeros((H, W, 4), np.float32)
    for k in range(n_shards):
        rows = rtw.distributed.shard_rows(H, rpb, n_shards, k)
        tile = np.zeros((len(rows) * W, 4), np.float32)
        rtw.distributed.render_rows_host(world, cam, rpb, n_shards, k, 0, 3, tile, seed=5)
        dt = torch.zeros((len(rows) * W, 4), dtype=torch.float32, device="cuda")
        rc = rtw.lib().rtw_render_rows_device(world.handle, C.byref(cam.derived), rpb, n_shards, k, 0, 3, 5,
                                              dt.data_ptr(), None, None)
        rtw._abi.check(rc, "rtw_render_rows_device")
        assert np.array_equal(tile, dt.cpu().numpy())
        image[rows] = tile.reshape(len(rows), W, 4)
    assert np.array_equal(image.reshape(-1, 4), full)


@pytest.fixture(scope="module")
def multi(rtw):
    import torch
    n = max(1, min(8, torch.cuda.device_count()))
    arr = rtw.flatten(rtw.worlds.generate_world(0, "book1"))
    worlds = [rtw.World(arr, device=k) for k in range(n)]
    m = rtw.distributed.MultiDeviceRender(worlds, rows_per_block=8)
    yield worlds, m
    m.close()
    for w in worlds:
        w.close()


def test_multi_info_counts_rccl_ranks(rtw, multi):
    """rtw_multi_info: the communicator sees one rank per device (ncclCommCount)."""
    worlds, m = multi
    assert m.info() == (len(worlds), len(worlds))


def test_multi_device_progress_stops_mid_frame(rtw, multi):
    """rtw_render_multi_device with spp_batch 2 and a progress callback that stops after the second batch:
    RTW_E_CANCELLED, and the frame holds the two finished batches gathered from every device -- bit-identical
    to a single-context render of [0, 4) -- with w = 4."""
    import torch
    worlds, m = multi
    cam = rtw.book1_camera(image_width=200, aspect_ratio=1.5, spp=10).init()
    one = torch.zeros((cam.size, 4), dtype=torch.float32, device="cuda:0")
    rc = rtw.lib().rtw_render_device(worlds[0].handle, C.byref(cam.derived), 0, cam.size, 0, 4, 7, one.data_ptr(),
                                     None, None)
    rtw._abi.check(rc, "rtw_render_device")
    frame = torch.full((cam.size, 4), 5.0, dtype=torch.float32, device="cuda:0")
    seen = []
    with pytest.raises(rtw.RtwError) as e:
        m.render_device(cam, 0, 10, frame.data_ptr(), seed=7, fresh=True, spp_batch=2,
                        progress=lambda d, t: seen.append((d, t)) or len(seen) == 2)
    assert e.value.code == rtw._abi.RTW_E_CANCELLED
    assert seen == [(cam.size * 2, cam.size * 10), (cam.size * 4, cam.size * 10)]
    torch.cuda.synchronize()
    assert torch.equal(one, frame)
    assert bool((frame[:, 3] == 4).all())


def test_multi_host_running_flag_and_resume(rtw, multi):
    """rtw_render_multi_ex on a host buffer: running = 0 -> cancelled with the buffer untouched; cleared
    after the first batch -> that batch kept (w = 3); resuming [3, 9) equals one 9-spp frame."""
    worlds, m = multi
    cam = rtw.book1_camera(image_width=160, aspect_ratio=16 / 9, spp=9).init()
    ref = np.zeros((cam.size, 4), np.float32)
    rtw._abi.check(rtw.lib().rtw_render(worlds[0].handle, C.byref(cam.derived), 0, cam.size, 0, 9, 2,
                                        ref.ctypes.data, None, rtw._abi.PROGRESS_FN(), None), "rtw_render")
    got = np.zeros((cam.size, 4), np.float32)
    running = C.c_uint8(0)
    with pytest.raises(rtw.RtwError):
        m.render_host(cam, 0, 9, got, seed=2, running=running)
    assert not got.any()
    running.value = 1

    def clear(done, total):
        running.value = 0
        return False

    with pytest.raises(rtw.RtwError) as e:
        m.render_host(cam, 0, 9, got, seed=2, spp_batch=3, running=running, progress=clear)
    assert e.value.code == rtw._abi.RTW_E_CANCELLED
    assert (got[:, 3] == 3).all()
    running.value = 1
    m.render_host(cam, 3, 9, got, seed=2, running=running)
    assert np.array_equal(got, ref)
    # the ABI-3 entry point (int32 cancel) polls between batches too
    flag = C.c_int32(1)
    assert rtw.lib().rtw_render_multi(m.handle, C.byref(cam.derived), 8, 0, 9, 2, got.ctypes.data,
                                      C.byref(flag)) == rtw._abi.RTW_E_CANCELLED


FAR = dict(aspect_ratio=16 / 9, vfov=0.4, lookfrom=(19500.0, 3000.0, 4500.0), lookat=(0.0, 0.0, 0.0),
           defocus_angle=0.0, focus_dist=20000.0, background_mode=1)


@pytest.mark.parametrize("case", ["far_camera", "fast_box_0"])
def test_l1l2_walk_honours_fast_box(rtw, case):
    """Trees read through L1/L2 (20 k spheres: the two-wide stack walk by default): a camera beyond
    7 x the scene extent (the box pad's range, so make_launch clears fast_box) and tuning.fast_box = 0
    both take the exact aabb.zig walk -- identical images to the exact 32-B walk."""
    arr = rtw.flatten(rtw.worlds.stress_world(20000, 3))
    if case == "far_camera":
        cam = rtw.Camera(image_width=256, samples_per_pixel=3, max_depth=50, **FAR).init()
        tun = (None, {"compact_nodes": 0, "tile_lists": 0})
    else:
        cam = rtw.book1_camera(image_width=256, aspect_ratio=16 / 9, spp=3).init()
        tun = ({"fast_box": 0}, {"fast_box": 0, "compact_nodes": 0, "tile_lists": 0})
    outs = []
    for tu in tun:
        w = rtw.World(arr, tuning=tu)
        outs.append(render_rows(rtw, w, cam, 0, cam.derived.image_height, 0, 3, 8))
        w.close()
    assert np.isfinite(outs[0]).all() and outs[0][:, :3].any()
    assert np.array_equal(outs[0], outs[1])
