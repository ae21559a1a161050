"""Concurrent callers of one context.  The reference renders with 8 RenderThreads that
call Camera.render at the same time on disjoint chunks (startRender, src/main.zig:314-326;
Camera.render, src/camera.zig:93-116); the Zig binding in INTEGRATION.md keeps those
Tasks.  rtw_render interleaves the calls' spp batches on the context's stream (its lock is held
only while a call enqueues a batch: the wavefront state is per context), and device-API calls on
different streams are ordered on the device: both give the images of back-to-back calls, bit for bit."""
import ctypes as C
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def world(rtw):
    w = rtw.World(rtw.flatten(rtw.worlds.generate_world(0, "book1")))
    yield w
    w.close()


def task_render(rtw, world, cam, start, chunk, buf, rcs, t):
    rcs[t] = rtw.lib().rtw_render(world.handle, C.byref(cam.derived), start, start + chunk, 0,
                                  cam.samples_per_pixel, 7, buf.ctypes.data, None, rtw._abi.PROGRESS_FN(0), None)


def test_eight_concurrent_tasks_match_sequential(rtw, world):
    cam = rtw.book1_camera(image_width=160, aspect_ratio=1.5, spp=6).init()
    chunk = cam.size // 8
    seq = np.zeros((cam.size, 4), np.float32)
    rcs = [0] * 8
    for t in range(8):
        task_render(rtw, world, cam, t * chunk, chunk, seq, rcs, t)
    assert rcs == [0] * 8
    par = np.zeros((cam.size, 4), np.float32)
    threads = [threading.Thread(target=task_render, args=(rtw, world, cam, t * chunk, chunk, par, rcs, t))
               for t in range(8)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert rcs == [0] * 8
    assert (par[: 8 * chunk, 3] == 6).all()
    assert np.array_equal(seq, par)


def test_device_calls_on_two_streams(rtw, world):
    """Unsynchronised rtw_render_device calls on two streams share the context's
    wavefront state; the second waits for the first on the device."""
    import torch
    cam = rtw.book1_camera(image_width=240, aspect_ratio=1.5, spp=4).init()
    half = cam.size // 2
    ref = torch.zeros((cam.size, 4), dtype=torch.float32, device="cuda")
    rtw._abi.check(rtw.lib().rtw_render_device(world.handle, C.byref(cam.derived), 0, cam.size, 0, 4, 3,
                                               ref.data_ptr(), None, None), "rtw_render_device")
    got = torch.zeros_like(ref)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    opts = rtw._abi.RtwRenderOpts(0, rtw._abi.RTW_RENDER_NO_SYNC, None, None)
    for k in range(3):  # alternate streams over disjoint halves and sample ranges
        for s, (p0, p1) in ((s1, (0, half)), (s2, (half, cam.size))):
            rtw._abi.check(rtw.lib().rtw_render_device(world.handle, C.byref(cam.derived), p0, p1, k, k + 1, 3,
                                                       got.data_ptr(), C.c_void_p(s.cuda_stream),
                                                       C.byref(opts)), "rtw_render_device")
    rtw._abi.check(rtw.lib().rtw_render_device(world.handle, C.byref(cam.derived), 0, cam.size, 3, 4, 3,
                                               got.data_ptr(), C.c_void_p(s1.cuda_stream), C.byref(opts)),
                   "rtw_render_device")
    torch.cuda.synchronize()
    assert torch.equal(got[:, 3], ref[:, 3])
    # samples added in the same order (0, 1, 2, 3) per pixel: identical sums
    assert torch.equal(got, ref)


def test_render_ex_and_render_rows_at_once(rtw, world):
    """rtw_render_ex releases the context lock between spp batches with its chunk staged on the device;
    an rtw_render_rows call on the same context in the meantime stages its tile in a buffer of its own
    (ADVICE r4): both give the images they give alone, bit for bit."""
    cam = rtw.book1_camera(image_width=200, aspect_ratio=1.5, spp=8).init()
    W, H = cam.derived.image_width, cam.derived.image_height
    rpb, n, shard = 8, 3, 1
    rows = rtw.lib().rtw_shard_rows(H, rpb, n, shard)

    def ex(buf, rc):
        o = rtw._abi.render_opts(spp_batch=1)
        rc[0] = rtw.lib().rtw_render_ex(world.handle, C.byref(cam.derived), 0, cam.size, 0, 8, 5, buf.ctypes.data,
                                        C.byref(o))

    def rows_call(tile, rc):
        o = rtw._abi.render_opts(spp_batch=1)
        rc[0] = rtw.lib().rtw_render_rows(world.handle, C.byref(cam.derived), rpb, n, shard, 0, 8, 5,
                                          tile.ctypes.data, C.byref(o))

    ref_img, ref_tile = np.zeros((cam.size, 4), np.float32), np.zeros((rows * W, 4), np.float32)
    r1, r2 = [None], [None]
    ex(ref_img, r1)
    rows_call(ref_tile, r2)
    assert r1 == [0] and r2 == [0]
    for _ in range(3):
        img, tile = np.zeros_like(ref_img), np.zeros_like(ref_tile)
        r1, r2 = [None], [None]
        ts = [threading.Thread(target=ex, args=(img, r1)), threading.Thread(target=rows_call, args=(tile, r2))]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=120)
        assert r1 == [0] and r2 == [0]
        assert np.array_equal(img, ref_img)
        assert np.array_equal(tile, ref_tile)
