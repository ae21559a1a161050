"""Multi-GPU frame through the C ABI (rtw_multi_*: shard renders + grouped RCCL
send/recv to device 0), against rtw_render_device on one context: bit-identical
for every visible device count (the box has 1: the RCCL communicator, the
self send/recv of the scatter and the gather, the pack/unpack kernels all run).
Reference: startRender's split of Camera.render (src/main.zig:314-326,
src/camera.zig:93-116)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _device_render(rtw, world, cam, s0, s1, seed, buf):
    rc = rtw.lib().rtw_render_device(world.handle, C.byref(cam.derived), 0, cam.size, s0, s1, seed, buf.data_ptr(),
                                     None, None)
    rtw._abi.check(rc, "rtw_render_device")


@pytest.fixture(scope="module")
def setup(rtw):
    import torch
    n = max(1, min(8, torch.cuda.device_count()))
    arr = rtw.flatten(rtw.worlds.generate_world(0, "book1"))
    worlds = [rtw.World(arr, device=k) for k in range(n)]
    yield arr, worlds
    for w in worlds:
        w.close()


@pytest.mark.parametrize("rpb", [8, 3, 8 | 0x80000000])
def test_multi_device_bit_identical(rtw, setup, rpb):
    import torch
    arr, worlds = setup
    cam = rtw.book1_camera(image_width=400, aspect_ratio=1.5, spp=6).init()
    one = torch.zeros((cam.size, 4), dtype=torch.float32, device="cuda:0")
    _device_render(rtw, worlds[0], cam, 0, 6, 17, one)
    m = rtw.distributed.MultiDeviceRender(worlds, rows_per_block=rpb)
    frame = torch.full((cam.size, 4), 123.0, dtype=torch.float32, device="cuda:0")
    m.render_device(cam, 0, 4, frame.data_ptr(), seed=17, fresh=True)   # ignores the 123s
    m.render_device(cam, 4, 6, frame.data_ptr(), seed=17)               # accumulates onto the frame
    m.close()
    torch.cuda.synchronize()
    assert torch.equal(one, frame)


def test_multi_host_progressive_matches_single(rtw, setup):
    """Host API: a progressive split [0,2) + [2,5) onto a host buffer == one 5-spp
    rtw_render of the same frame (rgb += in sample order, w = spp_end)."""
    arr, worlds = setup
    cam = rtw.book1_camera(image_width=240, aspect_ratio=16 / 9, spp=5).init()
    ref = np.zeros((cam.size, 4), np.float32)
    rc = rtw.lib().rtw_render(worlds[0].handle, C.byref(cam.derived), 0, cam.size, 0, 5, 3, ref.ctypes.data,
                              None, rtw._abi.PROGRESS_FN(), None)
    rtw._abi.check(rc, "rtw_render")
    m = rtw.distributed.MultiDeviceRender(worlds, rows_per_block=8)
    got = np.zeros((cam.size, 4), np.float32)
    m.render_host(cam, 0, 2, got, seed=3)
    m.render_host(cam, 2, 5, got, seed=3)
    m.close()
    assert np.array_equal(ref, got)
    assert (got[:, 3] == 5).all()


def test_multi_c3_geometry_rows(rtw, setup):
    """BASELINE config 3 geometry (3840x2160, 8-row blocks) at 1 spp: the frame through
    the multi-device path equals the single-context render."""
    import torch
    arr, worlds = setup
    cam = rtw.book1_camera(image_width=3840, aspect_ratio=16 / 9, spp=1).init()
    assert cam.derived.image_height == 2160
    one = torch.zeros((cam.size, 4), dtype=torch.float32, device="cuda:0")
    _device_render(rtw, worlds[0], cam, 0, 1, 0, one)
    m = rtw.distributed.MultiDeviceRender(worlds, rows_per_block=8)
    frame = torch.zeros_like(one)
    m.render_device(cam, 0, 1, frame.data_ptr(), seed=0, fresh=True)
    m.close()
    torch.cuda.synchronize()
    assert torch.equal(one, frame)
