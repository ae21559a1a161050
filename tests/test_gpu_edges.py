"""GPU edge cases of the drop-in boundary against the C oracle: path depth 0 and 1
(rayColor's `depth <= 0` and single-bounce cases, camera.zig:182-208), tiny and
odd image sizes (8x8 wavefront tiles padded at the borders), ragged pixel ranges
(Camera.render over [pix_begin, pix_end), camera.zig:93-116), and empty pixel or
sample ranges (the caller's buffer untouched).  Same tolerance as
test_gpu_parity.py (1e-5 relative per channel)."""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REL = 1e-5


@pytest.fixture(scope="module")
def world(rtw):
    arr = rtw.flatten(rtw.worlds.generate_world(0, "book1"))
    w = rtw.World(arr)
    yield w
    w.close()


@pytest.fixture(scope="module")
def oworld(oracle):
    sp, mt, tx = oracle.gen_book1(0, 0)
    return oracle.World(sp, mt, tx)


def cams(rtw, oracle, width, aspect, spp, depth):
    cam = rtw.book1_camera(image_width=width, aspect_ratio=aspect, spp=spp, max_depth=depth).init()
    ocam = oracle.camera(image_width=width, aspect_ratio=aspect, samples_per_pixel=spp, max_depth=depth,
                         background_mode=1)
    assert cam.derived.image_height == ocam.image_height
    return cam, ocam


def render(rtw, world, cam, p0, p1, s0, s1, seed, buf=None):
    if buf is None:
        buf = np.zeros((cam.size, 4), np.float32)
    rc = rtw.lib().rtw_render(world.handle, C.byref(cam.derived), p0, p1, s0, s1, seed, buf.ctypes.data, None,
                              rtw._abi.PROGRESS_FN(0), None)
    rtw._abi.check(rc, "rtw_render")
    return buf


def oracle_pixels(oworld, ocam, seed, pix, s0, s1):
    return oworld.render_pixels(ocam, seed, np.asarray(pix, dtype=np.uint32), s0, s1, threads=os.cpu_count() or 1)


def close(a, b):
    return np.abs(a - b) <= REL * np.maximum(1.0, np.abs(b))


@pytest.mark.parametrize("depth", [0, 1, 2])
def test_shallow_depths(rtw, oracle, world, oworld, depth):
    """max_depth 0: every sample is black (rayColor returns 0 at depth <= 0); 1 and 2:
    the first bounces only -- still the oracle's values and w = samples."""
    cam, ocam = cams(rtw, oracle, 96, 1.5, 5, depth)
    got = render(rtw, world, cam, 0, cam.size, 0, 5, 3)
    ref = oracle_pixels(oworld, ocam, 3, np.arange(cam.size), 0, 5)
    assert (got[:, 3] == 5).all()
    if depth == 0:
        assert (got[:, :3] == 0).all()
    assert close(got[:, :3], ref[:, :3]).all()


@pytest.mark.parametrize("width,aspect", [(1, 1.0), (7, 1.0), (9, 3.0), (33, 0.5)])
def test_tiny_and_odd_images(rtw, oracle, world, oworld, width, aspect):
    """Images smaller than or not a multiple of the 8x8 wavefront tile."""
    cam, ocam = cams(rtw, oracle, width, aspect, 6, 50)
    got = render(rtw, world, cam, 0, cam.size, 0, 6, 5)
    ref = oracle_pixels(oworld, ocam, 5, np.arange(cam.size), 0, 6)
    assert (got[:, 3] == 6).all()
    assert close(got[:, :3], ref[:, :3]).all()


def test_ragged_pixel_range(rtw, oracle, world, oworld):
    """[pix_begin, pix_end) cutting rows and tiles: those pixels match the oracle, every
    other pixel of the caller's buffer keeps its contents."""
    cam, ocam = cams(rtw, oracle, 101, 1.5, 4, 50)
    buf = np.full((cam.size, 4), 7.0, np.float32)
    p0, p1 = 137, 3001
    got = render(rtw, world, cam, p0, p1, 0, 4, 9, buf)
    ref = oracle_pixels(oworld, ocam, 9, np.arange(p0, p1), 0, 4)
    assert close(got[p0:p1, :3], ref[:, :3] + 7.0).all()  # rgb += the samples (camera.zig:55)
    assert (got[p0:p1, 3] == 4).all()  # w = number of samples (camera.zig:56)
    assert (got[:p0] == 7.0).all() and (got[p1:] == 7.0).all()


@pytest.mark.parametrize("p0,p1,s0,s1", [(500, 500, 0, 4), (0, 900, 3, 3)])
def test_empty_ranges_leave_the_buffer(rtw, oracle, world, p0, p1, s0, s1):
    cam = rtw.book1_camera(image_width=60, aspect_ratio=1.5, spp=4).init()
    buf = np.full((cam.size, 4), 2.5, np.float32)
    got = render(rtw, world, cam, p0, p1, s0, s1, 1, buf.copy())
    assert np.array_equal(got, buf)


def test_depth0_after_a_deep_render_on_the_same_context(rtw, world):
    """The path-state buffer is reused across renders of one context: a depth-0 render
    after a depth-50 render (same size, the fused single-batch path) must still add zeros
    (rayColor(r, 0) = 0, camera.zig:183-185), not the previous render's radiance."""
    deep = rtw.book1_camera(image_width=120, aspect_ratio=1.5, spp=6, max_depth=50).init()
    got = render(rtw, world, deep, 0, deep.size, 0, 6, 2)
    assert got[:, :3].max() > 0
    flat = rtw.book1_camera(image_width=120, aspect_ratio=1.5, spp=6, max_depth=0).init()
    got0 = render(rtw, world, flat, 0, flat.size, 0, 6, 2)
    assert (got0[:, :3] == 0).all() and (got0[:, 3] == 6).all()
