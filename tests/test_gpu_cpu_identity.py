"""The host backend (RTW_DEVICE_CPU, csrc/rtw_cpu.hip) and the GPU render the same image bit
for bit: both run sample_radiance's fp32 operations (the GPU's fast box / sphere filters and
compact nodes are exact), on Book-1 (C2 camera), HEAD's textured moving
spheres, Cornell box and Cornell smoke."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def render(rtw, arr, cam, spp, seed, device):
    world = rtw.World(arr, device=device)
    buf = np.zeros((cam.size, 4), np.float32)
    rc = rtw.lib().rtw_render(world.handle, C.byref(cam.derived), 0, cam.size, 0, spp, seed, buf.ctypes.data, None,
                              rtw._abi.PROGRESS_FN(0), None)
    rtw._abi.check(rc, "rtw_render")
    world.close()
    return buf


@pytest.mark.parametrize("scene", ["book1", "ref_head", "cornell", "cornell_smoke"])
def test_host_backend_bit_identical_to_gpu(rtw, earth_rgba, scene):
    if scene in ("book1", "ref_head"):
        arr = rtw.flatten(rtw.worlds.generate_world(0, scene, [rtw.Image(earth_rgba)]))
        cam = rtw.book1_camera(image_width=240, aspect_ratio=1.5, spp=4).init()
    else:
        arr = rtw.flatten(rtw.worlds.cornell_box() if scene == "cornell" else rtw.worlds.cornell_smoke())
        cam = rtw.Camera(image_width=96, samples_per_pixel=4, max_depth=50, aspect_ratio=1.0, vfov=40.0,
                         lookfrom=(278.0, 278.0, -800.0), lookat=(278.0, 278.0, 0.0), defocus_angle=0.0).init()
    gpu = render(rtw, arr, cam, 4, 9, 0)
    cpu = render(rtw, arr, cam, 4, 9, rtw._abi.RTW_DEVICE_CPU)
    assert np.array_equal(gpu, cpu), (np.abs(gpu - cpu).max(), (gpu != cpu).any(axis=1).mean())
