"""The benched configurations at their own batch sizes: the queues bench.py times, checked.

Direction bucketing (rtw_tuning.sort_iters / sort_iters_split) and the dynamic deal only switch on when a
wave's iteration 0 holds >= 192 chunks of 64 paths (rtw_wavefront.hip wf_coherence), so the small-image tests
never reach the stripe capacities, bucket blocks and claim counters of a 72 M - 1 G path batch.  Each test here
renders one BASELINE / SURVEY §8f configuration at its full bench geometry and spp (one wavefront batch, C5 two)
three ways -- product defaults, bucketing off, static deal -- and asserts
  * the three images are bit-identical on the whole frame (camera.zig:93-116: every pixel's samples in order,
    whatever queue a path went through), with w = spp everywhere;
  * the default image matches the oracle (camera.zig:182-208 recursion, bvh.zig:122-136 walk) at 1e-5 relative
    (tests/test_gpu_parity.py's bound; 5e-5 for depth-200 object scenes, test_gpu_objects.py) on 500 random
    pixels.  Object scenes on the SAH tree share quad edges whose exact ties go to whichever leaf the walk tests
    last (objects.zig:242 inclusive): there the oracle bound holds on >= 99 % of pixels, and every pixel of the
    same geometry is held strictly on the reference topology (also rendered at full size, bucketed and not).
"""
import ctypes as C
import dataclasses
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_PIX = 500


def ocamera(oracle, cam):
    kw = {f.name: getattr(cam, f.name) for f in dataclasses.fields(cam) if f.name != "derived"}
    return oracle.camera(**kw)


def render(rtw, arr, cam, tuning, seed=0):
    """The whole frame, samples [0, spp), on a fresh context (its path state freed afterwards)."""
    import torch
    world = rtw.World(arr, tuning=tuning)
    acc = torch.zeros((cam.size, 4), dtype=torch.float32, device="cuda")
    timing = rtw._abi.RtwKernelTiming()
    opts = rtw._abi.RtwRenderOpts(0, 0, None, C.pointer(timing))
    rc = rtw.lib().rtw_render_device(world.handle, C.byref(cam.derived), 0, cam.size, 0, cam.samples_per_pixel,
                                     seed, acc.data_ptr(), None, C.byref(opts))
    rtw._abi.check(rc, "rtw_render_device")
    out = acc.cpu().numpy()
    del acc
    world.close()
    torch.cuda.empty_cache()
    return out, int(timing.launches[rtw._abi.RTW_K_REDUCE])


def close(gpu, ref, rel):
    return np.abs(gpu - ref) <= rel * np.maximum(1.0, np.abs(ref))


def scene(rtw, name, earth_rgba, bvh_mode=None):
    c = rtw.configs.CONFIGS[name]
    if name == "c5":
        objs = rtw.worlds.earth_perlin_world(0, [rtw.Image(earth_rgba)])
    else:
        objs = c.objects()
    arr = rtw.flatten(objs) if bvh_mode is None else rtw.flatten(objs, bvh_mode=bvh_mode)
    return arr, c.camera().init()


NO_SORT = {"sort_iters": 0, "sort_iters_split": 0}
STATIC = {"deal": 0}


def check_three_ways(rtw, arr, cam, batches):
    spp = cam.samples_per_pixel
    ref, nb = render(rtw, arr, cam, None)
    assert nb == batches, f"expected {batches} wavefront batch(es), got {nb}"
    assert np.isfinite(ref).all() and (ref[:, 3] == spp).all()
    for tu in (NO_SORT, STATIC):
        got, _ = render(rtw, arr, cam, tu)
        same = (got == ref).all(axis=1)
        assert same.all(), (tu, int((~same).sum()), np.argwhere(~same)[:5, 0])
    return ref


@pytest.mark.parametrize("name,batches", [("c2", 1), ("c4", 1), ("c5", 2), ("c3", 16)])
def test_sphere_config_full_batch(rtw, oracle, earth_rgba, name, batches):
    """C2 (fused compact-LDS step + LDS tail), C4 (split trace / shade through L1/L2, sort_iters_split, the
    two-wide tail), C5 (fused textured step, every bounce a wavefront iteration) and C3 (BASELINE's 8-GPU frame,
    3840x2160x1024, on one GPU: 16 sample batches of the C2 kernels, each bucketed) at bench size."""
    arr, cam = scene(rtw, name, earth_rgba)
    ref = check_three_ways(rtw, arr, cam, batches)
    pix = np.sort(np.random.default_rng(7).choice(cam.size, N_PIX, replace=False)).astype(np.uint32)
    ow = oracle.World(arr.spheres, arr.materials, arr.textures, arr.perlins, [earth_rgba] if name == "c5" else [])
    want = ow.render_pixels(ocamera(oracle, cam), 0, pix, 0, cam.samples_per_pixel, threads=min(16, os.cpu_count() or 1))
    ok = close(ref[pix, :3], want[:, :3], 1e-5).all(axis=1)
    assert ok.all(), (pix[~ok][:5], np.abs(ref[pix, :3] - want[:, :3]).max())


@pytest.mark.parametrize("name", ["cornell", "cornell_smoke", "simple_light"])
def test_object_config_full_batch(rtw, oracle, earth_rgba, name):
    """Cornell (depth 200, fused LDS step + wf_tail_lds), Cornell smoke (media) at 600x600x200 and simple_light
    (Perlin texture, quad and sphere lights: every feature class) at 800x450x100."""
    arr, cam = scene(rtw, name, earth_rgba)
    ref = check_three_ways(rtw, arr, cam, 1)
    ocam = ocamera(oracle, cam)
    pix = np.sort(np.random.default_rng(8).choice(cam.size, N_PIX, replace=False)).astype(np.uint32)
    th = min(16, os.cpu_count() or 1)
    want = oracle.World.from_arrays(arr).render_pixels(ocam, 0, pix, 0, cam.samples_per_pixel, threads=th)
    ok = close(ref[pix, :3], want[:, :3], 5e-5).all(axis=1)
    assert ok.mean() >= 0.99, (ok.mean(), pix[~ok][:5])
    # the reference topology: no ties move, every pixel strict
    arr_r, _ = scene(rtw, name, earth_rgba, bvh_mode=rtw._abi.RTW_BVH_REFERENCE)
    ref_r = check_three_ways(rtw, arr_r, cam, 1)
    want_r = oracle.World.from_arrays(arr_r).render_pixels(ocam, 0, pix, 0, cam.samples_per_pixel, threads=th)
    ok = close(ref_r[pix, :3], want_r[:, :3], 5e-5).all(axis=1)
    assert ok.all(), (ok.mean(), pix[~ok][:5], np.abs(ref_r[pix, :3] - want_r[:, :3]).max())


def test_textured_small_forced_bucketing(rtw, earth_rgba):
    """The C5 scene class (fused textured step, no tail) on a small image with the benched batches' queues forced
    on (deal bit 128): every iteration bucketed, the split kernels bucketed, the static deal -- one image."""
    arr = rtw.flatten(rtw.worlds.earth_perlin_world(0, [rtw.Image(earth_rgba)]))
    cam = rtw.earth_perlin_camera(image_width=192, spp=6).init()
    outs = []
    for tu in (None, {"deal": 187}, {"deal": 187, "sort_iters": 100}, {"deal": 187, "fuse": 0, "sort_iters_split": 100},
               {"deal": 128, "sort_iters": 100}, {"deal": 187, "wf_iters": 4}, {"deal": 0}):
        w = rtw.World(arr, tuning=tu)
        buf = np.zeros((cam.size, 4), np.float32)
        rtw._abi.check(rtw.lib().rtw_render(w.handle, C.byref(cam.derived), 0, cam.size, 0, 6, 3, buf.ctypes.data, None,
                                            rtw._abi.PROGRESS_FN(0), None), "rtw_render")
        w.close()
        outs.append(buf)
    assert np.isfinite(outs[0]).all() and (outs[0][:, 3] == 6).all()
    for k, o in enumerate(outs[1:], 1):
        assert np.array_equal(outs[0], o), k
