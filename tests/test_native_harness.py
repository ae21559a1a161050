"""The drop-in driven from a native host the way the reference drives Camera.render: 8 pthreads
(RenderThread + Task, src/main.zig:41,49-69,314-326) calling rtw_render_ex on their chunks with
`running` as a one-byte bool, and a UI thread polling countSamples and clearing `running` mid-render
(main.zig:328-348, 470-514).  tests/native/tasks_harness.c, built by __graft_entry__.build() against
include/rtw_gpu.h and the in-tree librtw_gpu.so.

On a GPU context the 8 Tasks share one context: the library holds its lock only while a Task enqueues
one spp batch, so the Tasks advance samples-outer together (camera.zig:98-111) -- their samples done
differ by at most one batch while they run.  Host contexts (RTW_DEVICE_CPU) render the Tasks
concurrently on host threads (CPU tests)."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO

HARNESS = os.path.join(REPO, "tests", "native", "tasks_harness")
CPU = -1


def write_scene(rtw, path):
    arr = rtw.flatten(rtw.worlds.generate_world(0, "book1"))
    os.makedirs(path, exist_ok=True)
    for name, a in (("spheres", arr.spheres), ("materials", arr.materials), ("textures", arr.textures)):
        with open(os.path.join(path, name + ".bin"), "wb") as f:
            f.write(np.ascontiguousarray(a).tobytes())
    return arr


def run_harness(scene, device, width, spp, batch, mode, out):
    assert os.path.exists(HARNESS), "build it: make -C tests/native (or __graft_entry__.build())"
    r = subprocess.run([HARNESS, str(scene), str(device), str(width), str(spp), str(batch), mode, str(out)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    info = json.loads(r.stdout.strip().splitlines()[-1])
    buf = np.fromfile(out, np.float32).reshape(-1, 4)
    assert buf.shape[0] == info["size"]
    return info, buf


def direct(rtw, arr, device, width, s0, s1, pix0, pix1, buf_init=None):
    """One rtw_render_ex call over [pix0, pix1) x samples [s0, s1) on a fresh context."""
    import ctypes as C
    world = rtw.World(arr, device=device, tuning={"cpu_threads": 1} if device == CPU else None)
    cam = rtw.book1_camera(image_width=width, aspect_ratio=16 / 9, spp=s1, max_depth=50).init()
    buf = np.zeros((cam.size, 4), np.float32) if buf_init is None else buf_init.copy()
    o = rtw._abi.render_opts()
    rtw._abi.check(rtw.lib().rtw_render_ex(world.handle, C.byref(cam.derived), pix0, pix1, s0, s1, 0,
                                           buf.ctypes.data, C.byref(o)), "rtw_render_ex")
    world.close()
    return buf


def check_stopped(rtw, arr, device, width, info, buf):
    """A stopped frame: every Task returned RTW_E_CANCELLED after >= 2 whole batches; each chunk holds
    whole batches (uniform .w, a multiple of the batch), and equals a one-call render of [0, w) of it."""
    chunk, batch = info["chunk"], info["spp_batch"]
    assert all(rc == rtw._abi.RTW_E_CANCELLED for rc in info["rc"]), info
    for k in range(8):
        part = buf[k * chunk:(k + 1) * chunk]
        w = int(part[0, 3])
        assert (part[:, 3] == w).all() and w % batch == 0 and 2 * batch <= w < info["spp"], (k, w, info)
        assert info["samples_done"][k] == w * chunk
        init = np.zeros_like(buf)
        init[:, 3] = 1
        ref = direct(rtw, arr, device, width, 0, w, k * chunk, (k + 1) * chunk, init)
        assert np.array_equal(part, ref[k * chunk:(k + 1) * chunk])


def test_harness_host_backend_full_and_stop(rtw, tmp_path):
    """The native harness on host contexts (no GPU): the full frame equals one rtw_render_ex call bit
    for bit (trailing size % 8 pixels left at scrub's {0,0,0,1}), and a UI stop leaves whole batches."""
    arr = write_scene(rtw, tmp_path / "scene")
    info, buf = run_harness(tmp_path / "scene", CPU, 96, 3, 1, "full", tmp_path / "full.f32")
    chunk = info["chunk"]
    assert info["rc"] == [0] * 8 and info["count_samples"] == pytest.approx(8 * chunk * 3 + (info["size"] - 8 * chunk))
    init = np.zeros_like(buf)
    init[:, 3] = 1
    ref = direct(rtw, arr, CPU, 96, 0, 3, 0, 8 * chunk, init)
    assert np.array_equal(buf, ref)
    info, buf = run_harness(tmp_path / "scene", CPU, 96, 400, 2, "stop", tmp_path / "stop.f32")
    check_stopped(rtw, arr, CPU, 96, info, buf)


@pytest.mark.gpu
def test_harness_c1_eight_tasks_vs_oracle(rtw, oracle, tmp_path):
    """BASELINE config 1 (400x225, 10 spp) through the native 8-Task host on the GPU: every pixel within
    the parity tolerance of the oracle's 8-thread render, w = 10."""
    from test_gpu_parity import close
    arr = write_scene(rtw, tmp_path / "scene")
    info, buf = run_harness(tmp_path / "scene", 0, 400, 10, 2, "full", tmp_path / "c1.f32")
    assert info["rc"] == [0] * 8, info
    ow = oracle.World(arr.spheres, arr.materials, arr.textures)
    ocam = oracle.camera(image_width=400, aspect_ratio=16 / 9, samples_per_pixel=10, max_depth=50, background_mode=1)
    obuf, _ = ow.render_threads(ocam, 0, 8)
    assert close(buf[:, :3], obuf[:, :3]).all(), np.abs(buf[:, :3] - obuf[:, :3]).max()
    assert np.array_equal(buf[:, 3], obuf[:, 3])


@pytest.mark.gpu
def test_harness_tasks_advance_together(rtw, tmp_path):
    """The 8 Tasks on one GPU context advance samples-outer together (camera.zig:98-111): with batches
    long enough that the device, not host-thread wake-ups, paces them (1200x675, 96-sample batches, ~1.2 ms
    each, so a round of the 8 Tasks' batches is ~10 ms: a thread woken late by a loaded host still enqueues its
    next batch within the round; round 6 made the kernels fast enough that 24-sample batches (~0.3 ms) let host
    jitter show), the Tasks' samples done never differ by more than one batch while all of them run, and the
    frame equals one call over the whole chunk range."""
    arr = write_scene(rtw, tmp_path / "scene")
    info, buf = run_harness(tmp_path / "scene", 0, 1200, 768, 96, "full", tmp_path / "big.f32")
    assert info["rc"] == [0] * 8, info
    assert 0 < info["ui_polls"] and info["max_spread_batches"] <= 1.0 + 1e-9, info
    chunk = info["chunk"]
    init = np.zeros_like(buf)
    init[:, 3] = 1
    ref = direct(rtw, arr, 0, 1200, 0, 768, 0, 8 * chunk, init)
    assert np.array_equal(buf, ref)


@pytest.mark.gpu
def test_harness_stop_mid_render_gpu(rtw, tmp_path):
    """The UI clears every RenderThread.running mid-frame (stopRender): each Task returns RTW_E_CANCELLED
    with whole batches in its chunk (bit-identical to rendering [0, w) directly), and while they ran the 8
    Tasks' samples done stayed within one batch of each other (samples-outer, camera.zig:98-111)."""
    arr = write_scene(rtw, tmp_path / "scene")
    info, buf = run_harness(tmp_path / "scene", 0, 400, 400, 4, "stop", tmp_path / "stop.f32")
    check_stopped(rtw, arr, 0, 400, info, buf)
