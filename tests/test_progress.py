"""Progressive / resumable renders and the UI progress contract:
countSamples (src/main.zig:470-477), POWER (:495-503) inputs, checkpoint files.
CPU: encoding and validation; the render-side identities are in the GPU tests below."""
import ctypes as C
import os

import numpy as np
import pytest


def test_count_samples_is_sequential_f32(rtw):
    rng = np.random.default_rng(0)
    acc = np.zeros((100_000, 4), np.float32)
    acc[:, 3] = rng.integers(1, 500, 100_000).astype(np.float32)
    got = rtw.lib().rtw_count_samples(acc.ctypes.data, 100_000)
    want = np.add.accumulate(acc[:, 3], dtype=np.float32)[-1]     # f32, index order
    assert np.float32(got) == want


def make_ckpt(rtw, path, seed=7, spp_done=3, world=None):
    cam = rtw.book1_camera(image_width=40, aspect_ratio=2.0, spp=8).init()
    acc = np.random.default_rng(1).random((cam.size, 4)).astype(np.float32)
    rc = rtw.lib().rtw_checkpoint_write(str(path).encode(), C.byref(cam.derived), seed, 1234, spp_done,
                                        acc.ctypes.data)
    rtw._abi.check(rc, "write")
    return cam, acc


def test_checkpoint_roundtrip_and_validation(rtw, tmp_path):
    p = tmp_path / "a.ckpt"
    cam, acc = make_ckpt(rtw, p)
    back = np.zeros_like(acc)
    c2 = rtw._abi.RtwCamera()
    seed, h, done = C.c_uint64(), C.c_uint64(), C.c_uint32()
    rtw._abi.check(rtw.lib().rtw_checkpoint_read(str(p).encode(), C.byref(c2), C.byref(seed), C.byref(h),
                                                 C.byref(done), back.ctypes.data, cam.size), "read")
    assert np.array_equal(back, acc) and bytes(c2) == bytes(cam.derived)
    assert (seed.value, h.value, done.value) == (7, 1234, 3)
    # wrong capacity, truncation and a flipped bit are refused
    small = np.zeros((cam.size - 1, 4), np.float32)
    assert rtw.lib().rtw_checkpoint_read(str(p).encode(), None, None, None, None, small.ctypes.data,
                                         cam.size - 1) == rtw._abi.RTW_E_INVALID
    raw = bytearray(p.read_bytes())
    (tmp_path / "t.ckpt").write_bytes(raw[:-10])
    raw[100] ^= 1
    (tmp_path / "f.ckpt").write_bytes(raw)
    for name in ("t.ckpt", "f.ckpt", "missing.ckpt"):
        assert rtw.lib().rtw_checkpoint_read(str(tmp_path / name).encode(), None, None, None, None,
                                             back.ctypes.data, cam.size) == rtw._abi.RTW_E_INVALID
