"""Output formats over the C ABI encoders (rtw_output.hip).

* ``encode_ppm(accum, w, h, style)`` -- the reference's two P3 writers:
  ``RTW_PPM_WRITECOLOR`` = color.zig:64-69 (round(256*toGamma), one pixel per
  line; the format of image2.ppm) and ``RTW_PPM_STDOUT`` = stdout.zig:5-18
  (floor(255.999*toGamma), tab-separated; the format of image.ppm).
* ``encode_png(rgba, w, h)`` -- RGBA8 PNG of the SharedStateImageWriter texture
  (the "save to file" TODO of main.zig:47 / README "Output selector").
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi


def _encode(fn, *args) -> bytes:
    n = C.c_size_t()
    _abi.check(fn(*args, None, 0, C.byref(n)), fn.__name__)
    buf = C.create_string_buffer(n.value)
    _abi.check(fn(*args, buf, n.value, C.byref(n)), fn.__name__)
    return buf.raw[:n.value]


def encode_ppm(accum: np.ndarray, width: int, height: int, style: int = _abi.RTW_PPM_WRITECOLOR) -> bytes:
    a = np.ascontiguousarray(accum, np.float32).reshape(-1, 4)
    assert a.shape[0] == width * height
    return _encode(_abi.lib().rtw_encode_ppm, a.ctypes.data, width, height, style)


def encode_png(rgba: np.ndarray, width: int, height: int) -> bytes:
    t = np.ascontiguousarray(rgba, np.uint8).reshape(-1, 4)
    assert t.shape[0] == width * height
    return _encode(_abi.lib().rtw_encode_png, t.ctypes.data, width, height)


def write_ppm(path: str, accum: np.ndarray, width: int, height: int, style: int = _abi.RTW_PPM_WRITECOLOR) -> None:
    with open(path, "wb") as f:
        f.write(encode_ppm(accum, width, height, style))


def write_png(path: str, rgba: np.ndarray, width: int, height: int) -> None:
    with open(path, "wb") as f:
        f.write(encode_png(rgba, width, height))
