"""Output formats: the reference's two P3 PPM writers
(color.zig:64-69 writeColor, stdout.zig:5-18 printPpmToStdout) and an RGBA8
PNG of the toGamma2 texture, through the C ABI encoders.

Pinning: the header + pixel text layout of the reference's own image2.ppm /
image.ppm (tests/golden/ppm_heads.json, their first 400 bytes), and the sky
rows of those files re-rendered by the oracle and encoded by the library
(+-1 LSB, as tests/test_oracle.py pins the values).
"""
import json
import os
import struct
import zlib

import numpy as np
import pytest

from conftest import GOLDEN


def zig_write_color(acc):
    """color.zig:21-41 toGamma + :68 round(256*g) in f32."""
    g = np.clip(np.sqrt(acc[:, :3] * (np.float32(1) / acc[:, 3:4])), np.float32(0), np.float32(0.999))
    return np.round(np.float32(256) * g)


def parse_ppm(text: bytes):
    head, rest = text.split(b"\n", 3)[:3], text.split(b"\n", 3)[3]
    w, h = map(int, head[1].split())
    vals = np.array(rest.split(), np.int32).reshape(h, w, 3)
    return head, vals


def test_ppm_layout_matches_reference_files(rtw):
    heads = json.load(open(os.path.join(GOLDEN, "ppm_heads.json")))
    acc = np.tile(np.array([[0.75, 0.85, 1.0, 1.0]], np.float32), (400 * 225, 1))
    wc = rtw.output.encode_ppm(acc, 400, 225, rtw._abi.RTW_PPM_WRITECOLOR)
    ref2 = heads["image2.ppm"].encode()
    assert wc[:14] == ref2[:14] == b"P3\n400 225\n255\n"[:14]
    # one "r g b\n" per pixel (writeColor), values up to 256
    assert wc.split(b"\n")[3].count(b" ") == 2 and ref2.split(b"\n")[3].count(b" ") == 2
    acc2 = np.tile(np.array([[0.75, 0.85, 1.0, 1.0]], np.float32), (800 * 450, 1))
    so = rtw.output.encode_ppm(acc2, 800, 450, rtw._abi.RTW_PPM_STDOUT)
    ref1 = heads["image.ppm"].encode()
    assert so.startswith(b"P3\n800 450\n255\n") and ref1.startswith(b"P3\n800 450\n255\n")
    # "r g b\t" per pixel, no newline after the header (stdout.zig:15)
    body, rbody = so.split(b"\n", 3)[3], ref1.split(b"\n", 3)[3]
    assert b"\n" not in body and body.count(b"\t") == 800 * 450
    assert rbody.split(b"\t")[0].count(b" ") == 2


def test_ppm_values_restated(rtw):
    rng = np.random.default_rng(3)
    acc = np.concatenate([rng.random((300, 3), np.float32) * 20, rng.integers(1, 40, (300, 1)).astype(np.float32)], 1)
    acc[:3, :3] = 0
    acc[3:6, :3] = 1e6                       # clamp to 0.999 -> 256 (writeColor) / 255 (stdout)
    _, wc = parse_ppm(rtw.output.encode_ppm(acc, 30, 10, rtw._abi.RTW_PPM_WRITECOLOR))
    assert np.array_equal(wc.reshape(-1, 3), zig_write_color(acc).astype(np.int32))
    assert wc.max() == 256
    g = np.clip(np.sqrt(acc[:, :3] * (np.float32(1) / acc[:, 3:4])), np.float32(0), np.float32(0.999))
    _, so = parse_ppm(rtw.output.encode_ppm(acc, 30, 10, rtw._abi.RTW_PPM_STDOUT))
    assert np.array_equal(so.reshape(-1, 3), np.floor(g * np.float32(255.999)).astype(np.int32))
    with pytest.raises(rtw.RtwError):
        import ctypes as C
        n = C.c_size_t()
        buf = C.create_string_buffer(8)
        rtw._abi.check(rtw.lib().rtw_encode_ppm(acc.ctypes.data, 30, 10, 0, buf, 8, C.byref(n)), "encode")


def test_ppm_sky_rows_vs_reference_image2(rtw, oracle):
    """Oracle-rendered sky of the Book-1 camera (pixel_offset 0, see test_oracle), encoded by
    the library's writeColor PPM: rows 0-13 equal the reference's image2.ppm within 1 LSB."""
    with np.load(os.path.join(GOLDEN, "sky_rows.npz"), allow_pickle=False) as z:
        rows = z["image2_rows"].astype(np.int32)
    sp, mt, tx = oracle.gen_book1(0, 0)
    w = oracle.World(sp, mt, tx)
    cam = oracle.camera(image_width=400, aspect_ratio=16 / 9, samples_per_pixel=16, max_depth=50,
                        background_mode=1, pixel_offset=0)
    acc = w.render_pixels(cam, 0, np.arange(0, 14 * 400, dtype=np.uint32), 0, 16, threads=os.cpu_count() or 1)
    _, got = parse_ppm(rtw.output.encode_ppm(acc, 400, 14, rtw._abi.RTW_PPM_WRITECOLOR))
    assert np.abs(got - rows[:14]).max() <= 1


def read_png(data: bytes):
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, chunks = 8, []
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        typ, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(typ + body) & 0xFFFFFFFF
        chunks.append((typ, body))
        pos += 12 + n
    w, h, depth, ctype = struct.unpack(">IIBB", chunks[0][1][:10])
    raw = zlib.decompress(b"".join(b for t, b in chunks if t == b"IDAT"))
    rows = np.frombuffer(raw, np.uint8).reshape(h, 1 + 4 * w)
    assert (rows[:, 0] == 0).all() and depth == 8 and ctype == 6 and chunks[-1][0] == b"IEND"
    return rows[:, 1:].reshape(h, w, 4)


@pytest.mark.parametrize("w,h", [(1, 1), (37, 11), (300, 300)])   # 300x300: several 64 KiB stored blocks
def test_png_roundtrip(rtw, w, h):
    rgba = np.random.default_rng(w).integers(0, 256, (h, w, 4), dtype=np.uint8)
    assert np.array_equal(read_png(rtw.output.encode_png(rgba, w, h)), rgba)


def test_writer_save_png_and_ppm(rtw, tmp_path):
    wr = rtw.SharedStateImageWriter(8, 4)
    wr.buffer[:, :3] = np.linspace(0, 3, 32, dtype=np.float32)[:, None]
    wr.buffer[:, 3] = 3
    wr.update_texture()
    wr.save_png(str(tmp_path / "a.png"))
    wr.save_ppm(str(tmp_path / "a.ppm"))
    assert np.array_equal(read_png((tmp_path / "a.png").read_bytes()), wr.image())
    _, vals = parse_ppm((tmp_path / "a.ppm").read_bytes())
    assert np.array_equal(vals.reshape(-1, 3), zig_write_color(wr.buffer).astype(np.int32))
