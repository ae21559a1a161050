"""The f32 transcendentals of the hot path (objects.zig:109-110 std.math.acos/atan2,
textures.zig:120 @sin, objects.zig:484 @log) as the Zig toolchain computes them:
the product's restatement (csrc/rtw_libm.h, compiled here for the host with the
device's contract-off flags) and the oracle's independent one (oracle/zig_libm.h)
agree bit for bit, and both stay within 1 ulp of the float64 functions.  The
reference holds no vectors for these functions (parity of the algorithm choice is
unpinned); the test pins the two restatements to each other and to
the mathematical functions (acos, atan, sin, log < 1 ulp; atan2 < 2 ulp)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO

HARNESS = r"""
#include <stdint.h>
#include "rtw_libm.h"
void prod_libm(int fn, const float* a, const float* b, float* out, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) {
        switch (fn) {
            case 0: out[i] = rtw_acosf(a[i]); break;
            case 1: out[i] = rtw_atan2f(a[i], b[i]); break;
            case 2: out[i] = rtw_sinf(a[i]); break;
            case 3: out[i] = rtw_logf(a[i]); break;
            default: out[i] = rtw_atanf(a[i]); break;
        }
    }
}
"""


@pytest.fixture(scope="module")
def prod(tmp_path_factory):
    d = tmp_path_factory.mktemp("libm")
    src = d / "h.c"
    src.write_text(HARNESS)
    so = d / "libh.so"
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared", "-Wno-unknown-pragmas",
                           "-I", os.path.join(REPO, "zig-raytracing-weekend_amd", "csrc"), str(src), "-o", str(so)])
    lib = C.CDLL(str(so))
    lib.prod_libm.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
    return lib


def run(lib_fn, fn, a, b=None):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(a if b is None else b, np.float32)
    out = np.empty_like(a)
    lib_fn(fn, a.ctypes.data, b.ctypes.data, out.ctypes.data, a.size)
    return out


def ulp_err(got, exact):
    """|got - exact| in units of the float32 spacing at `exact` (float64 reference)."""
    e32 = exact.astype(np.float32)
    sp = np.spacing(np.abs(e32)).astype(np.float64)
    return np.abs(got.astype(np.float64) - exact) / sp


def inputs(seed=0):
    rng = np.random.default_rng(seed)
    n = 400_000
    specials = np.array([0.0, -0.0, 1.0, -1.0, 0.5, -0.5, 2 ** -26, -(2 ** -26), 2 ** -30, 0.4375, 1.1875, 2.4375,
                         np.pi / 4, 3 * np.pi / 4, 5 * np.pi / 4, 7 * np.pi / 4, 9 * np.pi / 4, 1e-40, 2.0, -2.0,
                         np.inf, -np.inf, np.nan], np.float32)
    return {
        0: np.concatenate([rng.uniform(-1, 1, n), rng.uniform(-1, 1, 1000) ** 9, specials]).astype(np.float32),
        2: np.concatenate([rng.uniform(-6000, 6000, n), rng.uniform(-10, 10, n), specials]).astype(np.float32),
        3: np.concatenate([rng.uniform(0, 1, n), rng.uniform(0, 1e4, 1000), 2.0 ** rng.uniform(-149, 127, 5000),
                           np.abs(specials)]).astype(np.float32),
        4: np.concatenate([rng.standard_normal(n) * 10, np.tan(rng.uniform(-1.57, 1.57, 1000)), specials]
                          ).astype(np.float32),
    }


def test_restatements_bit_identical(prod, oracle):
    ofn = oracle.lib().oracle_libm
    for fn, a in inputs().items():
        p, o = run(prod.prod_libm, fn, a), run(ofn, fn, a)
        assert np.array_equal(p.view(np.uint32), o.view(np.uint32)) or \
            np.array_equal(np.isnan(p), np.isnan(o)) and np.array_equal(p[~np.isnan(p)].view(np.uint32),
                                                                         o[~np.isnan(o)].view(np.uint32)), fn
    rng = np.random.default_rng(1)
    v = rng.standard_normal((300_000, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)   # sphere_uv's arguments: points of the unit sphere
    y, x = (-v[:, 2]).astype(np.float32), v[:, 0].astype(np.float32)
    zs = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf], np.float32)
    y = np.concatenate([y, np.repeat(zs, 6)])
    x = np.concatenate([x, np.tile(zs, 6)])
    p, o = run(prod.prod_libm, 1, y, x), run(ofn, 1, y, x)
    assert np.array_equal(p.view(np.uint32), o.view(np.uint32))


def test_restatements_within_one_ulp(prod):
    ins = inputs(2)
    a = ins[0][np.isfinite(ins[0]) & (np.abs(ins[0]) <= 1)]
    assert ulp_err(run(prod.prod_libm, 0, a), np.arccos(a.astype(np.float64))).max() <= 1.0
    a = ins[2][np.isfinite(ins[2])]
    assert ulp_err(run(prod.prod_libm, 2, a), np.sin(a.astype(np.float64))).max() <= 1.0
    a = ins[3][np.isfinite(ins[3]) & (ins[3] > 0)]
    assert ulp_err(run(prod.prod_libm, 3, a), np.log(a.astype(np.float64))).max() <= 1.0
    a = ins[4][np.isfinite(ins[4])]
    assert ulp_err(run(prod.prod_libm, 4, a), np.arctan(a.astype(np.float64))).max() <= 1.0
    rng = np.random.default_rng(3)
    y, x = rng.standard_normal(200_000).astype(np.float32), rng.standard_normal(200_000).astype(np.float32)
    # atan2f: atanf of the rounded quotient y / x -- musl's documented bound is < 2 ulp (measured 1.45)
    assert ulp_err(run(prod.prod_libm, 1, y, x), np.arctan2(y.astype(np.float64), x.astype(np.float64))).max() < 2.0


def test_special_values(prod):
    f = lambda fn, a, b=None: float(run(prod.prod_libm, fn, np.array([a], np.float32),
                                        None if b is None else np.array([b], np.float32))[0])
    # acos(-1) = 2 * pio2_hi + 0x1p-120 (acos.zig): 0x40490fda, one ulp below float(pi), as Zig returns it
    assert f(0, 1.0) == 0.0 and np.float32(f(0, -1.0)).view(np.uint32) == 0x40490FDA and np.isnan(f(0, 1.5))
    assert f(3, 0.0) == -np.inf and np.isnan(f(3, -1.0)) and f(3, 1.0) == 0.0 and f(3, np.inf) == np.inf
    assert f(1, 0.0, -1.0) == np.float32(np.pi) and f(1, -0.0, -1.0) == -np.float32(np.pi)
    assert f(1, 1.0, 0.0) == np.float32(np.pi / 2) and np.isnan(f(2, np.inf))
    # the UV table of objects.zig:105-107 (the reference's own known answers)
    import math
    for p, uv in (((1, 0, 0), (0.5, 0.5)), ((0, 1, 0), (0.5, 1.0)), ((0, 0, 1), (0.25, 0.5)),
                  ((-1, 0, 0), (0.0, 0.5)), ((0, -1, 0), (0.5, 0.0)), ((0, 0, -1), (0.75, 0.5))):
        theta = f(0, -np.float32(p[1]))  # -p[1] of an f32 vector: -0.0 for 0
        phi = np.float32(f(1, -np.float32(p[2]), p[0])) + np.float32(math.pi)
        got = (float(np.float32(phi) / np.float32(2 * np.float32(math.pi))), float(np.float32(theta) / np.float32(math.pi)))
        assert abs(got[0] - uv[0]) < 1e-6 and abs(got[1] - uv[1]) < 1e-6, (p, got)
