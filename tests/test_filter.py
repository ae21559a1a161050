"""The walk's sphere fast-reject (sphere_may_hit, rtw_device.h) never rejects a sphere test that Sphere.hit's
exact IEEE arithmetic accepts (objects.zig:127-136: the nearest root in the open interval (0.001, closest)).

The filter runs on the host through rtw_debug_sphere_filter -- the same fp32 operations as the device (FMAs
correctly rounded on both).  The inputs are built to sit on every boundary the derivation
covers: roots within a few ulp of tmin or of closest, tangent rays (disc ~ 0), rays leaving a sphere's
surface (the near-zero root of a large sphere: hb and sqrt(disc) cancelling), huge and tiny direction
lengths (the guard's [2^-40, 2^40] range and beyond), closest = inf, and overflowing squares."""
import numpy as np
import pytest


def run_filter(rtw, a, hb, c, closest):
    a, hb, c, closest = (np.ascontiguousarray(x, np.float32) for x in (a, hb, c, closest))
    n = a.size
    may = np.zeros(n, np.uint8)
    acc = np.zeros(n, np.uint8)
    rc = rtw.lib().rtw_debug_sphere_filter(n, a.ctypes.data, hb.ctypes.data, c.ctypes.data, closest.ctypes.data,
                                           may.ctypes.data, acc.ctypes.data)
    assert rc == 0
    return may.astype(bool), acc.astype(bool)


def check(rtw, a, hb, c, closest):
    may, acc = run_filter(rtw, a, hb, c, closest)
    bad = acc & ~may
    assert not bad.any(), (f"{bad.sum()} exact hits rejected, e.g. a={a[bad][:3]} hb={hb[bad][:3]} c={c[bad][:3]} "
                           f"closest={closest[bad][:3]}")
    return may, acc


def geometric(rng, n, scale_o, scale_d, radius):
    """Random rays and spheres: half_b = dot(oc, d), c = |oc|^2 - r^2, a = |d|^2 in fp32 as the walk computes."""
    oc = (rng.standard_normal((n, 3)) * scale_o).astype(np.float32)
    d = (rng.standard_normal((n, 3)) * scale_d).astype(np.float32)
    r = (rng.random(n) * radius).astype(np.float32)
    a = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
    hb = (oc[:, 0] * d[:, 0] + oc[:, 1] * d[:, 1]) + oc[:, 2] * d[:, 2]
    c = ((oc[:, 0] * oc[:, 0] + oc[:, 1] * oc[:, 1]) + oc[:, 2] * oc[:, 2]) - r * r
    return a.astype(np.float32), hb.astype(np.float32), c.astype(np.float32)


def roots(a, hb, c):
    """The reference's two roots in fp32 (objects.zig:130-136)."""
    disc = (hb * hb - a * c).astype(np.float32)
    with np.errstate(invalid="ignore"):
        sq = np.sqrt(disc).astype(np.float32)
    r1 = ((-hb - sq) / a).astype(np.float32)
    r2 = ((-hb + sq) / a).astype(np.float32)
    return r1, r2


def test_filter_random_scenes(rtw):
    rng = np.random.default_rng(7)
    n = 400_000
    for scale_o, scale_d, radius in ((10, 1, 2), (1000, 1, 1000), (1, 1e-3, 0.5), (50, 30, 5)):
        a, hb, c = geometric(rng, n, scale_o, scale_d, radius)
        closest = np.where(rng.random(n) < 0.3, np.float32(np.inf), (rng.random(n) * 50).astype(np.float32))
        may, acc = check(rtw, a, hb, c, closest)
        assert acc.any() and (~may).any()


@pytest.mark.parametrize("which", ["root1", "root2"])
def test_filter_roots_at_the_interval_ends(rtw, which):
    """closest (or the root against tmin) placed within +-8 ulp of each fp32 root: the comparisons the
    exact test makes at its boundaries."""
    rng = np.random.default_rng(11 if which == "root1" else 12)
    a, hb, c = geometric(rng, 200_000, 5, 1, 3)
    r1, r2 = roots(a, hb, c)
    r = r1 if which == "root1" else r2
    ok = np.isfinite(r) & (r > 0.002)
    a, hb, c, r = a[ok], hb[ok], c[ok], r[ok]
    for k in range(-8, 9):
        closest = (r.view(np.int32) + k).view(np.float32)
        check(rtw, a, hb, c, closest)


def test_filter_roots_at_tmin(rtw):
    """Spheres placed so that a root lands within a few ulp of tmin = 0.001 (camera.zig:187): rays leaving
    the surface they were scattered from, for small and for the r = 1000 ground sphere."""
    rng = np.random.default_rng(5)
    n = 200_000
    for radius in (0.2, 1.0, 1000.0):
        d = rng.standard_normal((n, 3)).astype(np.float32)
        d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
        d *= rng.uniform(0.5, 3, (n, 1)).astype(np.float32)
        center = np.zeros((n, 3), np.float32)
        # origin on the sphere (within rounding), nudged by +-few ulp of tmin along d
        nrm = rng.standard_normal((n, 3)).astype(np.float32)
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True).astype(np.float32)
        t0 = np.float32(0.001) * (1 + rng.integers(-6, 7, n).astype(np.float32) * np.float32(2 ** -23))
        o = (center + nrm * np.float32(radius) - d * t0[:, None]).astype(np.float32)
        oc = (o - center).astype(np.float32)
        a = ((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]).astype(np.float32)
        hb = ((oc[:, 0] * d[:, 0] + oc[:, 1] * d[:, 1]) + oc[:, 2] * d[:, 2]).astype(np.float32)
        c = (((oc[:, 0] * oc[:, 0] + oc[:, 1] * oc[:, 1]) + oc[:, 2] * oc[:, 2]) - np.float32(radius) ** 2).astype(np.float32)
        closest = np.where(rng.random(n) < 0.5, np.float32(np.inf), np.float32(2 * radius + 1))
        may, acc = check(rtw, a, hb, c, closest)
        assert acc.any()


def test_filter_tangent_and_extremes(rtw):
    """disc within ulps of 0 (tangent rays), direction lengths from 2^-60 to 2^60 (outside the guard the
    filter passes every disc >= 0), huge half_b (overflowing squares) and special values."""
    rng = np.random.default_rng(3)
    n = 100_000
    hb = (rng.standard_normal(n) * 10).astype(np.float32)
    a = rng.uniform(0.1, 10, n).astype(np.float32)
    c = ((hb * hb) / a).astype(np.float32)  # disc ~ 0
    c = (c.view(np.int32) + rng.integers(-4, 5, n).astype(np.int32)).view(np.float32)
    closest = (rng.random(n) * 100).astype(np.float32)
    check(rtw, a, hb, c, closest)
    check(rtw, a, -np.abs(hb), c, np.full(n, np.inf, np.float32))
    for e in (-60, -41, -40, -39, 39, 40, 41, 60):
        aa = np.full(n, np.float32(2.0 ** e))
        hb2 = (rng.standard_normal(n) * np.float32(2.0 ** (e / 2))).astype(np.float32)
        c2 = (rng.standard_normal(n) * 4).astype(np.float32)
        check(rtw, aa, hb2, c2, (rng.random(n) * 1e3).astype(np.float32))
    big = np.array([1e15, 1e18, 1e19, 3e19, 1e30, -1e19, -1e30, np.inf, -np.inf, np.nan], np.float32)
    m = big.size
    check(rtw, np.ones(m, np.float32), big, np.full(m, -1.0, np.float32), np.full(m, np.inf, np.float32))
    check(rtw, np.ones(m, np.float32), big, np.full(m, 1e20, np.float32), np.full(m, 5.0, np.float32))
    zero = np.zeros(4, np.float32)
    check(rtw, np.array([0.0, 1e-45, 1.0, 1.0], np.float32), np.array([0.0, -1.0, -0.0, 0.0], np.float32),
          np.array([-1.0, -1.0, -1.0, 0.0], np.float32), zero + np.float32(10.0))


def test_filter_rejects_most_misses(rtw):
    """It is a filter worth running: on random scene rays most exact misses are rejected (the exact path
    then runs for few of them)."""
    rng = np.random.default_rng(9)
    a, hb, c = geometric(rng, 200_000, 10, 1, 1)
    closest = np.full(a.size, np.inf, np.float32)
    may, acc = check(rtw, a, hb, c, closest)
    disc_ok = (hb * hb - a * c) >= 0
    # of the tests with real roots that the exact test rejects (both roots behind tmin), most are filtered
    miss = disc_ok & ~acc
    assert miss.any() and (~may[miss]).mean() > 0.95
