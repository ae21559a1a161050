"""Host-side seeded stream for scene generation.

The reference draws scene and BVH randomness from ``std.crypto.random``
(src/rtweekend.zig:14-27), which cannot be seeded.  This is the same keyed
SplitMix64 stream the device uses (csrc/rtw_rng.h), mapped to f32 like Zig's
``std.Random.float(f32)``.  All float arithmetic that follows a draw is done in
numpy float32 so scene values are bit-identical to a Zig f32 evaluation.
"""
from __future__ import annotations

import struct

import numpy as np

MASK = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15
DOMAIN_RENDER, DOMAIN_SCENE, DOMAIN_BVH, DOMAIN_PERLIN = 0, 1, 2, 3
f32 = np.float32


def mix64(z: int) -> int:
    z &= MASK
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK
    return z ^ (z >> 31)


def _clz64(x: int) -> int:
    return 64 - x.bit_length()


class Stream:
    """rtw_rng_stream(seed, domain, a, b) + rtw_rng_float / rtw_rng_range."""

    def __init__(self, seed: int, domain: int, a: int = 0, b: int = 0):
        k = mix64((seed + domain * GOLDEN) & MASK)
        self.s = mix64(k ^ (((a & 0xFFFFFFFF) << 32) | (b & 0xFFFFFFFF)))

    def next_u64(self) -> int:
        self.s = (self.s + GOLDEN) & MASK
        return mix64(self.s)

    def float(self) -> np.float32:
        """Zig std.Random.float(f32)."""
        x = self.next_u64()
        lz = _clz64(x)
        if lz >= 41:
            lz = 41 + _clz64(self.next_u64())
            if lz == 41 + 64:
                lz += 32 - ((self.next_u64() & 0xFFFFFFFF) | 0x7FF).bit_length()
        bits = ((126 - lz) << 23) | (x & 0x7FFFFF)
        return f32(struct.unpack("<f", struct.pack("<I", bits))[0])

    def path_float(self) -> np.float32:
        """Render-domain draw (rtw_rng.h rtw_path_float): Weyl step, lowbias32 of hi ^ lo, k * 2^-24."""
        self.s = (self.s + GOLDEN) & MASK
        x = ((self.s >> 32) ^ self.s) & 0xFFFFFFFF
        x ^= x >> 16
        x = (x * 0x7FEB352D) & 0xFFFFFFFF
        x ^= x >> 15
        x = (x * 0x846CA68B) & 0xFFFFFFFF
        x ^= x >> 16
        return f32((x >> 8) * 2.0 ** -24)

    def range(self, mn, mx) -> np.float32:
        """rtweekend.randomDoubleRange (src/rtweekend.zig:18-20)."""
        mn, mx = f32(mn), f32(mx)
        return f32(mn + f32(mx - mn) * self.float())

    def int_range(self, mn: int, mx: int) -> int:
        """rtweekend.randomIntRange (src/rtweekend.zig:23-27): round-half-away, up to max+1."""
        v = float(self.range(f32(mn), f32(mx + 1)))
        return int(np.floor(abs(v) + 0.5)) * (1 if v >= 0 else -1)

    def vec(self) -> np.ndarray:
        """vec3.random (src/vec3.zig:47-49)."""
        return np.array([self.float(), self.float(), self.float()], dtype=f32)

    def vec_range(self, mn, mx) -> np.ndarray:
        """vec3.randomRange (src/vec3.zig:51-57)."""
        return np.array([self.range(mn, mx), self.range(mn, mx), self.range(mn, mx)], dtype=f32)
