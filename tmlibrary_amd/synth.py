"""Synthetic site images — the stand-in for imextract output.

``v = 100 + illum(y, x) * LogNormal(6.0, 0.6) + N(0, 5)`` with a per-channel
vignetting field ``illum = exp(-1.5 r^2)``, clipped to [0, 65535], plus 0.01 %
injected zeros and 0.01 % saturated (65535) pixels.  About 6,000 distinct
values per site, which is what the per-site percentile histograms see.

``synth_sites_host`` is numpy (seeded per (seed, channel, site), reproducible
on any host with this numpy); it seeds the small golden fixtures.

``synth_exact_host`` is the host twin of the device generator
(``tmh_synth_sites_device``, csrc/synth_kernels.hip) that ``bench.py`` uses to
fill HBM: a splitmix64 counter hash of (seed, channel, site, pixel) mapped
through integer tables, integer arithmetic only, so both produce the same
pixels bit for bit and the bench's full-size result can be checked against
the CPU oracle (tests/golden/make_bench_fingerprint.py).
"""
from __future__ import annotations

import functools
import math

import numpy as np

STANDARD, BRIGHT, UNIFORM = 0, 1, 2  # TMH_SYNTH_* (include/tmhip.h)
DISTRIBUTIONS = {"synthetic": STANDARD, "bright": BRIGHT, "uniform": UNIFORM}
_TAB = 4096
_M64 = (1 << 64) - 1


def vignette(height: int, width: int) -> np.ndarray:
    y = (np.arange(height, dtype=np.float64) - (height - 1) / 2.0) / max(height / 2.0, 1.0)
    x = (np.arange(width, dtype=np.float64) - (width - 1) / 2.0) / max(width / 2.0, 1.0)
    r2 = (y[:, None] ** 2 + x[None, :] ** 2) / 2.0
    return np.exp(-1.5 * r2)


def synth_site_host(height, width, seed=12345, channel=0, site=0, dtype=np.uint16):
    rng = np.random.default_rng([int(seed), int(channel), int(site)])
    illum = vignette(height, width)
    v = 100.0 + illum * rng.lognormal(6.0, 0.6, size=(height, width)) \
        + rng.normal(0.0, 5.0, size=(height, width))
    top = 255.0 if np.dtype(dtype) == np.uint8 else 65535.0
    if top == 255.0:
        v = v / 16.0
    v = np.clip(np.rint(v), 0.0, top)
    u = rng.random((height, width))
    v[u < 1e-4] = 0.0
    v[u > 1.0 - 1e-4] = top
    return v.astype(dtype)


def synth_sites_host(n_sites, height, width, seed=12345, channel=0, first_site=0,
                     dtype=np.uint16):
    return [synth_site_host(height, width, seed, channel, first_site + i, dtype)
            for i in range(n_sites)]


# ---------------------------------------------------------------------------
# exact twin of the device generator (csrc/synth_kernels.hip)
# ---------------------------------------------------------------------------

_A = (-3.969683028665376e+01, 2.209460984245205e+02, -2.759285104469687e+02,
      1.383577518672690e+02, -3.066479806614716e+01, 2.506628277459239e+00)
_B = (-5.447609879822406e+01, 1.615858368580409e+02, -1.556989798598866e+02,
      6.680131188771972e+01, -1.328068155288572e+01)
_C = (-7.784894002430293e-03, -3.223964580411365e-01, -2.400758277161838e+00,
      -2.549732539343734e+00, 4.374664141464968e+00, 2.938163982698783e+00)
_D = (7.784695709041462e-03, 3.224671290700398e-01, 2.445134137142996e+00,
      3.754408661907416e+00)


def _ndtri(p):
    """Acklam's standard-normal quantile, the same op sequence as the C++."""
    c, d = _C, _D
    if p < 0.02425 or p > 1.0 - 0.02425:
        q = math.sqrt(-2.0 * math.log(p if p < 0.5 else 1.0 - p))
        num = ((((c[0] * q + c[1]) * q + c[2]) * q + c[3]) * q + c[4]) * q + c[5]
        den = (((d[0] * q + d[1]) * q + d[2]) * q + d[3]) * q + 1.0
        return num / den if p < 0.5 else -(num / den)
    a, b = _A, _B
    q = p - 0.5
    r = q * q
    num = (((((a[0] * r + a[1]) * r + a[2]) * r + a[3]) * r + a[4]) * r + a[5]) * q
    den = ((((b[0] * r + b[1]) * r + b[2]) * r + b[3]) * r + b[4]) * r + 1.0
    return num / den


def _axis(n):
    c = (float(n) - 1.0) / 2.0
    h = max(float(n) / 2.0, 1.0)
    out = np.empty(n, dtype=np.int32)
    for i in range(n):
        f = (float(i) - c) / h
        out[i] = math.floor(32768.0 * math.exp(-0.75 * (f * f)) + 0.5)
    return out


@functools.lru_cache(maxsize=16)
def synth_tables(distribution, height, width):
    """(ln16, nz16, ey, ex) int32 tables of the generator (tmh_synth_tables)."""
    mu = 8.5 if distribution == BRIGHT else 6.0
    ln = np.empty(_TAB, dtype=np.int32)
    nz = np.empty(_TAB, dtype=np.int32)
    for i in range(_TAB):
        z = _ndtri((float(i) + 0.5) / float(_TAB))
        e = math.exp(mu + 0.6 * z)
        ln[i] = math.floor(16.0 * e + 0.5)
        nz[i] = math.floor(80.0 * z + 0.5)
    return ln, nz, _axis(int(height)), _axis(int(width))


def _splitmix64_int(x):
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def _splitmix64(x):
    """splitmix64 on a uint64 array (numpy wraps on overflow)."""
    x = x + np.uint64(0x9E3779B97F4A7C15)
    x ^= x >> np.uint64(30)
    x *= np.uint64(0xBF58476D1CE4E5B9)
    x ^= x >> np.uint64(27)
    x *= np.uint64(0x94D049BB133111EB)
    x ^= x >> np.uint64(31)
    return x


def synth_key(seed, channel):
    return ((int(seed) * 0x100000001B3) & _M64) ^ ((int(channel) << 56) & _M64)


def synth_exact_host(height, width, seed=12345, channel=0, site=0, distribution=STANDARD):
    """One site of the device generator, bit for bit (uint16 [height, width])."""
    npx = int(height) * int(width)
    base = synth_key(seed, channel) ^ _splitmix64_int(int(site) & _M64)
    z1 = _splitmix64(np.arange(npx, dtype=np.uint64) ^ np.uint64(base))
    z2 = _splitmix64(z1)
    if distribution == UNIFORM:
        return (z2 >> np.uint64(48)).astype(np.uint16).reshape(height, width)
    ln, nz, ey, ex = synth_tables(distribution, int(height), int(width))
    ill = (ey.astype(np.uint64)[:, None] * ex.astype(np.uint64)[None, :]).ravel()
    prod = (ill * ln.astype(np.uint64)[(z1 >> np.uint64(52)).astype(np.intp)]) >> np.uint64(30)
    v = prod.astype(np.int64) + 1600
    v += nz.astype(np.int64)[((z1 >> np.uint64(40)) & np.uint64(4095)).astype(np.intp)]
    v = (v + 8) >> 4
    np.clip(v, 0, 65535, out=v)
    u3 = (z2 >> np.uint64(40)).astype(np.int64)
    v[u3 < 1678] = 0
    v[u3 >= (1 << 24) - 1678] = 65535
    return v.astype(np.uint16).reshape(height, width)


def synth_exact_sites_host(n_sites, height, width, seed=12345, channel=0, first_site=0,
                           distribution=STANDARD):
    return np.stack([synth_exact_host(height, width, seed, channel, first_site + i, distribution)
                     for i in range(n_sites)])
