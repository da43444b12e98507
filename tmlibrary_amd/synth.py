"""Synthetic site images — the stand-in for imextract output.

``v = 100 + illum(y, x) * LogNormal(6.0, 0.6) + N(0, 5)`` with a per-channel
vignetting field ``illum = exp(-1.5 r^2)``, clipped to [0, 65535], plus 0.01 %
injected zeros and 0.01 % saturated (65535) pixels.  About 6,000 distinct
values per site, which is what the per-site percentile histograms see.

``synth_sites_host`` is numpy (seeded per (seed, channel, site), reproducible
on any host with this numpy); the device generator used by ``bench.py`` lives
in the HIP library (``tmh_synth_sites``) and draws the same distribution from
a counter-based hash, so large configs are generated in HBM directly.
"""
from __future__ import annotations

import numpy as np


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
