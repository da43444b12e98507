"""Host precompute of the percentile index/weight tables.

The per-site percentile of the reference (tmlib/workflow/corilla/stats.py:76,
``np.percentile(image.array, self._q)``) is numpy 2.2.6's 'linear' method:

    q      = np.true_divide(q_percent, 100)               (percentile)
    vi     = (n - 1) * q                                  (_QuantileMethods['linear'])
    prev   = floor(vi); next = prev + 1                   (_get_indexes)
    prev = next = -1 where vi >= n - 1;  = 0 where vi < 0
    gamma  = vi - prev   (prev after substitution, intp)  (_get_gamma)
    value  = lerp(arr_sorted[prev], arr_sorted[next], gamma)   (_lerp)

These are rounding-sensitive f64 expressions, so they are evaluated here
with numpy itself and handed to the device as integer positions + weights;
the GPU only finds the order statistics and applies ``_lerp``.
"""
from __future__ import annotations

import numpy as np


def quantile_table(n_values: int, q_percent: np.ndarray):
    q = np.true_divide(np.asarray(q_percent, dtype=np.float64), 100)
    vi = (n_values - 1) * q
    prev = np.floor(vi)
    nxt = prev + 1
    above = vi >= n_values - 1
    prev[above] = -1
    nxt[above] = -1
    below = vi < 0
    prev[below] = 0
    nxt[below] = 0
    prev_i = prev.astype(np.intp)
    next_i = nxt.astype(np.intp)
    gamma = np.ascontiguousarray(np.asarray(vi - prev_i, dtype=vi.dtype))
    lo = np.ascontiguousarray(np.where(prev_i < 0, n_values + prev_i, prev_i), dtype=np.int64)
    hi = np.ascontiguousarray(np.where(next_i < 0, n_values + next_i, next_i), dtype=np.int64)
    return lo, hi, gamma


def stats_log10_lut() -> np.ndarray:
    """log10 of every uint16 value as the stats update computes it
    (stats.py:78-85: astype(float) -> np.log10 -> zeros set to 0)."""
    x = np.arange(65536, dtype=np.float64)
    with np.errstate(divide="ignore"):
        lut = np.log10(x)
    lut[0] = 0.0
    return np.ascontiguousarray(lut)
