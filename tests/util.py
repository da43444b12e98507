"""Shared test helpers (fixture loading, tolerance checks)."""
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def assert_close_rel(got, want, rtol=1e-6, atol=1e-9):
    """north_star tolerance for mean/std: 1e-6 relative, with an absolute floor
    where the value is ~0 (pixels that are 0/1 in every site have mean 0)."""
    got = np.asarray(got)
    want = np.asarray(want)
    assert got.shape == want.shape
    nan_g, nan_w = np.isnan(got), np.isnan(want)
    assert np.array_equal(nan_g, nan_w), "NaN pattern differs"
    ok = ~nan_w
    err = np.abs(got[ok] - want[ok])
    lim = atol + rtol * np.abs(want[ok])
    assert np.all(err <= lim), "max rel err %.3g" % float(np.max(err / np.maximum(np.abs(want[ok]), 1e-300)))


def dn_diff(a, b, bits=16):
    """|a - b| in DN, NOT modulo the uint wrap: a corrected pixel that lands on
    the other side of 2**bits from the reference counts as a large difference
    here (see wrap_flips)."""
    return np.abs(np.asarray(a, np.int64) - np.asarray(b, np.int64))


def wrap_flips(a, b, bits=16):
    """Pixels whose values differ by 1 only modulo 2**bits (e.g. 65535 vs 0:
    the f32 result and the reference's f64 result fell on opposite sides of a
    2**16 boundary before numpy's wrapping astype)."""
    d = dn_diff(a, b, bits)
    return int(np.count_nonzero(d == (1 << bits) - 1))


def dn_report(a, b, bits=16):
    """(max |d| over non-flipped pixels, wrap flips, pixels at +-1 DN)."""
    d = dn_diff(a, b, bits)
    flips = d == (1 << bits) - 1
    rest = d[~flips]
    return (int(rest.max()) if rest.size else 0, int(np.count_nonzero(flips)),
            int(np.count_nonzero(rest == 1)))


def assert_dn(a, b, bits=16, max_flips=0, tol=1):
    """Corrected values within +-tol DN (non-modular), at most max_flips wrap flips."""
    worst, flips, _ = dn_report(a, b, bits)
    assert worst <= tol, "corrected values differ by %d DN" % worst
    assert flips <= max_flips, "%d wrap flips (limit %d)" % (flips, max_flips)
