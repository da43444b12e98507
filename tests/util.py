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
    """|a-b| in DN, modulo the uint wrap (numpy's astype wraps at 2**bits)."""
    d = np.abs(np.asarray(a, np.int64) - np.asarray(b, np.int64))
    return np.minimum(d, (1 << bits) - d)
