"""CPU: pin the oracle (and the product's host-side precompute) against the
golden fixtures generated from the reference itself (tests/golden/make_goldens.py)."""
import numpy as np
import pytest
import scipy.ndimage as ndi

from util import load_golden
from oracle import corilla_oracle as orc
from tmlibrary_amd.workflow.corilla.quantiles import quantile_table, stats_log10_lut

STATS_CASES = ["stats_small", "stats_medium", "stats_extremes", "stats_single", "stats_odd",
               "stats_nolog", "stats_dec1", "stats_dec0", "stats_u8"]


@pytest.mark.parametrize("name", STATS_CASES)
def test_oracle_stats_bit_exact(name):
    g = load_golden(name)
    sites = list(g["sites"])
    st = orc.run_illumstats(sites, log_transform=bool(g["log_transform"]),
                            decimals=int(g["decimals"]))
    assert st.n == int(g["n"])
    assert np.array_equal(st.mean, g["mean"], equal_nan=True)
    assert np.array_equal(st.std, g["std"], equal_nan=True)
    assert np.array_equal(st.percentile_sums, g["pct_sums"])
    assert np.array_equal(orc.percentile_values(st.percentile_sums, st.n), g["pct_values"])
    if "pct_keys" in g:
        assert np.array_equal(orc.percentile_keys(int(g["decimals"])), g["pct_keys"])


@pytest.mark.parametrize("name", STATS_CASES)
def test_quantile_table_matches_numpy(name):
    """The product's host precompute (positions + gamma) reproduces np.percentile."""
    g = load_golden(name)
    q = np.linspace(0, 100, 10 ** (int(g["decimals"]) + 2))
    for site in g["sites"]:
        lo, hi, gamma = quantile_table(site.size, q)
        srt = np.sort(site.ravel())
        got = orc.lerp(srt[lo], srt[hi], gamma)
        assert np.array_equal(got, np.percentile(site, q))


@pytest.mark.parametrize("n", [1, 2, 3, 7, 64, 5120, 100001])
def test_percentile_restatement_edge_sizes(n):
    rng = np.random.default_rng(n)
    a = rng.integers(0, 65536, size=n, dtype=np.uint16)
    q = np.linspace(0, 100, 100000)
    assert np.array_equal(orc.percentile_linear(a, q), np.percentile(a, q))
    lo, hi, gamma = quantile_table(n, q)
    olo, ohi, og = orc.quantile_table(n, q)
    assert np.array_equal(lo, olo) and np.array_equal(hi, ohi) and np.array_equal(gamma, og)
    assert lo.min() >= 0 and hi.max() <= n - 1 and np.all(np.diff(lo) >= 0)


def test_stats_lut_matches_reference_transform():
    lut = stats_log10_lut()
    x = np.arange(65536, dtype=np.float64)
    with np.errstate(divide="ignore"):
        want = np.log10(x)
    want[0] = 0
    assert np.array_equal(lut, want)


@pytest.mark.parametrize("name", ["apply_log", "apply_nolog"])
def test_oracle_apply_bit_exact(name):
    g = load_golden(name)
    log = name == "apply_log"
    got = np.stack([orc.correct_illumination(t, g["smooth_mean"], g["smooth_std"], log)
                    for t in g["images"]])
    assert np.array_equal(got, g["corrected"])
    clipped = np.stack([orc.clip(c, int(g["clip_lo"]), int(g["clip_hi"])) for c in got])
    assert np.array_equal(clipped, g["clipped"])


def test_oracle_apply_u8():
    g = load_golden("apply_u8")
    got = orc.correct_illumination(g["images"][0], g["smooth_mean"], g["smooth_std"])
    assert np.array_equal(got, g["corrected"][0])


def test_cast_rule():
    g = load_golden("cast_rule")
    assert np.array_equal(orc.cast_float_to_uint_x86(g["values"], np.uint16), g["as_u16"])
    assert np.array_equal(orc.cast_float_to_uint_x86(g["values"], np.uint8), g["as_u8"])


@pytest.mark.parametrize("name", ["apply_log", "apply_nolog"])
def test_smoothing_vs_scipy(name):
    """Parity vs mahotas is unpinned (absent); pinned vs scipy reflect."""
    g = load_golden(name)
    for src, sm in (("stats_mean", "smooth_mean"), ("stats_std", "smooth_std")):
        got = orc.smooth_reflect(g[src], 5)
        assert np.allclose(got, g[sm], rtol=1e-12, atol=1e-14)
        ref = ndi.gaussian_filter(g[src], 5, mode="reflect", truncate=4.0)
        assert np.allclose(got, ref, rtol=1e-12, atol=1e-14)


def test_smoothing_tiny_planes_reflect_wraps():
    rng = np.random.default_rng(3)
    for shape in [(1, 1), (3, 5), (7, 41), (50, 2)]:
        a = rng.random(shape)
        assert np.allclose(orc.smooth_reflect(a, 5),
                           ndi.gaussian_filter(a, 5, mode="reflect", truncate=4.0),
                           rtol=1e-12, atol=1e-14)


def test_closest_percentile():
    g = load_golden("stats_small")
    pct = dict(zip(g["pct_keys"].tolist(), g["pct_values"].tolist()))
    assert orc.get_closest_percentile(pct, 0.001) == pct[0.001]
    assert orc.get_closest_percentile(pct, 99.9) == pct[99.9]
    assert orc.get_closest_percentile(pct, 99.90049) == pct[99.9]


def test_fullsize_inputs_reproducible():
    """The host generator still produces the sites the full-size goldens were made from."""
    import hashlib

    from tmlibrary_amd.synth import synth_sites_host
    g = load_golden("fullsize_2site")
    sites = synth_sites_host(int(g["n_sites"]), int(g["height"]), int(g["width"]),
                             seed=int(g["seed"]))
    for s, d in zip(sites, g["input_digest"]):
        assert hashlib.sha256(np.ascontiguousarray(s).tobytes()).hexdigest() == str(d)


def test_numpy_percentile_mode_matches_cdf_mode():
    """The CPU-baseline mode (np.percentile, stats.py:76 as written) and the
    histogram/CDF restatement give identical sums."""
    rng = np.random.default_rng(3)
    sites = [rng.integers(0, 4000, size=(48, 64), dtype=np.uint16) for _ in range(3)]
    a = orc.OracleOnlineStatistics((48, 64), percentile="numpy")
    b = orc.OracleOnlineStatistics((48, 64))
    for s in sites:
        a.update(s)
        b.update(s)
    assert np.array_equal(a.percentile_sums, b.percentile_sums)
    assert np.array_equal(a.mean, b.mean) and np.array_equal(a.std, b.std)
