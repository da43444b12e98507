"""GPU parity: the HIP path (through the C-ABI) vs the oracle and the golden
fixtures.  Bars (BASELINE.json north_star): mean/std 1e-6 relative,
percentiles and histograms bit-exact, corrected uint16 within +-1 DN."""
import ctypes as C
import hashlib

import numpy as np
import pytest

from util import assert_close_rel, assert_dn, dn_report, load_golden
from oracle import corilla_oracle as orc

pytestmark = pytest.mark.gpu

STATS_CASES = ["stats_small", "stats_medium", "stats_extremes", "stats_single", "stats_odd",
               "stats_nolog", "stats_dec1", "stats_dec0", "stats_u8"]


@pytest.fixture(scope="module")
def L():
    from tmlibrary_amd import hip
    return hip.lib()


class Dev:
    """Raw device buffer via the C-ABI helpers (no torch needed)."""

    def __init__(self, L, nbytes):
        self.L = L
        self.p = C.c_void_p()
        assert L.tmh_malloc_device(C.byref(self.p), max(int(nbytes), 1)) == 0
        self.nbytes = nbytes

    def put(self, a):
        a = np.ascontiguousarray(a)
        assert self.L.tmh_memcpy(self.p, a.ctypes.data, a.nbytes, 0, None) == 0

    def get(self, dtype, shape):
        out = np.empty(shape, dtype)
        assert self.L.tmh_memcpy(out.ctypes.data, self.p, out.nbytes, 1, None) == 0
        return out

    def free(self):
        self.L.tmh_free_device(self.p)


def site_order_stats(L, h, sites, Q):
    """(previous, next) order statistics of the given sites of the handle's
    last batch, decoded from the device's (compact or dense) storage."""
    from tmlibrary_amd import hip
    res = []
    for i in sites:
        a, b = np.empty(Q, np.uint16), np.empty(Q, np.uint16)
        hip.check(L.tmh_stats_site_order_stats(h, i, hip.ptr(a), hip.ptr(b)))
        res.append((a, b))
    return res


def check_order_stats(sites, got, q=None):
    """Every site's (previous, next) order statistics equal the oracle's
    (numpy 'linear' positions read off the exact CDF)."""
    q = np.linspace(0, 100, 100000) if q is None else q
    lo, hi, _ = orc.quantile_table(sites[0].size, q)
    for i, (s, (a, b)) in enumerate(zip(sites, got)):
        hs = orc.histogram_u16(s)
        assert np.array_equal(a, orc.order_statistics_from_hist(hs, lo)), "site %d previous" % i
        assert np.array_equal(b, orc.order_statistics_from_hist(hs, hi)), "site %d next" % i


def run_stats(sites, log=True, decimals=3, batch=3, flags=0):
    from tmlibrary_amd.image import ChannelImage
    from tmlibrary_amd.workflow.corilla.stats import OnlineStatistics
    st = OnlineStatistics(sites[0].shape, decimals=decimals, batch_size=batch, flags=flags)
    for s in sites:
        st.update(ChannelImage(np.ascontiguousarray(s)), log_transform=log)
    return st


@pytest.mark.parametrize("name", STATS_CASES)
@pytest.mark.parametrize("batch", [1, 3, 64])
def test_stats_vs_golden(L, name, batch):
    g = load_golden(name)
    st = run_stats(list(g["sites"]), bool(g["log_transform"]), int(g["decimals"]), batch)
    assert st.n == int(g["n"])
    assert_close_rel(st.mean.array, g["mean"])
    assert_close_rel(st.std.array, g["std"])
    assert np.array_equal(st.percentile_sums, g["pct_sums"]), "percentile sums not bit-exact"
    pct = st.percentiles
    vals = np.array([pct[k] for k in sorted(pct)], dtype=np.int64)
    assert np.array_equal(vals, g["pct_values"])
    if "pct_keys" in g:
        assert np.array_equal(np.array(sorted(pct), dtype=np.float64), g["pct_keys"])
    pooled = sum(orc.histogram_u16(s) for s in g["sites"])
    assert np.array_equal(st.histogram, pooled), "pooled histogram not bit-exact"


def test_site_histograms_bit_exact(L):
    from tmlibrary_amd import hip
    g = load_golden("stats_extremes")
    sites = list(g["sites"])
    st = run_stats(sites, batch=64, flags=hip.TMH_STATS_KEEP_SITE_HIST)
    st._finalize()
    for i, s in enumerate(sites):
        h = np.empty(65536, np.uint32)
        hip.check(L.tmh_stats_site_histogram(st._h, i, hip.ptr(h)))
        assert np.array_equal(h.astype(np.uint64), orc.histogram_u16(s))


@pytest.mark.parametrize("kind", ["constant_low", "constant_high", "uniform", "two_values",
                                  "all_max", "sparse_hi"])
def test_histogram_stress(L, kind):
    """Worst cases for the LDS/global histogram split: every pixel in one bin
    (below and above the LDS range), uniform over all 65,536 values."""
    rng = np.random.default_rng(11)
    h, w = 512, 640
    if kind == "constant_low":
        sites = [np.full((h, w), 123, np.uint16) for _ in range(3)]
    elif kind == "constant_high":
        sites = [np.full((h, w), 50000, np.uint16) for _ in range(3)]
    elif kind == "uniform":
        sites = [rng.integers(0, 65536, (h, w), dtype=np.uint16) for _ in range(3)]
    elif kind == "two_values":
        sites = [np.where(rng.random((h, w)) < 0.5, 1, 65534).astype(np.uint16) for _ in range(3)]
    elif kind == "all_max":
        sites = [np.full((h, w), 65535, np.uint16) for _ in range(2)]
    else:
        base = rng.integers(90, 4000, (h, w), dtype=np.uint16)
        base[rng.random((h, w)) < 1e-3] = 65535
        base[rng.random((h, w)) < 1e-3] = 40000
        sites = [base, base[::-1].copy(), base[:, ::-1].copy()]
    st = run_stats(sites, batch=2)
    ref = orc.run_illumstats(sites)
    assert np.array_equal(st.percentile_sums, ref.percentile_sums)
    assert np.array_equal(st.histogram, sum(orc.histogram_u16(s) for s in sites))
    assert_close_rel(st.mean.array, ref.mean)
    assert_close_rel(st.std.array, ref.std)


def test_repeatable_bitwise(L):
    """Percentiles and histograms do not depend on how sites are batched
    (bit-exact); mean/std are merged per launch (shifted sums + Chan), so
    batching moves them only in the last bits, and a rerun is bit-identical."""
    sites = list(load_golden("stats_medium")["sites"])
    a = run_stats(sites, batch=2)
    b = run_stats(sites, batch=4)
    c = run_stats(sites, batch=4)
    assert np.array_equal(a.percentile_sums, b.percentile_sums)
    assert np.array_equal(a.histogram, b.histogram)
    assert np.allclose(a.std.array, b.std.array, rtol=1e-12, atol=1e-15)
    assert np.allclose(a.mean.array, b.mean.array, rtol=1e-13, atol=1e-15)
    assert np.array_equal(b.std.array, c.std.array)
    assert np.array_equal(b.mean.array, c.mean.array)


def test_log_transform_switch_and_zero_warning(L, caplog):
    sites = list(load_golden("stats_small")["sites"])
    from tmlibrary_amd.image import ChannelImage
    from tmlibrary_amd.workflow.corilla.stats import OnlineStatistics
    st = OnlineStatistics(sites[0].shape, batch_size=4)
    ref = orc.OracleOnlineStatistics(sites[0].shape)
    logs = [True, False, True, True, False]
    with caplog.at_level("WARNING"):
        for s, lg in zip(sites, logs):
            st.update(ChannelImage(s), log_transform=lg)
            ref.update(s, log_transform=lg)
        _ = st.mean
    assert_close_rel(st.mean.array, ref.mean)
    assert_close_rel(st.std.array, ref.std)
    assert np.array_equal(st.percentile_sums, ref.percentile_sums)
    n_warn = sum("image contains zero values" in r.message for r in caplog.records)
    assert n_warn == ref.zero_sites


def test_empty_stats_behaviour(L):
    from tmlibrary_amd.workflow.corilla.stats import OnlineStatistics
    st = OnlineStatistics((8, 8))
    assert st.n == 0
    assert np.all(np.isnan(st.var)) and np.all(np.isnan(st.std.array))
    assert np.array_equal(st.mean.array, np.zeros((8, 8)))
    with pytest.raises(ZeroDivisionError):
        st.percentiles
    from tmlibrary_amd.image import ChannelImage
    with pytest.raises(ValueError):
        st.update(ChannelImage(np.zeros((8, 9), np.uint16)))
    with pytest.raises(TypeError):
        st.update(np.zeros((8, 8), np.uint16))


@pytest.mark.parametrize("name", ["apply_log", "apply_nolog"])
def test_smooth_and_correct_vs_golden(L, name):
    from tmlibrary_amd.image import (ChannelImage, IllumstatsContainer, IllumstatsImage,
                                     smooth_f64)
    from tmlibrary_amd.metadata import ChannelImageMetadata, IllumstatsImageMetadata
    g = load_golden(name)
    log = name == "apply_log"
    # smoothing (pinned vs scipy reflect; mahotas itself is unavailable)
    assert np.allclose(smooth_f64(g["stats_mean"], 5), g["smooth_mean"], rtol=1e-10, atol=1e-13)
    assert np.allclose(smooth_f64(g["stats_std"], 5), g["smooth_std"], rtol=1e-10, atol=1e-13)
    md = IllumstatsImageMetadata(channel_id=7)
    cont = IllumstatsContainer(IllumstatsImage(g["stats_mean"].copy(), md),
                               IllumstatsImage(g["stats_std"].copy(), md), {})
    cont.smooth()
    assert cont.mean.metadata.is_smoothed and cont.std.metadata.is_smoothed
    for img, want, want_clip in zip(g["images"], g["corrected"], g["clipped"]):
        got = ChannelImage._correct_illumination(img, g["smooth_mean"], g["smooth_std"], log)
        assert_dn(got, want)
        assert np.mean(got == want) > 0.999
        if log:
            ci = ChannelImage(img.copy(), ChannelImageMetadata(7, 1, 1, 0, 0))
            ci.correct(cont)
            assert ci.metadata.is_corrected
            assert_dn(ci.array, want)
            ci.clip(int(g["clip_lo"]), int(g["clip_hi"]))
            assert ci.metadata.is_clipped
            assert_dn(ci.array, want_clip)
        clipped = ChannelImage(want.copy(), ChannelImageMetadata(7, 1, 1, 0, 0)).clip(
            int(g["clip_lo"]), int(g["clip_hi"]))
        assert np.array_equal(clipped.array, want_clip)


@pytest.mark.parametrize("shape", [(2160, 2560), (300, 217), (37, 53), (20, 30), (1, 300),
                                   (300, 1), (5, 5), (21, 41), (34, 41), (35, 234), (48, 64),
                                   (100, 235), (53, 433)])
def test_smooth_one_pass_bit_identical(L, shape, monkeypatch):
    """The one-pass 2-D smoothing kernel (k_smooth_2d_blk, sigma 5; planes of
    <= 20 rows: k_smooth_2d) equals the two separable passes bit for bit,
    edges and planes narrower than the kernel included, and matches the
    oracle.  21 / 34 rows and 41 / 64 / 234 / 235 columns: tiles whose halo
    threads and rows reach past one reflection (clamped, apply_kernels.hip)."""
    from tmlibrary_amd.image import smooth_f64
    rng = np.random.default_rng(shape[0] * 7 + shape[1])
    plane = rng.random(shape) * 4.0 + 1.0
    one = smooth_f64(plane, 5)
    monkeypatch.setenv("TMH_SMOOTH_2PASS", "1")
    two = smooth_f64(plane, 5)
    monkeypatch.delenv("TMH_SMOOTH_2PASS")
    assert np.array_equal(one, two)
    if plane.size <= 1e6:
        assert np.allclose(one, orc.smooth_reflect(plane, 5), rtol=1e-10, atol=1e-13)


@pytest.mark.parametrize("shape", [(1, 1), (1, 9), (3, 5), (20, 40), (40, 41), (41, 3), (7, 100)])
def test_smooth_small_planes(L, shape):
    """Planes smaller than the 41-tap kernel (sigma 5, radius 20): the
    reflected border indices repeat (apply_kernels.hip reflect rule,
    mahotas/scipy 'reflect' as restated by the oracle, itself pinned against
    scipy in test_oracle_golden)."""
    from tmlibrary_amd.image import smooth_f64
    rng = np.random.default_rng(shape[0] * 131 + shape[1])
    plane = rng.random(shape) * 4.0 + 1.0
    got = smooth_f64(plane, 5)
    want = orc.smooth_reflect(plane, 5)
    assert np.allclose(got, want, rtol=1e-10, atol=1e-13), np.abs(got - want).max()
    if plane.size > 1:
        assert np.allclose(smooth_f64(plane, 2), orc.smooth_reflect(plane, 2), rtol=1e-10,
                           atol=1e-13)


@pytest.mark.parametrize("shape,sigma", [((2160, 2560), 5.0), ((37, 53), 5.0), ((96, 128), 2.0),
                                         ((8, 700), 40.0)])
def test_smooth2_equals_two_planes(L, shape, sigma):
    """tmh_smooth2_f64_device (a job's mean and std in one launch per axis)
    is bit-identical to two tmh_smooth_f64_device calls, for the radius-20
    strip kernel, the generic axis-0 kernel and the wide (radius > 128)
    axis-1 kernel."""
    from tmlibrary_amd import hip
    H, W = shape
    rng = np.random.default_rng(H * 7 + W)
    a = rng.random(shape) * 3.0 + 0.5
    b = rng.random(shape) * 0.2 + 0.01
    bufs = [Dev(L, H * W * 8) for _ in range(8)]
    ia, ib, o1a, o1b, o2a, o2b, t0, t1 = bufs
    ia.put(a)
    ib.put(b)
    hip.check(L.tmh_smooth_f64_device(ia.p, o1a.p, t0.p, H, W, sigma, None))
    hip.check(L.tmh_smooth_f64_device(ib.p, o1b.p, t0.p, H, W, sigma, None))
    hip.check(L.tmh_smooth2_f64_device(ia.p, ib.p, o2a.p, o2b.p, t0.p, t1.p, H, W, sigma, None))
    L.tmh_synchronize(None)
    ra, rb = o1a.get(np.float64, shape), o1b.get(np.float64, shape)
    assert np.array_equal(o2a.get(np.float64, shape), ra)
    assert np.array_equal(o2b.get(np.float64, shape), rb)
    assert np.allclose(ra, orc.smooth_reflect(a, sigma), rtol=1e-10, atol=1e-13)
    # scratch aliasing an input or output is refused
    assert L.tmh_smooth2_f64_device(ia.p, ib.p, o2a.p, o2b.p, ia.p, t1.p, H, W, sigma, None) == -22
    for d in bufs:
        d.free()


def test_corrector_cache_sees_in_place_writes(L):
    """the container's cached corrector is keyed on content.
    Building it marks the planes read-only, so an in-place write raises; a
    caller who re-enables writing gets a rebuilt corrector on the next call."""
    from tmlibrary_amd.image import ChannelImage, IllumstatsContainer, IllumstatsImage
    from tmlibrary_amd.metadata import ChannelImageMetadata, IllumstatsImageMetadata
    rng = np.random.default_rng(9)
    img = rng.integers(1, 5000, (48, 64), dtype=np.uint16)
    mean = rng.random((48, 64)) * 0.2 + 2.5
    std = rng.random((48, 64)) * 0.1 + 0.2
    md = IllumstatsImageMetadata(channel_id=3)
    cont = IllumstatsContainer(IllumstatsImage(mean.copy(), md), IllumstatsImage(std.copy(), md), {})

    def corrected():
        ci = ChannelImage(img.copy(), ChannelImageMetadata(3, 1, 1, 0, 0))
        return ci.correct(cont).array

    first = corrected()
    assert_dn(first, orc.correct_illumination(img, mean, std))
    with pytest.raises(ValueError):
        cont.mean.array[0, 0] = 9.0  # read-only while a corrector is cached
    c1 = cont.corrector()
    assert cont.corrector() is c1  # unchanged planes: cached
    cont.mean.array.flags.writeable = True
    cont.mean.array[:, :32] += 0.05
    second = corrected()
    assert_dn(second, orc.correct_illumination(img, cont.mean.array, std))
    assert not np.array_equal(first, second)
    assert not cont.mean.array.flags.writeable  # protected again
    old_mean = cont.mean.array
    cont.smooth()  # replaced planes: rebuilt
    third = corrected()
    assert_dn(third, orc.correct_illumination(img, cont.mean.array, cont.std.array))
    assert old_mean.flags.writeable  # the replaced plane is unlocked again
    cont.release()  # drops the corrector, the current planes are writeable again
    assert cont.mean.array.flags.writeable and cont.std.array.flags.writeable
    cont.mean.array[0, 0] += 0.0


def test_corrector_outlives_container(L):
    """a Corrector handed out by ``corrector()`` keeps working after
    its container is released, rebuilt or collected (the cache only drops its
    reference; the Corrector's own __del__ frees the handle)."""
    import gc

    from tmlibrary_amd.image import IllumstatsContainer, IllumstatsImage
    from tmlibrary_amd.metadata import IllumstatsImageMetadata
    rng = np.random.default_rng(10)
    img = rng.integers(1, 5000, (40, 56), dtype=np.uint16)
    mean = rng.random((40, 56)) * 0.2 + 2.5
    std = rng.random((40, 56)) * 0.1 + 0.2
    want = orc.correct_illumination(img, mean, std)
    md = IllumstatsImageMetadata(channel_id=1)

    def make():
        return IllumstatsContainer(IllumstatsImage(mean.copy(), md),
                                   IllumstatsImage(std.copy(), md), {})

    corr = make().corrector()  # the container is a temporary
    gc.collect()
    assert_dn(corr.apply(img), want)
    cont = make()
    c1 = cont.corrector()
    cont.release()
    assert_dn(c1.apply(img), want)
    c2 = cont.corrector()
    cont.smooth()
    cont.corrector()  # rebuilt: the old one is only dropped
    assert_dn(c2.apply(img), want)
    del cont
    gc.collect()
    assert_dn(c2.apply(img), want)


def test_correct_channel_mismatch(L):
    from tmlibrary_amd.image import ChannelImage, IllumstatsContainer, IllumstatsImage
    from tmlibrary_amd.metadata import ChannelImageMetadata, IllumstatsImageMetadata
    md = IllumstatsImageMetadata(channel_id=1)
    cont = IllumstatsContainer(IllumstatsImage(np.ones((4, 4)), md),
                               IllumstatsImage(np.ones((4, 4)), md), {})
    ci = ChannelImage(np.ones((4, 4), np.uint16), ChannelImageMetadata(2, 1, 1, 0, 0))
    with pytest.raises(ValueError):
        ci.correct(cont)
    with pytest.raises(TypeError):
        ci.correct("stats")


def test_correct_u8(L):
    from tmlibrary_amd.image import ChannelImage
    g = load_golden("apply_u8")
    got = ChannelImage._correct_illumination(g["images"][0], g["smooth_mean"], g["smooth_std"])
    assert got.dtype == np.uint8
    assert_dn(got, g["corrected"][0], bits=8)


def test_correct_special_stats(L):
    """std = 0 / NaN (n < 2) and extreme outputs follow the x86 cast rule."""
    from tmlibrary_amd.image import ChannelImage
    rng = np.random.default_rng(5)
    img = rng.integers(0, 65536, (64, 80), dtype=np.uint16)
    img[0, :4] = [0, 1, 65535, 2]
    mean = rng.random((64, 80)) * 3
    std = rng.random((64, 80)) * 0.5 + 0.01
    std[5, :] = 0.0
    std[6, :] = np.nan
    for log in (True, False):
        got = ChannelImage._correct_illumination(img, mean, std, log)
        want = orc.correct_illumination(img, mean, std, log)
        worst, flips, _ = dn_report(got, want)
        assert worst <= 1 and flips == 0, (log, worst, flips)


def test_fullsize_two_sites(L):
    """2160x2560: samples/digests of the reference outputs (fixture)."""
    from tmlibrary_amd.image import ChannelImage, Corrector, smooth_f64
    from tmlibrary_amd.synth import synth_sites_host
    g = load_golden("fullsize_2site")
    H, W = int(g["height"]), int(g["width"])
    sites = synth_sites_host(int(g["n_sites"]), H, W, seed=int(g["seed"]))
    st = run_stats(sites, batch=2)
    iy, ix = g["sample_y"], g["sample_x"]
    assert_close_rel(st.mean.array[iy, ix], g["mean_samples"])
    assert_close_rel(st.std.array[iy, ix], g["std_samples"])
    assert np.array_equal(st.percentile_sums, g["pct_sums"])
    pct = st.percentiles
    assert np.array_equal(np.array([pct[k] for k in sorted(pct)]), g["pct_values"])
    sm, ss = smooth_f64(st.mean.array, 5), smooth_f64(st.std.array, 5)
    assert np.allclose(sm[iy, ix], g["smooth_mean_samples"], rtol=1e-9, atol=1e-12)
    corr = Corrector(sm, ss).apply(sites[0])
    assert_dn(corr[iy, ix], g["corrected_samples"])
    h = np.bincount(corr.ravel(), minlength=65536)
    # +-1 DN: the corrected histogram moves by at most the pixels that flip a bin
    assert np.abs(h - g["corrected_hist"]).sum() <= 0.002 * corr.size
    exact = hashlib.sha256(corr.tobytes()).hexdigest() == str(g["corrected_digest"])
    print("fullsize corrected bit-identical to reference:", exact)


def test_device_path_large_batch(L):
    """Sites generated in HBM, one update_device call, vs the oracle on a copy."""
    from tmlibrary_amd import hip
    from tmlibrary_amd.workflow.corilla.quantiles import quantile_table, stats_log10_lut
    H, W, n = 540, 640, 40
    npx = H * W
    d = Dev(L, n * npx * 2)
    hip.check(L.tmh_synth_sites_device(d.p, n, H, W, 99, 0, 0, hip.TMH_SYNTH_STANDARD, None))
    L.tmh_synchronize(None)
    sites = d.get(np.uint16, (n, H, W))
    from tmlibrary_amd.synth import synth_exact_host  # the device generator's host twin
    for i in (0, n - 1):
        assert np.array_equal(sites[i], synth_exact_host(H, W, 99, 0, i))
    q = np.linspace(0, 100, 100000)
    lo, hi, gamma = quantile_table(npx, q)
    lut = stats_log10_lut()
    h = C.c_void_p()
    hip.check(L.tmh_stats_create(H, W, 100000, hip.ptr(lo), hip.ptr(hi), hip.ptr(gamma),
                                 hip.ptr(lut), 8, 0, C.byref(h)))
    hip.check(L.tmh_stats_update_device(h, d.p, n, 1, None))
    mean = np.empty((H, W))
    std = np.empty((H, W))
    acc = np.empty(100000)
    nn = C.c_int64()
    hip.check(L.tmh_stats_finalize(h, C.byref(nn), hip.ptr(mean), hip.ptr(std), hip.ptr(acc), None))
    ref = orc.run_illumstats(list(sites))
    assert nn.value == n
    assert_close_rel(mean, ref.mean)
    assert_close_rel(std, ref.std)
    assert np.array_equal(acc, ref.percentile_sums)
    L.tmh_stats_destroy(h)
    d.free()


def test_deferred_chain_and_merge_single_gpu(L):
    """Two handles = two 'ranks' on one GPU: Chan merge + ordered percentile
    chain reproduce the single-handle result (mean/std 1e-6, pct bit-exact)."""
    from tmlibrary_amd import hip
    from tmlibrary_amd.workflow.corilla.quantiles import quantile_table, stats_log10_lut
    sites = np.stack(load_golden("stats_medium")["sites"])
    n, H, W = sites.shape
    npx = H * W
    q = np.linspace(0, 100, 100000)
    lo, hi, gamma = quantile_table(npx, q)
    lut = stats_log10_lut()

    def mk(flags):
        h = C.c_void_p()
        hip.check(L.tmh_stats_create(H, W, 100000, hip.ptr(lo), hip.ptr(hi), hip.ptr(gamma),
                                     hip.ptr(lut), 4, flags, C.byref(h)))
        return h

    parts = [sites[:1], sites[1:]]
    hs = [mk(hip.TMH_STATS_DEFERRED_PCT) for _ in parts]
    for h, p in zip(hs, parts):
        hip.check(L.tmh_stats_update(h, hip.ptr(np.ascontiguousarray(p)), len(p), 1, None))
    # all-reduce emulated by host sums of the device buffers
    bufs = [Dev(L, npx * 8) for _ in hs]
    for h, b in zip(hs, bufs):
        hip.check(L.tmh_stats_merge_stage1(h, b.p, None))
    L.tmh_synchronize(None)
    s1 = sum(b.get(np.float64, npx) for b in bufs)
    sum_dev = Dev(L, npx * 8)
    sum_dev.put(s1)
    for h, b in zip(hs, bufs):
        hip.check(L.tmh_stats_merge_stage2(h, sum_dev.p, n, b.p, None))
    L.tmh_synchronize(None)
    s2 = sum(b.get(np.float64, npx) for b in bufs)
    sum_dev.put(s2)
    for h in hs:
        hip.check(L.tmh_stats_merge_stage3(h, n, sum_dev.p, None))
    acc = Dev(L, 100000 * 8)
    acc.put(np.zeros(100000))
    for h in hs:  # rank order; each handle has its own stream, so wait in between
        hip.check(L.tmh_stats_pct_accumulate(h, acc.p, None))
        L.tmh_synchronize(None)
    for h in hs:
        hip.check(L.tmh_stats_set_pct_sum(h, acc.p, None))
    L.tmh_synchronize(None)
    ref = orc.run_illumstats(list(sites))
    for h in hs:
        mean = np.empty((H, W))
        std = np.empty((H, W))
        pct = np.empty(100000)
        nn = C.c_int64()
        hip.check(L.tmh_stats_finalize(h, C.byref(nn), hip.ptr(mean), hip.ptr(std), hip.ptr(pct),
                                       None))
        assert nn.value == n
        assert_close_rel(mean, ref.mean)
        assert_close_rel(std, ref.std)
        assert np.array_equal(pct, ref.percentile_sums)
        L.tmh_stats_destroy(h)
    for b in bufs + [sum_dev, acc]:
        b.free()


def test_profile_counters(L):
    from tmlibrary_amd import hip
    L.tmh_profile_enable(1)
    L.tmh_profile_reset()
    run_stats(list(load_golden("stats_small")["sites"]), batch=8)._finalize()
    ms, k = C.c_double(), C.c_int64()
    hip.check(L.tmh_profile_read(b"welford", C.byref(ms), C.byref(k)))
    assert k.value >= 1 and ms.value > 0
    L.tmh_profile_enable(0)


@pytest.mark.parametrize("decode,block", [("host", 128), ("gpu", 128), ("gpu", 3)])
def test_run_job_end_to_end(L, tmp_path, decode, block, caplog):
    """IllumstatsCalculator.run_job: gzip HDF5 sites in batch order -> GPU stats
    -> IllumstatsFile (4 datasets) -> IllumstatsFile.get (smoothed).  The
    sites decoded on the host (libhdf5 + zlib) or inflated on the GPU, in one
    device block or in blocks of 3 (several blocks in flight): the same bits."""
    pytest.importorskip("tmlibrary_amd.models.file")
    from tmlibrary_amd.models import file as h5
    try:
        h5.h5lib()
    except RuntimeError as e:
        pytest.skip(str(e))
    from tmlibrary_amd.workflow.corilla.api import IllumstatsCalculator
    g = load_golden("stats_medium")
    sites = list(g["sites"])
    store = h5.ExperimentStore(str(tmp_path), {100 + i: (5, i, 0, 0, 0) for i in range(len(sites))})
    (tmp_path / "channel_image_files").mkdir()
    for i, s in enumerate(sites):
        h5.write_channel_image(store.channel_image_file(100 + i).location, s)
    batch = {"id": 1, "channel_image_files_ids": [[100 + i] for i in range(len(sites))],
             "channel_id": 5}
    with caplog.at_level("WARNING"):
        IllumstatsCalculator(1, store=store, batch_size=2, decode=decode,
                             device_block=block).run_job(batch)
    n_warn = sum("image contains zero values" in r.message for r in caplog.records)
    assert n_warn == sum(int(np.any(s == 0)) for s in sites)
    mean, std, keys, vals = h5.read_illumstats(store.illumstats_file(5).location)
    assert_close_rel(mean, g["mean"])
    assert_close_rel(std, g["std"])
    got = dict(zip(keys.tolist(), vals.tolist()))
    assert [got[k] for k in sorted(got)] == g["pct_values"].tolist()
    cont = store.illumstats_file(5).get()
    assert cont.mean.metadata.is_smoothed
    assert np.allclose(cont.mean.array, orc.smooth_reflect(g["mean"]), rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("plain", [(), (0,), (2,), (3,)])
def test_run_job_auto_mixed_layouts(L, tmp_path, plain):
    """decode="auto" over a job whose files mix the reference's gzip chunks
    with contiguous (uncompressed) ones: the GPU path runs up to the first
    block it cannot read and the host decodes from that file on -- every site
    counted once, in order (a fallback that restarted on the host
    counted the GPU blocks twice).  A file of another shape raises the
    reference's broadcast ValueError, and the calculator's next job is clean."""
    from tmlibrary_amd.models import file as h5
    try:
        h5.h5lib()
    except RuntimeError as e:
        pytest.skip(str(e))
    from tmlibrary_amd.workflow.corilla.api import IllumstatsCalculator
    g = load_golden("stats_medium")
    sites = list(g["sites"])
    store = h5.ExperimentStore(str(tmp_path), {100 + i: (5, i, 0, 0, 0) for i in range(len(sites))})
    (tmp_path / "channel_image_files").mkdir()
    for i, s in enumerate(sites):
        h5.write_channel_image(store.channel_image_file(100 + i).location, s,
                               gzip_level=-1 if i in plain else 4)
    batch = {"id": 1, "channel_image_files_ids": [[100 + i] for i in range(len(sites))],
             "channel_id": 5}
    # blocks of one file: the GPU path takes the files before the first plain one
    calc = IllumstatsCalculator(1, store=store, batch_size=2, decode="auto", device_block=1)
    calc.run_job(batch)
    mean, std, keys, vals = h5.read_illumstats(store.illumstats_file(5).location)
    assert_close_rel(mean, g["mean"])
    assert_close_rel(std, g["std"])
    got = dict(zip(keys.tolist(), vals.tolist()))
    assert [got[k] for k in sorted(got)] == g["pct_values"].tolist()
    if plain:
        with pytest.raises(h5.RawChunksUnsupported):  # strict GPU decode refuses them
            IllumstatsCalculator(1, store=store, batch_size=2, decode="gpu",
                                 device_block=1).run_job(batch)
        return
    # a site of another shape in a later block: the reference's broadcast error
    odd = 100 + len(sites) - 1
    h5.write_channel_image(store.channel_image_file(odd).location, sites[-1][:-1])
    with pytest.raises(ValueError):
        calc.run_job(batch)
    h5.write_channel_image(store.channel_image_file(odd).location, sites[-1])
    calc.run_job(batch)  # the calculator's decoder carries nothing over
    mean2, _, _, vals2 = h5.read_illumstats(store.illumstats_file(5).location)
    assert np.array_equal(mean2, mean) and np.array_equal(vals2, vals)


def _fused_job(L, sites, clip=(-1, -1), q=None):
    """Split pipeline through the C-ABI: Welford-only update -> finalize ->
    smooth -> corrector -> fused correct+histogram.  Returns host results."""
    from tmlibrary_amd import hip
    from tmlibrary_amd.image import ZERO_LOG10
    from tmlibrary_amd.workflow.corilla.quantiles import quantile_table, stats_log10_lut
    n, H, W = sites.shape
    npx = H * W
    q = np.linspace(0, 100, 100000) if q is None else q
    Q = len(q)
    lo, hi, gamma = quantile_table(npx, q)
    lut = stats_log10_lut()
    h = C.c_void_p()
    hip.check(L.tmh_stats_create(H, W, Q, hip.ptr(lo), hip.ptr(hi), hip.ptr(gamma),
                                 hip.ptr(lut), 4, hip.TMH_STATS_KEEP_SITE_HIST, C.byref(h)))
    d_in, d_out = Dev(L, sites.nbytes), Dev(L, sites.nbytes)
    d_in.put(sites)
    planes = [Dev(L, npx * 8) for _ in range(5)]
    mean, std, smean, sstd, tmp = planes
    hip.check(L.tmh_stats_update_welford_device(h, d_in.p, n, 1, None))
    hip.check(L.tmh_stats_finalize_device(h, mean.p, std.p, None))
    L.tmh_synchronize(None)
    hip.check(L.tmh_smooth_f64_device(mean.p, smean.p, tmp.p, H, W, 5.0, None))
    hip.check(L.tmh_smooth_f64_device(std.p, sstd.p, tmp.p, H, W, 5.0, None))
    L.tmh_synchronize(None)
    c = C.c_void_p()
    hip.check(L.tmh_corrector_create_device(smean.p, sstd.p, H, W, 1, ZERO_LOG10, None, C.byref(c)))
    hip.check(L.tmh_correct_u16_hist_device(c, h, d_in.p, d_out.p, n, clip[0], clip[1], None))
    L.tmh_synchronize(None)
    acc = np.empty(Q)
    nn = C.c_int64()
    m_h = np.empty((H, W))
    s_h = np.empty((H, W))
    hist = np.empty(65536, np.uint64)
    hip.check(L.tmh_stats_finalize(h, C.byref(nn), hip.ptr(m_h), hip.ptr(s_h), hip.ptr(acc),
                                   hip.ptr(hist)))
    site_h = []
    for i in range(n):
        sh = np.empty(65536, np.uint32)
        hip.check(L.tmh_stats_site_histogram(h, i, hip.ptr(sh)))
        site_h.append(sh)
    out = d_out.get(np.uint16, sites.shape)
    pc, wb, fc = (C.c_uint32 * 3)(), C.c_int(), C.c_int()
    hip.check(L.tmh_stats_job_choice(h, pc, C.byref(wb), C.byref(fc)))
    res = dict(n=nn.value, mean=m_h, std=s_h, acc=acc, hist=hist, site_hist=site_h, out=out,
               fused_cfg=fc.value, welford_bright=wb.value,
               smean=smean.get(np.float64, (H, W)), sstd=sstd.get(np.float64, (H, W)),
               order_stats=site_order_stats(L, h, range(n), Q))
    L.tmh_corrector_destroy(c)
    L.tmh_stats_destroy(h)
    for b in planes + [d_in, d_out]:
        b.free()
    return res


@pytest.mark.parametrize("kind", ["synth", "extremes", "uniform", "tiny", "many", "saturated",
                                  "constant", "two_values", "dark_prefix_wide_tail"])
def test_fused_correct_hist_pipeline(L, kind):
    """The fused pass and its percentile tail: one-bin sites, Q > pixel
    count, sparse tails, the very wide path of the uniform case, each
    bit-exact.  dark_prefix_wide_tail: the job's site probe sees only the
    first 64 sites (dark), so the narrow configuration runs and the wide
    tail's values take its global-atomic path (tmhip.h, the probe's first-sites
    assumption): slower, and still bit-exact."""
    from tmlibrary_amd.synth import synth_exact_sites_host, synth_sites_host
    rng = np.random.default_rng(97)
    if kind == "saturated":  # corrected values far above 2**16 (f64 refinement, common.h)
        sites = synth_exact_sites_host(6, 240, 320, 5, 0)
        sites[:, ::7, ::5] = 65535
        sites[1:, 3::11, 1::13] = 0
    elif kind == "synth":
        sites = np.stack(synth_sites_host(7, 240, 320, seed=31))
        sites[2, :4, :4] = 65535
        sites[3, 5, :9] = 40000  # beyond the LDS bins and the LDS LUT
    elif kind == "uniform":  # most values beyond the per-site LDS slices
        sites = rng.integers(0, 65536, size=(6, 96, 160), dtype=np.uint16)
    elif kind == "tiny":  # bands far narrower than a workgroup
        sites = np.stack(synth_sites_host(5, 16, 24, seed=5))
    elif kind == "many":  # several site groups per band, ragged last group
        sites = np.stack(synth_sites_host(37, 64, 96, seed=8))
        sites[::5, 3, :] = 65000
    elif kind == "constant":  # one bin per site (one compact-CDF entry)
        sites = np.stack([np.full((48, 64), v, np.uint16) for v in (0, 777, 65535, 4096)])
    elif kind == "dark_prefix_wide_tail":
        dark = np.stack(synth_sites_host(64, 48, 64, seed=12))
        assert dark.max() < 4096 or (dark >= 4096).mean() < 1e-3
        wide = rng.integers(0, 65536, size=(6, 48, 64), dtype=np.uint16)
        sites = np.concatenate([dark, wide])
    elif kind == "two_values":  # every quantile chunk inside one of two entries
        sites = np.stack([np.where(rng.random((48, 64)) < 0.3, 3, 60000).astype(np.uint16)
                          for _ in range(5)])
    else:
        sites = np.stack(load_golden("stats_extremes")["sites"])
    r = _fused_job(L, sites)
    ref = orc.run_illumstats(list(sites))
    assert r["n"] == len(sites)
    if kind == "dark_prefix_wide_tail":
        assert r["fused_cfg"] == 3, "the probe saw only the dark prefix: narrow configuration"
    assert_close_rel(r["mean"], ref.mean)
    assert_close_rel(r["std"], ref.std)
    assert np.array_equal(r["acc"], ref.percentile_sums), "fused percentile sums not bit-exact"
    for s, sh in zip(sites, r["site_hist"]):
        assert np.array_equal(sh.astype(np.uint64), orc.histogram_u16(s))
    assert np.array_equal(r["hist"], sum(orc.histogram_u16(s) for s in sites))
    for s, o in zip(sites, r["out"]):
        want = orc.correct_illumination(s, r["smean"], r["sstd"])
        assert_dn(o, want)
    check_order_stats(sites, r["order_stats"])


def test_bright_welford_table_edges(L):
    """The bright Welford form's table covers values below 20,472 (160 KB of
    LDS, stats_kernels.hip kWfLutBright; indices clamped, not masked): values
    on both sides of its end and of round 6's 16,384-entry end, in every
    site and as constant columns (std exactly 0 on either path), against the
    oracle at the 1e-6 bar everywhere and 1e-9 on the edge pixels (the
    log10_big path past the table is within 3e-10 of numpy's log10)."""
    from tmlibrary_amd.synth import BRIGHT, synth_exact_host
    n, H, W = 100, 48, 64  # >= 96 sites: the bright form's three site parts
    sites = np.stack([synth_exact_host(H, W, 77, 1, i, BRIGHT) for i in range(n)])
    edges = np.array([16383, 16384, 20470, 20471, 20472, 20473, 32768, 65535], np.uint16)
    for i in range(n):
        sites[i, 0, :16] = np.roll(np.tile(edges, 2), i)
    sites[:, 1, 0] = 20471  # constant columns: table / log10_big path
    sites[:, 1, 1] = 20472
    r = _fused_job(L, sites)
    assert r["welford_bright"] == 1, "the probe should pick the bright Welford form"
    ref = orc.run_illumstats(list(sites))
    assert_close_rel(r["mean"], ref.mean)
    assert_close_rel(r["std"], ref.std)
    assert_close_rel(r["mean"][0, :16], ref.mean[0, :16], rtol=1e-9)
    assert_close_rel(r["std"][0, :16], ref.std[0, :16], rtol=1e-9)
    assert r["std"][1, 0] == 0.0 and r["std"][1, 1] == 0.0
    assert np.array_equal(r["acc"], ref.percentile_sums)


@pytest.mark.parametrize("kind", ["lognormal_tails", "uniform", "constant", "two_values",
                                  "sparse", "tiny"])
def test_order_statistics_scatter_path(L, kind):
    """The per-site order statistics of the non-fused update path (one
    histogram workgroup per site, all 64 rounds) decode to the oracle's for
    every quantile: dense middles (compact tiles), sparse tails (dense
    fallback tiles), one-bin sites, Q > pixel count (tiny)."""
    from tmlibrary_amd.synth import synth_sites_host
    rng = np.random.default_rng(5)
    h, w = 240, 320
    if kind == "lognormal_tails":
        sites = [np.clip(rng.lognormal(7.0, 1.1, (h, w)), 0, 65535).astype(np.uint16)
                 for _ in range(3)]
    elif kind == "uniform":
        sites = [rng.integers(0, 65536, (h, w), dtype=np.uint16) for _ in range(3)]
    elif kind == "constant":
        sites = [np.full((h, w), 777, np.uint16), np.full((h, w), 0, np.uint16),
                 np.full((h, w), 65535, np.uint16)]
    elif kind == "two_values":
        sites = [np.where(rng.random((h, w)) < 0.3, 3, 60000).astype(np.uint16) for _ in range(3)]
    elif kind == "sparse":  # few distinct values spread over the range
        vals = np.sort(rng.choice(65536, 40, replace=False)).astype(np.uint16)
        sites = [vals[rng.integers(0, 40, (h, w))] for _ in range(3)]
    else:
        sites = synth_sites_host(4, 20, 30, seed=3)
    st = run_stats(sites, batch=len(sites))
    st._finalize()
    check_order_stats(sites, site_order_stats(L, st._h, range(len(sites)), 100000))
    ref = orc.run_illumstats(sites)
    assert np.array_equal(st.percentile_sums, ref.percentile_sums)


@pytest.mark.parametrize("qkind", ["linspace", "custom"])
def test_quantile_tables(L, qkind):
    """Percentile sums stay bit-exact for the reference's linspace q
    (stats.py:59-60, another Q) and for arbitrary non-uniform q tables."""
    from tmlibrary_amd.synth import synth_sites_host
    sites = np.stack(synth_sites_host(5, 120, 160, seed=12))
    if qkind == "linspace":
        q = np.linspace(0, 100, 10000)
    else:
        rng = np.random.default_rng(4)
        q = np.concatenate([[0.0], np.sort(rng.uniform(0, 100, 997)), [99.99, 100.0]])
    r = _fused_job(L, sites, q=q)
    want = np.zeros(len(q))
    for s in sites:
        want += orc.percentile_linear(s, q)
    assert np.array_equal(r["acc"], want)
    check_order_stats(sites, r["order_stats"], q)


@pytest.mark.parametrize("parts", [2, 3, 4])
def test_welford_site_parts(L, parts):
    """Site-split Welford launches (TMH_OPT_WELFORD_PARTS forces the split the
    launch policy picks at 2160x2560): parts merged in order, then into the
    state of the previous launch -- mean/std still within the 1e-6 bar, and
    var = M2 / (n - 1) from the device (stats.py:94-102)."""
    from tmlibrary_amd import hip
    from tmlibrary_amd.image import ChannelImage
    from tmlibrary_amd.synth import synth_sites_host
    from tmlibrary_amd.workflow.corilla.stats import OnlineStatistics
    sites = synth_sites_host(400, 48, 64, seed=31)
    st = OnlineStatistics((48, 64), batch_size=200, options={hip.TMH_OPT_WELFORD_PARTS: parts})
    for s in sites:
        st.update(ChannelImage(s))
    ref = orc.run_illumstats(sites)
    assert st.n == ref.n == 400
    assert_close_rel(st.mean.array, ref.mean)
    assert_close_rel(st.std.array, ref.std)
    assert_close_rel(st.var, ref.var)
    assert np.array_equal(st.percentile_sums, ref.percentile_sums)
    st.close()


def test_pipelined_chain_ranges_bit_exact(L):
    """tmh_stats_pct_accumulate_range over quantile chunks, chunk-major across
    two 'ranks' (the pipelined chain's order), equals the sequential sum."""
    from tmlibrary_amd import hip
    from tmlibrary_amd.workflow.corilla.quantiles import quantile_table, stats_log10_lut
    from tmlibrary_amd.workflow.corilla.sharded import chain_chunks
    sites = np.stack(load_golden("stats_medium")["sites"])
    n, H, W = sites.shape
    Q = 100000
    lo, hi, gamma = quantile_table(H * W, np.linspace(0, 100, Q))
    lut = stats_log10_lut()
    parts = [sites[:2], sites[2:]]
    hs = []
    for p in parts:
        h = C.c_void_p()
        hip.check(L.tmh_stats_create(H, W, Q, hip.ptr(lo), hip.ptr(hi), hip.ptr(gamma),
                                     hip.ptr(lut), 4, hip.TMH_STATS_DEFERRED_PCT, C.byref(h)))
        hip.check(L.tmh_stats_update(h, hip.ptr(np.ascontiguousarray(p)), len(p), 1, None))
        hs.append(h)
    L.tmh_synchronize(None)
    acc = Dev(L, Q * 8)
    acc.put(np.zeros(Q))
    for q0, qn in chain_chunks(Q, 2, chunks=7) + [(Q, 0)]:
        for h in hs:
            hip.check(L.tmh_stats_pct_accumulate_range(h, C.c_void_p(acc.p.value + 8 * q0), q0, qn,
                                                       None))
            L.tmh_synchronize(None)
    got = acc.get(np.float64, Q)
    ref = orc.run_illumstats(list(sites))
    assert np.array_equal(got, ref.percentile_sums)
    assert hip.lib().tmh_stats_pct_accumulate_range(hs[0], acc.p, Q - 2, 4, None) != 0
    for h in hs:
        L.tmh_stats_destroy(h)
    acc.free()
