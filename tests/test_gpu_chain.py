"""GPU parity of the illuminati post-correct chain:
Image.align, ChannelImage._map_to_uint8 / scale, and the fused
correct -> align(crop=False) -> clip -> scale pass, against fixtures generated
from the reference (tests/golden/make_goldens.py: align, map_uint8, chain).

Bars: align and the uint16 -> uint8 LUT bit-exact; the fused chain within the
correction's +-1 DN carried through clip/scale (<= 1 uint8 step)."""
import numpy as np
import pytest

from util import load_golden
from oracle import corilla_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    from tmlibrary_amd import hip
    return hip.lib()


def _md(y=0, x=0, residues=(0, 0, 0, 0)):
    from tmlibrary_amd.metadata import ChannelImageMetadata
    md = ChannelImageMetadata(channel_id=1, site_id=1, cycle_id=1, tpoint=0, zplane=0)
    md.y_shift, md.x_shift = int(y), int(x)
    md.bottom_residue, md.top_residue, md.right_residue, md.left_residue = map(int, residues)
    return md


@pytest.mark.parametrize("dtype", [np.uint16, np.uint8])
def test_align_vs_reference(L, dtype):
    from tmlibrary_amd.image import ChannelImage
    g = load_golden("align")
    img = g["image"]
    if dtype == np.uint8:
        img = (img >> 8).astype(np.uint8)
    for i, (y, x, b, t, r, l) in enumerate(g["cases"]):
        for crop in (False, True):
            got = ChannelImage(img.copy(), _md(y, x, (b, t, r, l))).align(crop=crop).array
            want = g["cropped_%d" % i] if crop else g["padded"][i]
            if dtype == np.uint8:
                want = orc.shift_and_crop(img, y, x, b, t, r, l, crop=crop)
            assert got.dtype == dtype
            assert np.array_equal(got, want), (i, crop)


def test_align_needs_metadata(L):
    from tmlibrary_amd.image import ChannelImage
    with pytest.raises(AttributeError):
        ChannelImage(np.zeros((4, 4), np.uint16)).align()


def test_map_to_uint8_lut_exhaustive(L):
    """Every uint16 value through the GPU scale == the reference's numpy LUT."""
    from tmlibrary_amd.image import ChannelImage
    g = load_golden("map_uint8")
    full = np.arange(65536, dtype=np.uint16).reshape(256, 256)
    for (lo, hi), lut in zip(g["bounds"], g["luts"]):
        got = ChannelImage._map_to_uint8(full, int(lo), int(hi))
        assert np.array_equal(got.ravel(), lut), (lo, hi)


def test_map_to_uint8_errors_and_defaults(L):
    from tmlibrary_amd.image import ChannelImage
    a = np.array([[5, 9], [300, 7]], dtype=np.uint16)
    with pytest.raises(TypeError):
        ChannelImage._map_to_uint8(a.astype(np.uint8), 0, 10)
    with pytest.raises(ValueError):
        ChannelImage._map_to_uint8(a, 10, 10)
    with pytest.raises(ValueError):
        ChannelImage._map_to_uint8(a, 0, 70000)
    assert np.array_equal(ChannelImage._map_to_uint8(a), orc.map_to_uint8(a))
    im = ChannelImage(a.copy(), _md()).scale(5, 300)
    assert im.array.dtype == np.uint8 and im.metadata.is_rescaled
    u8 = ChannelImage(np.ones((2, 2), np.uint8), _md())
    assert u8.scale(0, 10) is u8


def _chain_inputs():
    from tmlibrary_amd.image import align_window
    g = load_golden("chain")
    wins = [align_window(g["images"].shape[1:], y, x, *g["residues"], crop=False)[0]
            for y, x in g["shifts"]]
    return g, np.stack(wins)


def test_chain_fused_vs_reference(L):
    from tmlibrary_amd.image import Corrector
    g, wins = _chain_inputs()
    corr = Corrector(g["smooth_mean"], g["smooth_std"])
    got = corr.chain_u8(g["images"], wins, int(g["clip_lo"]), int(g["clip_hi"]))
    corr.close()
    d = np.abs(got.astype(np.int32) - g["scaled"].astype(np.int32))
    assert d.max() <= 1
    assert (d == 0).mean() > 0.99


def _layer_percentiles(sites):
    """the channel's percentile dict (stats.py:114-121) from the pinned oracle"""
    st = orc.run_illumstats(sites)
    keys, vals = orc.percentile_keys(3), orc.percentile_values(st.percentile_sums, st.n)
    return dict(zip(keys.tolist(), vals.tolist()))


def test_chain_with_derived_clip_bounds(L):
    """illuminati's layer (api.py:119-164, 389-405): the clip bounds derived
    from the channel's percentiles (workflow/illuminati.clip_bounds) fed to
    the fused chain -- the chain fixture's layer, whose bounds the reference
    took from the same statistics sites (make_goldens.py)."""
    from tmlibrary_amd.image import IllumstatsContainer, IllumstatsImage
    from tmlibrary_amd.synth import synth_sites_host
    from tmlibrary_amd.workflow.illuminati import correct_chain_u8
    g, wins = _chain_inputs()
    pct = _layer_percentiles(synth_sites_host(6, 96, 128, seed=1111))
    stats = IllumstatsContainer(IllumstatsImage(g["smooth_mean"].copy()),
                                IllumstatsImage(g["smooth_std"].copy()), pct)
    got, bounds = correct_chain_u8(stats, g["images"], wins)
    stats.release()
    assert bounds == (int(g["clip_lo"]), int(g["clip_hi"]))
    d = np.abs(got.astype(np.int32) - g["scaled"].astype(np.int32))
    assert d.max() <= 1 and (d == 0).mean() > 0.99


def test_chain_dim_channel_floor(L):
    """A dim channel's layer: clip_max raised to 700 (api.py:142-153), the
    chain against the oracle at those bounds."""
    from tmlibrary_amd.image import IllumstatsContainer, IllumstatsImage
    from tmlibrary_amd.synth import synth_sites_host
    from tmlibrary_amd.workflow.illuminati import correct_chain_u8
    g, wins = _chain_inputs()
    dim = [(s // 8).astype(np.uint16) for s in synth_sites_host(6, 96, 128, seed=1111)]
    st = orc.run_illumstats(dim)
    sm_mean, sm_std = orc.smooth_reflect(st.mean), orc.smooth_reflect(st.std)
    pct = _layer_percentiles(dim)
    stats = IllumstatsContainer(IllumstatsImage(sm_mean), IllumstatsImage(sm_std), pct)
    imgs = np.stack([(s // 8).astype(np.uint16) for s in g["images"]])
    got, (lo, hi) = correct_chain_u8(stats, imgs, wins)
    stats.release()
    assert hi == 700 and lo == orc.get_closest_percentile(pct, 0.001)
    for img, (y, x), o in zip(imgs, g["shifts"], got):
        want = orc.illuminati_chain(img, sm_mean, sm_std, (int(y), int(x)),
                                    tuple(int(v) for v in g["residues"]), lo, hi)
        assert np.abs(o.astype(np.int32) - want.astype(np.int32)).max() <= 1


def test_chain_by_steps_vs_reference(L):
    """The same chain through the drop-in API, one method at a time."""
    from tmlibrary_amd.image import ChannelImage, IllumstatsContainer, IllumstatsImage
    from tmlibrary_amd.metadata import IllumstatsImageMetadata
    g, _ = _chain_inputs()
    md_s = IllumstatsImageMetadata(channel_id=1)
    stats = IllumstatsContainer(IllumstatsImage(g["smooth_mean"].copy(), md_s),
                                IllumstatsImage(g["smooth_std"].copy(), md_s), {})
    lo, hi = int(g["clip_lo"]), int(g["clip_hi"])
    for img, (y, x), want in zip(g["images"], g["shifts"], g["scaled"]):
        im = ChannelImage(img.copy(), _md(y, x, g["residues"]))
        im = im.correct(stats).align(crop=False).clip(lo, hi).scale(lo, hi)
        d = np.abs(im.array.astype(np.int32) - want.astype(np.int32))
        assert d.max() <= 1


@pytest.mark.parametrize("shape,bounds", [((256, 320), (100, 3000)), ((70, 90), (100, 3000)),
                                          ((256, 320), (0, 65535)), ((256, 320), (700, 20000)),
                                          ((256, 320), (500, 501))])
def test_chain_device_random_windows(L, shape, bounds):
    """Device-resident batch with per-site shifts (incl. odd column shifts and
    an empty window) vs the oracle chain; odd widths take the scalar path.
    Clip bounds: the usual range, the whole 16-bit range, one wider than the
    old 16,384-entry table limit, and a single-step range (the lone 0 of
    _map_to_uint8) -- all through the 64 KB clip + scale table."""
    import ctypes as C
    from tmlibrary_amd import hip
    from tmlibrary_amd.image import Corrector, align_window
    from tmlibrary_amd.synth import synth_sites_host
    H, W = shape
    base = synth_sites_host(5, H, W, seed=41)
    st = orc.run_illumstats(base)
    sm, ss = orc.smooth_reflect(st.mean), orc.smooth_reflect(st.std)
    sites = np.stack(synth_sites_host(7, H, W, seed=42))
    sites[0, 3, :9] = 0
    # (1, 0): a whole-row shift, 8-byte aligned but not line aligned when W = 320
    shifts = [(0, 0), (3, -5), (-4, 7), (1, 1), (-2, -3), (0, 6), (1, 0)]
    res = (4, 4, 7, 7)
    wins = np.stack([align_window((H, W), y, x, *res, crop=False)[0] for y, x in shifts])
    wins[5]["rows"] = 0  # all padding
    lo, hi = bounds
    corr = Corrector(sm, ss)
    d_in = C.c_void_p()
    d_out = C.c_void_p()
    assert L.tmh_malloc_device(C.byref(d_in), sites.nbytes) == 0
    assert L.tmh_malloc_device(C.byref(d_out), sites.size) == 0
    assert L.tmh_memcpy(d_in, sites.ctypes.data, sites.nbytes, 0, None) == 0
    hip.check(L.tmh_correct_chain_u8_device(corr._h, d_in, d_out, len(sites), hip.ptr(wins), lo,
                                            hi, None))
    got = np.empty(sites.shape, np.uint8)
    assert L.tmh_memcpy(got.ctypes.data, d_out, got.nbytes, 1, None) == 0
    L.tmh_free_device(d_in)
    L.tmh_free_device(d_out)
    corr.close()
    for i, ((y, x), s) in enumerate(zip(shifts, sites)):
        if i == 5:
            assert not got[i].any()
            continue
        want = orc.illuminati_chain(s, sm, ss, (y, x), res, lo, hi)
        d = np.abs(got[i].astype(np.int32) - want.astype(np.int32))
        assert d.max() <= 1, i


@pytest.mark.parametrize("bounds", [(0, 65535), (100, 3000)])
def test_chain_overflow_wrap_and_beyond_int32(L, bounds):
    """Pixels with a tiny smoothed std (a = mean(std)/std ~ 1,000) whose
    corrected values land below 65,536, wrap modulo 65,536 (x86 cast of values
    in [65,536, 2^31)), pass 2^31 (the x86 cast gives INT_MIN: low half 0) or
    overflow to inf: k_chain_u8t casts without clamping and relies on every
    |value| >= T (T < 2^18) being refined in f64 -- checked here against the
    oracle's x86 cast (oracle/corilla_oracle.py cast_float_to_uint_x86)."""
    import ctypes as C
    from tmlibrary_amd import hip
    from tmlibrary_amd.image import Corrector, align_window
    H, W = 64, 320
    rng = np.random.default_rng(5)
    mu = np.full((H, W), 2.5) + 0.01 * rng.random((H, W))
    sd = np.full((H, W), 0.1)
    sd[:, 96:160] = 1e-4  # a ~ 1,000 in these columns
    sd[:, 200:208] = 1e-6  # a ~ 1e5: 10**t overflows to inf
    # pixels around 10**mu: log10 offsets -0.02 .. +0.02 -> exponents far below
    # and far above the uint16 range
    off = rng.uniform(-0.02, 0.02, (4, H, W))
    sites = np.clip(np.round(10.0 ** (mu + off)), 0, 65535).astype(np.uint16)
    sites[1, :, :8] = 0
    sites[2, 5, :] = 65535
    shifts = [(0, 0), (2, -3), (-1, 5), (0, 8)]
    res = (4, 4, 8, 8)
    wins = np.stack([align_window((H, W), y, x, *res, crop=False)[0] for y, x in shifts])
    lo, hi = bounds
    corr = Corrector(mu, sd)
    d_in, d_out = C.c_void_p(), C.c_void_p()
    assert L.tmh_malloc_device(C.byref(d_in), sites.nbytes) == 0
    assert L.tmh_malloc_device(C.byref(d_out), sites.size) == 0
    assert L.tmh_memcpy(d_in, sites.ctypes.data, sites.nbytes, 0, None) == 0
    hip.check(L.tmh_correct_chain_u8_device(corr._h, d_in, d_out, len(sites), hip.ptr(wins), lo,
                                            hi, None))
    got = np.empty(sites.shape, np.uint8)
    assert L.tmh_memcpy(got.ctypes.data, d_out, got.nbytes, 1, None) == 0
    L.tmh_free_device(d_in)
    L.tmh_free_device(d_out)
    corr.close()
    # the case mix this test is about, from the oracle's own f64 values
    a = sd.mean() / sd
    t = (np.log10(np.maximum(sites.astype(np.float64), 1e-10)) - mu) * a + np.mean(mu)
    with np.errstate(over="ignore"):
        v = 10.0 ** t
    assert (v >= 65536).any() and (v >= 2.0 ** 31).any() and np.isinf(v).any()
    assert ((v > 1) & (v < 65536)).any()
    for i, ((y, x), s) in enumerate(zip(shifts, sites)):
        want = orc.illuminati_chain(s, mu, sd, (y, x), res, lo, hi)
        d = np.abs(got[i].astype(np.int32) - want.astype(np.int32))
        assert d.max() <= 1, (i, int(d.max()))
        assert (d == 0).mean() > 0.99


@pytest.mark.parametrize("bounds", [(0, 65535), (300, 5000)])
def test_chain_without_log_transform(L, bounds):
    """log_transform=False (raw-intensity statistics): k_chain_u8t<LOG=false>
    -- no zero floor, values may be negative before the x86 cast -- against
    the oracle chain with log_transform=False; one column of tiny std drives
    values past 2^16 and 2^31 (refined in f64)."""
    import ctypes as C
    from tmlibrary_amd import hip
    from tmlibrary_amd.image import Corrector, align_window
    from tmlibrary_amd.synth import synth_sites_host
    H, W = 96, 256
    base = np.stack(synth_sites_host(6, H, W, seed=77)).astype(np.float64)
    mu = base.mean(axis=0)
    sd = base.std(axis=0) + 1.0
    sd[:, 40:48] = 1e-3
    sd[:, 44:46] = 1e-5
    sites = np.stack(synth_sites_host(4, H, W, seed=78))
    shifts = [(0, 0), (2, -3), (-1, 5), (1, 0)]
    res = (4, 4, 8, 8)
    wins = np.stack([align_window((H, W), y, x, *res, crop=False)[0] for y, x in shifts])
    lo, hi = bounds
    corr = Corrector(mu, sd, log_transform=False)
    d_in, d_out = C.c_void_p(), C.c_void_p()
    assert L.tmh_malloc_device(C.byref(d_in), sites.nbytes) == 0
    assert L.tmh_malloc_device(C.byref(d_out), sites.size) == 0
    assert L.tmh_memcpy(d_in, sites.ctypes.data, sites.nbytes, 0, None) == 0
    hip.check(L.tmh_correct_chain_u8_device(corr._h, d_in, d_out, len(sites), hip.ptr(wins), lo,
                                            hi, None))
    got = np.empty(sites.shape, np.uint8)
    assert L.tmh_memcpy(got.ctypes.data, d_out, got.nbytes, 1, None) == 0
    L.tmh_free_device(d_in)
    L.tmh_free_device(d_out)
    corr.close()
    for i, ((y, x), s) in enumerate(zip(shifts, sites)):
        want = orc.illuminati_chain(s, mu, sd, (y, x), res, lo, hi, log_transform=False)
        d = np.abs(got[i].astype(np.int32) - want.astype(np.int32))
        assert d.max() <= 1, (i, int(d.max()))
        assert (d == 0).mean() > 0.99


def test_chain_rejects_bad_windows(L):
    from tmlibrary_amd.image import Corrector, align_window
    g, wins = _chain_inputs()
    corr = Corrector(g["smooth_mean"], g["smooth_std"])
    bad = wins.copy()
    bad[0]["rows"] = 10 ** 6
    with pytest.raises(ValueError):
        corr.chain_u8(g["images"], bad, 10, 20)
    with pytest.raises(ValueError):
        corr.chain_u8(g["images"], wins, 20, 20)
    corr.close()
