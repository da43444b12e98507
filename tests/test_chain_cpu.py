"""CPU checks of the illuminati-chain host logic and of the oracle against
the reference fixtures (align, map_uint8, chain)."""
import numpy as np
import pytest

from util import load_golden
from oracle import corilla_oracle as orc


def test_oracle_align_matches_reference():
    g = load_golden("align")
    for i, (y, x, b, t, r, l) in enumerate(g["cases"]):
        assert np.array_equal(orc.shift_and_crop(g["image"], y, x, b, t, r, l, crop=False),
                              g["padded"][i])
        assert np.array_equal(orc.shift_and_crop(g["image"], y, x, b, t, r, l, crop=True),
                              g["cropped_%d" % i])


def test_align_window_matches_reference_slicing():
    from tmlibrary_amd.image import align_window
    g = load_golden("align")
    img = g["image"]
    for i, (y, x, b, t, r, l) in enumerate(g["cases"]):
        for crop in (False, True):
            w, shape = align_window(img.shape, y, x, b, t, r, l, crop)
            w = w[()]
            out = np.zeros(shape, img.dtype)
            out[w["dst_r0"]:w["dst_r0"] + w["rows"], w["dst_c0"]:w["dst_c0"] + w["cols"]] = \
                img[w["src_r0"]:w["src_r0"] + w["rows"], w["src_c0"]:w["src_c0"] + w["cols"]]
            want = g["cropped_%d" % i] if crop else g["padded"][i]
            assert np.array_equal(out, want), (i, crop)


def test_align_window_numpy_edge_semantics():
    from tmlibrary_amd.image import align_window
    img = np.arange(100, dtype=np.uint16).reshape(10, 10)
    # img[-1:10] (1 row) pasted into aligned[-1:0] (0 rows): numpy broadcasts it away
    w, _ = align_window((10, 10), 0, 0, 0, -1, 0, 0, crop=False)
    assert w[()]["rows"] == 0
    assert not orc.shift_and_crop(img, 0, 0, 0, -1, 0, 0, crop=False).any()
    # img[-2:10] (2 rows) into aligned[-2:0]: numpy raises, so does the window
    with pytest.raises(Exception):
        orc.shift_and_crop(img, 0, 0, 0, -2, 0, 0, crop=False)
    with pytest.raises(Exception):
        align_window((10, 10), 0, 0, 0, -2, 0, 0, crop=False)
    # empty extraction (shift larger than the residue window) pads everything
    w, shape = align_window((10, 10), -4, 0, 0, 0, 0, 0, crop=False)
    assert w[()]["rows"] == 0 and shape == (10, 10)
    assert not orc.shift_and_crop(img, -4, 0, 0, 0, 0, 0, crop=False).any()


def test_scale_formula_matches_reference_lut():
    """The per-pixel form the GPU evaluates (one f64 multiply; linspace's end
    point forced to 255; n = 1 gives 0) reproduces the reference's LUTs."""
    g = load_golden("map_uint8")
    v = np.arange(65536, dtype=np.int64)
    for (lo, hi), lut in zip(g["bounds"], g["luts"]):
        lo, hi = int(lo), int(hi)
        n = hi - lo
        step = 255.0 / (n - 1) if n > 1 else 0.0
        i = v - lo
        out = np.trunc(i.astype(np.float64) * step).astype(np.int64)
        out[i == n - 1] = 255
        if n == 1:
            out[i == 0] = 0
        out[v < lo] = 0
        out[v >= hi] = 255
        assert np.array_equal(out.astype(np.uint8), lut), (lo, hi)
        assert np.array_equal(orc.map_to_uint8(v.astype(np.uint16).reshape(256, 256), lo,
                                               hi).ravel(), lut)


def test_oracle_chain_matches_reference():
    g = load_golden("chain")
    for img, (y, x), want in zip(g["images"], g["shifts"], g["scaled"]):
        got = orc.illuminati_chain(img, g["smooth_mean"], g["smooth_std"], (int(y), int(x)),
                                   tuple(int(r) for r in g["residues"]), int(g["clip_lo"]),
                                   int(g["clip_hi"]))
        assert np.array_equal(got, want)
