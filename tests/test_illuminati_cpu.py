"""CPU: illuminati's clip bounds from a channel's percentiles
(tmlib/workflow/illuminati/api.py:119-164, image.py:1195-1213) --
tmlibrary_amd.workflow.illuminati.clip_bounds -- against the bounds the
golden generator derived for the apply fixtures (tests/golden/make_goldens.py:
get_closest_percentile(0.001) and max(get_closest_percentile(99.9), 700) over
the reference's own percentile dict), a dim channel that hits the 700 floor,
an 8-bit channel (255 floor) and the clip_value / no-clip branches."""
import numpy as np
import pytest

from util import load_golden
from oracle import corilla_oracle as orc


def _container(mean, std, pct_sums, n, decimals=3):
    from tmlibrary_amd.image import IllumstatsContainer, IllumstatsImage
    keys = orc.percentile_keys(decimals)
    vals = orc.percentile_values(pct_sums, n)
    return IllumstatsContainer(IllumstatsImage(np.asarray(mean, np.float64)),
                               IllumstatsImage(np.asarray(std, np.float64)),
                               dict(zip(keys.tolist(), vals.tolist())))


@pytest.mark.parametrize("name", ["apply_log", "apply_nolog"])
def test_clip_bounds_match_the_apply_goldens(name):
    """The apply fixtures' clip bounds came from the reference's percentile
    dict of the same 6 statistics sites (make_goldens.py 'apply cases'); the
    oracle's statistics of those sites equal the fixture's (pinned), so their
    percentiles are the reference's."""
    from tmlibrary_amd.synth import synth_sites_host
    from tmlibrary_amd.workflow.illuminati import clip_bounds
    g = load_golden(name)
    st = orc.run_illumstats(synth_sites_host(6, 96, 128, seed=1111))
    assert np.allclose(st.mean, g["stats_mean"], rtol=1e-12, atol=0)
    cont = _container(st.mean, st.std, st.percentile_sums, st.n)
    lo, hi = clip_bounds(cont)
    assert (lo, hi) == (int(g["clip_lo"]), int(g["clip_hi"]))
    assert hi >= 700


def test_clip_bounds_dim_channel_floor():
    """A dim ("empty") 16-bit channel: its 99.9th percentile is below 700, so
    clip_max is raised to 700 (api.py:142-153); clip_min stays its 0.001st."""
    from tmlibrary_amd.synth import synth_sites_host
    from tmlibrary_amd.workflow.illuminati import clip_bounds
    dim = [(s // 8).astype(np.uint16) for s in synth_sites_host(4, 64, 80, seed=77)]
    st = orc.run_illumstats(dim)
    cont = _container(st.mean, st.std, st.percentile_sums, st.n)
    p999 = cont.get_closest_percentile(99.9)
    assert p999 < 700
    lo, hi = clip_bounds(cont)
    assert hi == 700 and lo == cont.get_closest_percentile(0.001)
    assert lo == orc.get_closest_percentile(cont.percentiles, 0.001)
    # the same channel declared 8-bit: the floor is 255 (below its p99.9 here)
    lo8, hi8 = clip_bounds(cont, bit_depth=8)
    assert hi8 == max(p999, 255) and lo8 == lo


def test_clip_bounds_u8_golden():
    """An 8-bit channel from the u8 statistics fixture (the reference's
    percentile values): floor 255."""
    from tmlibrary_amd.workflow.illuminati import clip_bounds
    g = load_golden("stats_u8")
    cont = _container(g["mean"], g["std"], g["pct_sums"], int(g["n"]), int(g["decimals"]))
    vals = dict(zip(orc.percentile_keys(int(g["decimals"])).tolist(), g["pct_values"].tolist()))
    assert cont.percentiles == vals  # the fixture's own percentile values
    lo, hi = clip_bounds(cont, bit_depth=8)
    assert hi == max(orc.get_closest_percentile(vals, 99.9), 255)
    assert lo == orc.get_closest_percentile(vals, 0.001)


def test_clip_bounds_other_branches():
    from tmlibrary_amd.workflow.illuminati import clip_bounds
    assert clip_bounds(None, clip=True, clip_value=1234) == (0, 1234)  # api.py:156-160
    assert clip_bounds(None, clip=False) == (0, 65535)                 # api.py:161-164
    assert clip_bounds(None, clip=False, bit_depth=8) == (0, 255)
