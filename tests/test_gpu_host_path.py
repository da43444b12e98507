"""GPU: the host-buffer entry points (tmh_stats_update, tmh_correct_u16) stage
numpy sites through two pinned slots per direction and overlap the copy of
chunk k with the DMA and kernels of chunk k-1.  These tests run stacks that
span several chunks (so both slots are reused) and check the pipelined result
against the one-chunk-per-call path bit for bit and against the oracle."""
import logging

import numpy as np
import pytest

from util import assert_close_rel, assert_dn
from oracle import corilla_oracle as orc

pytestmark = pytest.mark.gpu


def _sites(n, h=40, w=56, seed=3):
    from tmlibrary_amd.synth import synth_sites_host
    s = np.stack(synth_sites_host(n, h, w, seed=seed))
    s[1, 0, :5] = 0          # zero pixels -> one warning per site that has them
    s[n - 1, 3, 3] = 0
    s[2, 1, 1] = 65535
    return np.ascontiguousarray(s)


@pytest.mark.parametrize("batch", [1, 2, 3])
def test_stats_update_batch_pipelined(batch, caplog):
    from tmlibrary_amd.image import ChannelImage
    from tmlibrary_amd.workflow.corilla.stats import OnlineStatistics
    sites = _sites(7)
    ref = OnlineStatistics(sites[0].shape, batch_size=batch)
    for s in sites:  # per-site update: one chunk per tmh_stats_update call
        ref.update(ChannelImage(s.copy()))
    st = OnlineStatistics(sites[0].shape, batch_size=batch)
    caplog.clear()
    with caplog.at_level(logging.WARNING):
        st.update_batch(sites)  # one call, ceil(7 / batch) chunks through the pinned slots
    assert sum("image contains zero values" in r.getMessage() for r in caplog.records) == \
        sum(bool((s == 0).any()) for s in sites)
    assert st.n == ref.n == 7
    # same chunking -> the same launches -> bitwise equal
    assert np.array_equal(st.mean.array, ref.mean.array)
    assert np.array_equal(st.std.array, ref.std.array)
    assert np.array_equal(st.percentile_sums, ref.percentile_sums)
    want = orc.OracleOnlineStatistics(sites[0].shape)
    for s in sites:
        want.update(s)
    assert_close_rel(st.mean.array, want.mean)
    assert_close_rel(st.std.array, want.std)
    assert np.array_equal(st.percentile_sums, want.percentile_sums)
    # a second call reuses the (retired) slots
    st.update_batch(sites[:3])
    assert st.n == 10
    st.close()
    ref.close()


@pytest.mark.parametrize("n", [1, 16, 37])
def test_correct_u16_pipelined(n):
    from tmlibrary_amd.image import Corrector
    sites = _sites(max(n, 3), seed=11)[:n]
    rng = np.random.default_rng(5)
    mean = 2.0 + rng.random(sites.shape[1:]) * 0.5
    std = 0.1 + rng.random(sites.shape[1:]) * 0.05
    corr = Corrector(mean, std)
    got = corr.apply(sites)  # chunks of 16 sites, two slots per direction
    one = np.stack([corr.apply(s) for s in sites])
    assert np.array_equal(got, one)
    for s, g in zip(sites, got):
        want = orc.correct_illumination(s, mean, std, True)
        assert_dn(g, want)
    clipped = corr.apply(sites, clip=(120, 3000))
    assert np.array_equal(clipped, np.clip(got, 120, 3000))
    corr.close()


def test_correct_into_out_buffer():
    from tmlibrary_amd.image import Corrector
    sites = _sites(20, seed=13)
    rng = np.random.default_rng(6)
    corr = Corrector(2.0 + rng.random(sites.shape[1:]), 0.1 + 0.05 * rng.random(sites.shape[1:]))
    want = corr.apply(sites)
    out = np.full_like(sites, 7)
    assert corr.apply(sites, out=out) is out
    assert np.array_equal(out, want)
    with pytest.raises(ValueError):
        corr.apply(sites, out=np.empty((20, 40, 55), np.uint16))
    with pytest.raises(ValueError):
        corr.apply(sites, out=sites)
    corr.close()
