"""CPU: host-side behaviour of the drop-in API (types, errors, metadata flags)."""
import numpy as np
import pytest

from util import load_golden
from tmlibrary_amd.image import ChannelImage, IllumstatsContainer, IllumstatsImage
from tmlibrary_amd.metadata import ChannelImageMetadata, IllumstatsImageMetadata


def test_channel_image_type_checks():
    ChannelImage(np.zeros((4, 5), np.uint16))
    ChannelImage(np.zeros((4, 5), np.uint8))
    with pytest.raises(TypeError):
        ChannelImage([[1, 2]])
    with pytest.raises(ValueError):
        ChannelImage(np.zeros(5, np.uint16))
    with pytest.raises(ValueError):
        ChannelImage(np.zeros((4, 5), np.float64))
    with pytest.raises(ValueError):
        ChannelImage(np.zeros((4, 5), np.uint32))
    with pytest.raises(TypeError):
        ChannelImage(np.zeros((4, 5), np.uint16), metadata=object())


def test_illumstats_image_type_checks():
    IllumstatsImage(np.zeros((3, 3)))
    with pytest.raises(ValueError):
        IllumstatsImage(np.zeros((3, 3), np.float32))
    with pytest.raises(TypeError):
        IllumstatsImage(np.zeros((3, 3)), metadata=ChannelImageMetadata(1, 1, 1, 0, 0))
    with pytest.raises(TypeError):
        IllumstatsContainer(np.zeros((3, 3)), IllumstatsImage(np.zeros((3, 3))), {})


def test_metadata_flags_and_types():
    md = ChannelImageMetadata(channel_id=3, site_id=1, cycle_id=0, tpoint=0, zplane=0)
    assert md.is_corrected is False and md.is_clipped is False and md.is_rescaled is False
    with pytest.raises(TypeError):
        md.channel_id = "3"
    with pytest.raises(TypeError):
        md.is_corrected = 1
    im = IllumstatsImageMetadata(channel_id=3)
    assert im.is_smoothed is False
    with pytest.raises(TypeError):
        im.is_smoothed = "yes"


def test_get_closest_percentile_matches_golden():
    g = load_golden("stats_small")
    pct = dict(zip(g["pct_keys"].tolist(), g["pct_values"].tolist()))
    c = IllumstatsContainer(IllumstatsImage(np.zeros((2, 2))), IllumstatsImage(np.ones((2, 2))), pct)
    assert c.get_closest_percentile(99.9) == pct[99.9]
    assert c.get_closest_percentile(0.001) == pct[0.001]
    assert c.get_closest_percentile(-5) == pct[0.0]
    assert c.get_closest_percentile(500) == pct[100.0]


def test_stats_rejects_bad_decimals():
    from tmlibrary_amd.workflow.corilla.stats import OnlineStatistics
    with pytest.raises(ValueError):
        OnlineStatistics((4, 4), decimals=4)
    with pytest.raises(ValueError):
        OnlineStatistics((4, 4), decimals=-1)


def test_create_run_batches(tmp_path, caplog):
    from tmlibrary_amd.models.file import ExperimentStore
    from tmlibrary_amd.workflow.corilla.api import SITE_LIMIT, IllumstatsCalculator
    calc = IllumstatsCalculator(1, store=ExperimentStore(str(tmp_path)))
    files = {3: list(range(50)), 1: list(range(1000, 1000 + SITE_LIMIT + 7)), 2: []}
    with caplog.at_level("WARNING"):
        batches = list(calc.create_run_batches(channel_files=files, seed=0))
    assert [b["channel_id"] for b in batches] == [1, 3]
    assert [b["id"] for b in batches] == [1, 2]
    big = [f[0] for f in batches[0]["channel_image_files_ids"]]
    assert len(big) == SITE_LIMIT and len(set(big)) == SITE_LIMIT
    assert set(big) <= set(files[1])
    assert [f[0] for f in batches[1]["channel_image_files_ids"]] == files[3]
    msgs = " ".join(r.message for r in caplog.records)
    assert "only 50 images" in msgs and 'no image files found for channel "2"' in msgs


@pytest.mark.parametrize("prefetch,batch", [(1, 3), (2, 4), (4, 2), (3, 32)])
def test_run_job_read_ahead_order(tmp_path, prefetch, batch):
    """IllumstatsCalculator._blocks: several blocks decoded at once into a
    bounded pool of reused buffers, yielded in file order."""
    import os

    from tmlibrary_amd.models import file as h5
    from tmlibrary_amd.workflow.corilla.api import IllumstatsCalculator
    store = h5.ExperimentStore(str(tmp_path))
    os.makedirs(tmp_path / "channel_image_files")
    rng = np.random.default_rng(prefetch * 10 + batch)
    want = {}
    for fid in range(13):
        a = rng.integers(0, 65536, (24, 40), dtype=np.uint16)
        h5.write_channel_image(store.channel_image_file(fid).location, a)
        want[fid] = a
    order = [7, 3, 12, 0, 1, 2, 11, 10, 4, 5, 6, 8, 9]
    calc = IllumstatsCalculator(1, store=store, batch_size=batch, prefetch=prefetch,
                                decode_threads=3)
    for rep in range(2):  # the second job reuses the buffers
        got_ids = []
        for ids, sites in calc._blocks(order):
            assert sites.shape == (len(ids), 24, 40)
            for fid, s in zip(ids, sites):
                assert np.array_equal(s, want[fid]), (rep, fid)
            got_ids += list(ids)
        assert got_ids == order
    # two live generators on one calculator: each owns its buffers
    g1, g2 = calc._blocks(order), calc._blocks(order[::-1])
    for (i1, s1), (i2, s2) in zip(g1, g2):
        for fid, s in zip(i1, s1):
            assert np.array_equal(s, want[fid]), ("interleaved", fid)
        for fid, s in zip(i2, s2):
            assert np.array_equal(s, want[fid]), ("interleaved reverse", fid)
    # abandoning the generator early does not hang
    gen = calc._blocks(order)
    next(gen)
    gen.close()
    # an unreadable file surfaces in the caller, and the workers stop
    os.remove(store.channel_image_file(12).location)
    with pytest.raises((IOError, OSError, KeyError, ValueError)):
        for _ in calc._blocks(order):
            pass
