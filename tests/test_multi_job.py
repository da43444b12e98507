"""corilla as one sharded job over all channels:
tmlibrary_amd/workflow/corilla/multi.py.

CPU (gloo, world 2 and 3): the orchestration -- batch order, contiguous
shards of the recorded site order, parallel decode of each rank's block, the
Welford + ordered-percentile merge, rank 0 writing the illumstats file -- with
a CPU statistics double (the oracle), against the oracle over the whole
channel.  GPU: the default GPU statistics in one process against the oracle.
"""
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import corilla_oracle as orc
from util import REPO

h5 = pytest.importorskip("tmlibrary_amd.models.file")
try:
    h5.h5lib()
except RuntimeError as e:  # libhdf5 absent on this host
    pytest.skip(str(e), allow_module_level=True)

SHAPE = (40, 56)
CHANNELS = {1: list(range(0, 7)), 2: list(range(100, 105))}


def _make_store(root):
    from tmlibrary_amd.models.file import ExperimentStore
    from tmlibrary_amd.synth import synth_sites_host
    d = os.path.join(root, "channel_image_files")
    os.makedirs(d, exist_ok=True)
    sites = {}
    for ch, ids in CHANNELS.items():
        imgs = synth_sites_host(len(ids), *SHAPE, seed=300 + ch, channel=ch)
        imgs[0][0, :5] = 0
        for fid, img in zip(ids, imgs):
            h5.write_channel_image(os.path.join(d, "channel_image_file_%d.h5" % fid), img, 4,
                                   chunks=(16, 24))
            sites[fid] = img
    return ExperimentStore(root), sites


def _batches():
    """create_run_batches (corilla/api.py:45-105) over the channels' file ids."""
    from tmlibrary_amd.workflow.corilla.api import IllumstatsCalculator
    calc = IllumstatsCalculator.__new__(IllumstatsCalculator)  # no store needed to batch
    return list(calc.create_run_batches(channel_files=CHANNELS))


class OracleChannelStats(object):
    """CPU double of multi.GpuChannelStats built on the oracle."""

    def __init__(self, dims):
        self.st = orc.OracleOnlineStatistics(dims)
        self.q = np.linspace(0, 100, 100000)
        self.site_pcts = []

    def update_batch(self, sites):
        for s in sites:
            self.st.update(s)
            self.site_pcts.append(orc.percentile_linear(s, self.q))
            self.local_hist = getattr(self, "local_hist", 0) + orc.histogram_u16(s)

    def merge(self, d, group=None):
        from test_distributed_gloo import HostOps
        from tmlibrary_amd.workflow.corilla.sharded import merge_shards
        ops = HostOps(self.st.n, self.st.mean, self.st._M2, self.site_pcts or [np.zeros(len(self.q))],
                      getattr(self, "local_hist", np.zeros(65536, np.uint64)))
        if not self.site_pcts:
            ops.site_pcts = []
        if d is not None:
            self.n = merge_shards(ops, d, group)
            acc = ops.acc.numpy()
        else:
            self.n = self.st.n
            acc = np.zeros(len(self.q))
            for p in self.site_pcts:  # site order
                acc += p
        self.mean = ops.mean.numpy().reshape(self.st.mean.shape)
        self.std = np.sqrt(ops.m2.numpy().reshape(self.st.mean.shape) / (self.n - 1))
        self.acc = acc
        self.histogram = ops.hist.numpy().astype(np.uint64)
        return self.n

    def container(self):
        from tmlibrary_amd.image import IllumstatsContainer, IllumstatsImage
        keys = orc.percentile_keys(3)
        vals = orc.percentile_values(self.acc, self.n)
        return IllumstatsContainer(IllumstatsImage(self.mean), IllumstatsImage(self.std),
                                   dict(zip(keys.tolist(), vals.tolist())))

    def close(self):
        pass


class Recorder(object):
    """stats_factory wrapper keeping every channel's statistics object, so
    the merged pooled histogram can be checked after the job."""

    def __init__(self, factory):
        self.factory = factory
        self.made = []

    def __call__(self, dims):
        st = self.factory(dims)
        self.made.append(st)
        return st


def _check_hist(made, sites):
    for st, ids in zip(made, CHANNELS.values()):
        want = sum((orc.histogram_u16(sites[i]) for i in ids), np.zeros(65536, np.uint64))
        assert np.array_equal(np.asarray(st.histogram, np.uint64), want), "pooled histogram"


def _check(results, sites, rtol=1e-6):
    for ch, ids in CHANNELS.items():
        ref = orc.run_illumstats([sites[i] for i in ids])
        cont = results[ch]
        assert np.allclose(cont.mean.array, ref.mean, rtol=rtol, atol=1e-12)
        assert np.allclose(cont.std.array, ref.std, rtol=rtol, atol=1e-12)
        want = orc.percentile_values(ref.percentile_sums, ref.n)
        got = np.array([cont.percentiles[k] for k in orc.percentile_keys(3).tolist()])
        assert np.array_equal(got, want)


def _worker(rank, world, port, root):
    import sys
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from tmlibrary_amd.models.file import ExperimentStore
    from tmlibrary_amd.workflow.corilla.multi import run_channels_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    store = ExperimentStore(root)
    rec = Recorder(OracleChannelStats)
    res = run_channels_sharded(store, _batches(), dist=dist, stats_factory=rec,
                               block=2, decode_threads=2)
    np.savez(os.path.join(root, "r%d.npz" % rank),
             **{"mean%d" % ch: c.mean.array for ch, c in res.items()},
             **{"std%d" % ch: c.std.array for ch, c in res.items()},
             **{"hist%d" % ch: st.histogram for ch, st in zip(CHANNELS, rec.made)})
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_job_gloo(tmp_path, world):
    from test_distributed_gloo import _free_port
    store, sites = _make_store(str(tmp_path))
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    for ch, ids in CHANNELS.items():
        ref = orc.run_illumstats([sites[i] for i in ids])
        for r in range(world):
            z = np.load(tmp_path / ("r%d.npz" % r))
            assert np.allclose(z["mean%d" % ch], ref.mean, rtol=1e-6, atol=1e-12)
            assert np.allclose(z["std%d" % ch], ref.std, rtol=1e-6, atol=1e-12)
            want = sum((orc.histogram_u16(sites[i]) for i in ids), np.zeros(65536, np.uint64))
            assert np.array_equal(z["hist%d" % ch], want), "merged pooled histogram"
        # rank 0 wrote the channel's illumstats file (4 datasets, unsmoothed)
        mean, std, keys, vals = h5.read_illumstats(store.illumstats_file(ch).location)
        assert np.allclose(mean, ref.mean, rtol=1e-6, atol=1e-12)
        assert np.array_equal(vals[np.argsort(keys)],
                              orc.percentile_values(ref.percentile_sums, ref.n))


def test_single_process_cpu_double(tmp_path):
    from tmlibrary_amd.workflow.corilla.multi import run_channels_sharded
    store, sites = _make_store(str(tmp_path))
    rec = Recorder(OracleChannelStats)
    res = run_channels_sharded(store, _batches(), dist=None, stats_factory=rec, block=3)
    _check(res, sites)
    _check_hist(rec.made, sites)


@pytest.mark.gpu
def test_single_process_gpu(tmp_path):
    from tmlibrary_amd.workflow.corilla.multi import run_channels_sharded
    from tmlibrary_amd.workflow.corilla.multi import GpuChannelStats
    store, sites = _make_store(str(tmp_path))
    rec = Recorder(lambda d: GpuChannelStats(d, 1, batch_size=3))
    res = run_channels_sharded(store, _batches(), dist=None, stats_factory=rec, block=3)
    _check(res, sites)
    _check_hist(rec.made, sites)


_RCCL_SCRIPT = r"""
import os, sys
sys.path.insert(0, {repo!r}); sys.path.insert(0, os.path.join({repo!r}, "tests"))
import torch, torch.distributed as dist
from test_multi_job import _make_store, _batches, _check, _check_hist, Recorder
from tmlibrary_amd.workflow.corilla.multi import GpuChannelStats, run_channels_sharded
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, init_method="tcp://127.0.0.1:{port}",
                        device_id=dev)
store, sites = _make_store({root!r})
rec = Recorder(lambda d: GpuChannelStats(d, 1, device=dev, merge_single=True))
res = run_channels_sharded(store, _batches(), dist=dist, block=3, device=dev, stats_factory=rec)
_check(res, sites)
_check_hist(rec.made, sites)  # through get -> RCCL all_reduce -> set
dist.destroy_process_group()
print("rccl merge ok")
"""


@pytest.mark.gpu
def test_single_rank_rccl_merge_path(tmp_path):
    """The GPU merge path (deferred percentiles, StatsOps, RCCL all-reduce,
    chunked chain, broadcast) in a one-rank NCCL/RCCL group."""
    import subprocess
    import sys
    from test_distributed_gloo import _free_port
    code = _RCCL_SCRIPT.format(repo=REPO, port=_free_port(), root=str(tmp_path))
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "rccl merge ok" in r.stdout


def _gpu_decode_worker(rank, world, port, root):
    """One rank of the sharded job on GPU 0 (ranks share it): its shard
    through the GPU inflate into GpuChannelStats, merged over gloo with
    host-staged device buffers."""
    import sys
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import torch
    from tmlibrary_amd.models.file import ExperimentStore
    from tmlibrary_amd.workflow.corilla.multi import GpuChannelStats, run_channels_sharded
    from tmlibrary_amd.workflow.corilla.sharded import HostStagedDist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    store = ExperimentStore(root)
    rec = Recorder(lambda d: GpuChannelStats(d, world, device=dev, batch_size=3))
    tm = {}
    res = run_channels_sharded(store, _batches(), dist=HostStagedDist(dist), stats_factory=rec,
                               block=3, device=dev, decode="gpu", device_block=2, timing=tm)
    keys = orc.percentile_keys(3).tolist()
    np.savez(os.path.join(root, "g%d.npz" % rank),
             **{"mean%d" % ch: c.mean.array for ch, c in res.items()},
             **{"std%d" % ch: c.std.array for ch, c in res.items()},
             **{"pct%d" % ch: np.array([c.percentiles[k] for k in keys]) for ch, c in res.items()},
             **{"hist%d" % ch: np.asarray(st.histogram, np.uint64)
                for ch, st in zip(CHANNELS, rec.made)},
             **{"gpu%d" % ch: np.array([t["sites"], t["gpu_decoded"]]) for ch, t in tm.items()})
    dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_job_gpu_decode_two_ranks(tmp_path):
    """two ranks sharing GPU 0, each decoding its
    contiguous shard of the reference-layout gzip files with the GPU inflate
    and updating on the device, merged (gloo, host-staged) -- equal to the
    single-process job with host decode: percentiles and pooled histograms
    bit-exact, mean/std within 1e-6 (tmlib/workflow/corilla/api.py:131-136,
    stats.py:64-121)."""
    from test_distributed_gloo import _free_port
    from tmlibrary_amd.workflow.corilla.multi import GpuChannelStats, run_channels_sharded
    store, sites = _make_store(str(tmp_path))
    rec = Recorder(lambda d: GpuChannelStats(d, 1, batch_size=3))
    ref = run_channels_sharded(store, _batches(), dist=None, stats_factory=rec, block=3,
                               decode="host")
    keys = orc.percentile_keys(3).tolist()
    world = 2
    mp.start_processes(_gpu_decode_worker, args=(world, _free_port(), str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    for ch, ids in CHANNELS.items():
        want_pct = np.array([ref[ch].percentiles[k] for k in keys])
        want_hist = np.asarray(rec.made[list(CHANNELS).index(ch)].histogram, np.uint64)
        for r in range(world):
            z = np.load(tmp_path / ("g%d.npz" % r))
            n_sites, n_gpu = z["gpu%d" % ch]
            assert n_gpu == n_sites > 0, "rank %d: every site of its shard through the GPU" % r
            assert np.array_equal(z["pct%d" % ch], want_pct)
            assert np.array_equal(z["hist%d" % ch], want_hist)
            assert np.allclose(z["mean%d" % ch], ref[ch].mean.array, rtol=1e-6, atol=1e-12)
            assert np.allclose(z["std%d" % ch], ref[ch].std.array, rtol=1e-6, atol=1e-12)
    _check(ref, sites)


class _HostFeeder(object):
    """CPU stand-in for DeviceSiteFeeder: host decode, then the statistics'
    update (the orchestration around the GPU inflate, without a GPU)."""

    def __init__(self, **kw):
        self.fed = 0

    def feed(self, paths, stats, strict=False):
        from tmlibrary_amd.models.file import read_channel_images
        stats.update_batch(read_channel_images(paths, 2).astype(np.uint16))
        self.fed += len(paths)
        return len(paths)


class OracleDeviceDouble(OracleChannelStats):
    """The oracle double with the attribute that selects the GPU decode path."""

    def update_device(self, *a, **k):  # never reached: the stand-in feeder updates on the host
        raise AssertionError("update_device")


def _empty_shard_worker(rank, world, port, root):
    import sys
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import tmlibrary_amd.models.device_decode as dd
    from tmlibrary_amd.models.file import ExperimentStore
    from tmlibrary_amd.workflow.corilla.multi import run_channels_sharded
    from test_multi_job import _HostFeeder as feeder_cls, OracleDeviceDouble as double
    dd.DeviceSiteFeeder = feeder_cls
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tm = {}
    res = run_channels_sharded(ExperimentStore(root), _batches(), dist=dist, stats_factory=double,
                               block=2, decode_threads=2, decode="gpu", timing=tm)
    np.savez(os.path.join(root, "e%d.npz" % rank),
             **{"mean%d" % ch: c.mean.array for ch, c in res.items()},
             **{"std%d" % ch: c.std.array for ch, c in res.items()},
             **{"n%d" % ch: np.array([tm[ch]["sites"], tm[ch]["gpu_decoded"]]) for ch in res})
    dist.destroy_process_group()


def test_sharded_job_empty_shard_gpu_decode(tmp_path):
    """with decode="gpu" and more ranks than a channel's
    files, the rank with an empty shard goes straight to the merge (no
    RawChunksUnsupported, no peer left waiting in a collective).  World 6
    over channels of 7 and 5 files: channel 2 leaves one rank empty."""
    from test_distributed_gloo import _free_port
    store, sites = _make_store(str(tmp_path))
    world = 6
    mp.start_processes(_empty_shard_worker, args=(world, _free_port(), str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    empty = 0
    for ch, ids in CHANNELS.items():
        ref = orc.run_illumstats([sites[i] for i in ids])
        got = 0
        for r in range(world):
            z = np.load(tmp_path / ("e%d.npz" % r))
            n_sites, n_fed = z["n%d" % ch]
            assert n_fed == n_sites, "every site of the shard through the (stand-in) GPU feeder"
            got += n_sites
            empty += n_sites == 0
            assert np.allclose(z["mean%d" % ch], ref.mean, rtol=1e-6, atol=1e-12)
            assert np.allclose(z["std%d" % ch], ref.std, rtol=1e-6, atol=1e-12)
        assert got == len(ids)
    assert empty >= 1
