"""CPU, world_size 2 (gloo): the multi-GPU merge sequencing of
tmlibrary_amd/workflow/corilla/sharded.py reproduces the single-process
statistics — Welford merge within 1e-6, percentile chain bit-exact.

The device kernels are replaced by a host-memory test double with the same
stage arithmetic; the GPU kernels themselves are covered by
test_gpu_parity.py::test_deferred_chain_and_merge_single_gpu."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from util import REPO, load_golden
from oracle import corilla_oracle as orc


class HostOps(object):
    """Test double of sharded.StatsOps on numpy/torch CPU state."""

    def __init__(self, n, mean, m2, site_pcts, hist, Q=None):
        self.n = int(n)
        self.hist = torch.tensor(np.asarray(hist, dtype=np.uint64).astype(np.int64))
        self.mean = torch.tensor(np.asarray(mean, dtype=np.float64).ravel())
        self.m2 = torch.tensor(np.asarray(m2, dtype=np.float64).ravel())
        self.site_pcts = [np.asarray(p, dtype=np.float64) for p in site_pcts]
        self.Q = self.site_pcts[0].size if Q is None else int(Q)  # Q: an empty shard's
        self.acc = None
        self.device = "cpu"

    def n_local(self):
        return self.n

    def empty_plane(self):
        return torch.empty(self.mean.numel(), dtype=torch.float64)

    def empty_acc(self):
        return torch.zeros(self.Q, dtype=torch.float64)

    def stage1(self, buf):
        buf.copy_(self.n * self.mean)

    def stage2(self, sum_nmean, n_total, m2c):
        mu = sum_nmean / n_total
        d = self.mean - mu
        m2c.copy_(self.m2 + self.n * d * d)
        self.mean = mu.clone()

    def stage3(self, n_total, sum_m2c):
        self.m2 = sum_m2c.clone()
        self.n = n_total

    def pct_accumulate(self, acc):
        a = acc.numpy().copy()
        for p in self.site_pcts:
            a += p  # in site order
        acc.copy_(torch.from_numpy(a))

    def pct_accumulate_range(self, acc_range, q_begin, q_count):
        a = acc_range.numpy().copy()
        for p in self.site_pcts:
            a += p[q_begin:q_begin + q_count]  # in site order
        acc_range.copy_(torch.from_numpy(a))

    def set_pct_sum(self, acc):
        self.acc = acc.clone()

    def empty_hist(self):
        return torch.empty(65536, dtype=torch.int64)

    def get_hist(self, buf):
        buf.copy_(self.hist)

    def set_hist(self, buf):
        self.hist = buf.clone()


class WholeOps(HostOps):
    """Ops without the ranged accumulate: the chain falls back to one step."""
    pct_accumulate_range = None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, out_dir, staged=False):
    import sys
    sys.path.insert(0, REPO)
    from oracle import corilla_oracle as orc
    from tmlibrary_amd.workflow.corilla.sharded import merge_shards, shard_bounds
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = load_golden(name)
    sites = list(g["sites"])
    a, b = shard_bounds(len(sites), world, rank)
    mine = sites[a:b]
    q = np.linspace(0, 100, 10 ** (int(g["decimals"]) + 2))
    st = orc.OracleOnlineStatistics(sites[0].shape, int(g["decimals"]))
    for s in mine:
        st.update(s)
    cls = WholeOps if name == "stats_small" and world == 2 else HostOps
    local_hist = sum((orc.histogram_u16(s) for s in mine), np.zeros(65536, np.uint64))
    ops = cls(st.n, st.mean, st._M2, [orc.percentile_linear(s, q) for s in mine], local_hist)
    if staged:  # the same merge through the host-staging facade (sharded.HostStagedDist)
        from tmlibrary_amd.workflow.corilla.sharded import HostStagedDist
        n_total = merge_shards(ops, HostStagedDist(dist))
    else:
        n_total = merge_shards(ops, dist)
    np.savez(os.path.join(out_dir, "r%d.npz" % rank), n=n_total, mean=ops.mean.numpy(),
             m2=ops.m2.numpy(), acc=ops.acc.numpy(), hist=ops.hist.numpy().astype(np.uint64))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,name,staged", [(2, "stats_medium", False), (2, "stats_small", False),
                                               (3, "stats_small", False), (2, "stats_medium", True)])
def test_merge_shards_gloo(tmp_path, world, name, staged):
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, name, str(tmp_path), staged), nprocs=world,
                       join=True, start_method="spawn")
    g = load_golden(name)
    want_var = g["std"] ** 2
    for r in range(world):
        z = np.load(tmp_path / ("r%d.npz" % r))
        assert int(z["n"]) == int(g["n"])
        assert np.allclose(z["mean"].reshape(g["mean"].shape), g["mean"], rtol=1e-6, atol=1e-12)
        var = z["m2"].reshape(g["mean"].shape) / (int(z["n"]) - 1)
        assert np.allclose(var, want_var, rtol=1e-6, atol=1e-12)
        assert np.array_equal(z["acc"], g["pct_sums"]), "chained percentile sum not bit-exact"
        want_hist = sum((orc.histogram_u16(s) for s in g["sites"]), np.zeros(65536, np.uint64))
        assert np.array_equal(z["hist"], want_hist), "merged histogram differs from the oracle's"


def test_chain_chunks_even_cover():
    from tmlibrary_amd.workflow.corilla.sharded import chain_chunks
    for Q in (1, 2, 7, 100, 1000, 100000):
        for w in (1, 2, 3, 8):
            spans = chain_chunks(Q, w)
            assert spans[0][0] == 0 and sum(n for _, n in spans) == Q
            assert all(a + n == b for (a, n), (b, _) in zip(spans, spans[1:]))
            assert all(a % 2 == 0 for a, _ in spans)


def test_shard_bounds_cover_in_order():
    from tmlibrary_amd.workflow.corilla.sharded import shard_bounds
    for n in (0, 1, 7, 3456, 13824):
        for w in (1, 2, 3, 8):
            spans = [shard_bounds(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))


def _multi_worker(rank, world, port, name, out_dir, whole):
    """Two jobs sharded over the same ranks (a rank's channels), merged with
    the batched collectives (sharded.merge_welford_multi / merge_counts_multi):
    job 0 = the golden's sites, job 1 = the same sites in reverse order."""
    import sys
    sys.path.insert(0, REPO)
    from oracle import corilla_oracle as orc
    from tmlibrary_amd.workflow.corilla.sharded import (merge_counts_multi, merge_welford_multi,
                                                         shard_bounds)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = load_golden(name)
    jobs = [list(g["sites"]), list(g["sites"])[::-1]]
    q = np.linspace(0, 100, 10 ** (int(g["decimals"]) + 2))
    ops_list = []
    for sites in jobs:
        a, b = shard_bounds(len(sites), world, rank)
        mine = sites[a:b]
        st = orc.OracleOnlineStatistics(sites[0].shape, int(g["decimals"]))
        for s in mine:
            st.update(s)
        local_hist = sum((orc.histogram_u16(s) for s in mine), np.zeros(65536, np.uint64))
        cls = WholeOps if whole else HostOps
        ops_list.append(cls(st.n, st.mean, st._M2, [orc.percentile_linear(s, q) for s in mine],
                            local_hist))
    n_totals = merge_welford_multi(ops_list, dist)
    merge_counts_multi(ops_list, dist)
    np.savez(os.path.join(out_dir, "m%d.npz" % rank), n=np.array(n_totals),
             **{"mean%d" % j: o.mean.numpy() for j, o in enumerate(ops_list)},
             **{"m2%d" % j: o.m2.numpy() for j, o in enumerate(ops_list)},
             **{"acc%d" % j: o.acc.numpy() for j, o in enumerate(ops_list)},
             **{"hist%d" % j: o.hist.numpy().astype(np.uint64) for j, o in enumerate(ops_list)})
    dist.destroy_process_group()


@pytest.mark.parametrize("world,whole", [(2, False), (3, False), (2, True)])
def test_merge_multi_jobs_gloo(tmp_path, world, whole):
    """Batched multi-job merges: each job's results equal its own sequential
    oracle -- Welford within 1e-6, percentile sums bit-exact (each job's sites
    in its own order through the shared chain), pooled histograms exact."""
    name = "stats_medium"
    mp.start_processes(_multi_worker, args=(world, _free_port(), name, str(tmp_path), whole),
                       nprocs=world, join=True, start_method="spawn")
    g = load_golden(name)
    jobs = [list(g["sites"]), list(g["sites"])[::-1]]
    refs = [orc.run_illumstats(s) for s in jobs]
    want_hist = sum((orc.histogram_u16(s) for s in g["sites"]), np.zeros(65536, np.uint64))
    for r in range(world):
        z = np.load(tmp_path / ("m%d.npz" % r))
        assert z["n"].tolist() == [len(jobs[0])] * 2
        for j, ref in enumerate(refs):
            assert np.allclose(z["mean%d" % j].reshape(ref.mean.shape), ref.mean, rtol=1e-6,
                               atol=1e-12)
            var = z["m2%d" % j].reshape(ref.mean.shape) / (len(jobs[j]) - 1)
            assert np.allclose(var, ref.std ** 2, rtol=1e-6, atol=1e-12)
            assert np.array_equal(z["acc%d" % j], ref.percentile_sums), (r, j)
            assert np.array_equal(z["hist%d" % j], want_hist)


# The N = 8 geometry of configs[2] (VERDICT r5 "next round" item 3): four
# channels, each channel's sites in 8 contiguous shards of the recorded site
# order (uneven, and one channel with fewer sites than ranks: empty shards),
# decimals 3 (Q = 100,000), merged with the batched collectives and the
# default chain (chain_chunks(Q, 8): 8 quantile chunks flowing down an 8-hop
# chain, [C, chunk] messages) -- the transport the first 8-GPU run uses,
# rehearsed on CPU (reference: corilla/api.py:64-105, one job per channel;
# stats.py:75-76, the sequential percentile sum the chain must keep).
W8_SITES = (19, 8, 5, 11)  # per channel
W8_SHAPE = (24, 40)


def _w8_sites(c):
    from tmlibrary_amd.synth import synth_sites_host
    return synth_sites_host(W8_SITES[c], *W8_SHAPE, seed=900 + c, channel=c)


def _w8_worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, REPO)
    from oracle import corilla_oracle as orc
    from tmlibrary_amd.workflow.corilla.sharded import (chain_chunks, merge_counts_multi,
                                                         merge_welford_multi, shard_bounds)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    q = np.linspace(0, 100, 100000)
    ops_list = []
    for c in range(len(W8_SITES)):
        sites = _w8_sites(c)
        a, b = shard_bounds(len(sites), world, rank)
        mine = sites[a:b]
        st = orc.OracleOnlineStatistics(W8_SHAPE, 3)
        for s in mine:
            st.update(s)
        local_hist = sum((orc.histogram_u16(s) for s in mine), np.zeros(65536, np.uint64))
        ops_list.append(HostOps(st.n, st.mean, st._M2, [orc.percentile_linear(s, q) for s in mine],
                                local_hist, Q=q.size))
    n_totals = merge_welford_multi(ops_list, dist)
    merge_counts_multi(ops_list, dist)
    np.savez(os.path.join(out_dir, "w8_%d.npz" % rank), n=np.array(n_totals),
             chunks=np.array(len(chain_chunks(q.size, world))),
             **{"mean%d" % j: o.mean.numpy() for j, o in enumerate(ops_list)},
             **{"m2%d" % j: o.m2.numpy() for j, o in enumerate(ops_list)},
             **{"acc%d" % j: o.acc.numpy() for j, o in enumerate(ops_list)},
             **{"hist%d" % j: o.hist.numpy().astype(np.uint64) for j, o in enumerate(ops_list)})
    dist.destroy_process_group()


def test_merge_multi_world8_geometry(tmp_path):
    world = 8
    mp.start_processes(_w8_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    refs = [orc.run_illumstats(_w8_sites(c)) for c in range(len(W8_SITES))]
    hists = [sum((orc.histogram_u16(s) for s in _w8_sites(c)), np.zeros(65536, np.uint64))
             for c in range(len(W8_SITES))]
    for r in range(world):
        z = np.load(tmp_path / ("w8_%d.npz" % r))
        assert int(z["chunks"]) == 8
        assert z["n"].tolist() == list(W8_SITES)
        for c, ref in enumerate(refs):
            assert np.allclose(z["mean%d" % c].reshape(W8_SHAPE), ref.mean, rtol=1e-6, atol=1e-12)
            std = np.sqrt(z["m2%d" % c].reshape(W8_SHAPE) / (W8_SITES[c] - 1))
            assert np.allclose(std, ref.std, rtol=1e-6, atol=1e-12)
            assert np.array_equal(z["acc%d" % c], ref.percentile_sums), (r, c)
            assert np.array_equal(z["hist%d" % c], hists[c]), (r, c)
