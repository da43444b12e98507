"""Multi-GPU illumination statistics: sites sharded across ranks, one process per GPU.

The reference runs one single-threaded process per channel and never
exchanges data inside a channel (tmlib/workflow/corilla/api.py:64-105,
:115-146).  Here one channel's sites are split into contiguous blocks in site
order, one block per rank; every rank streams its block through the same
kernels as a single GPU, then the partial states are merged:

  Welford   Chan et al.'s pairwise combine written as two sums, so one RCCL
            all-reduce per quantity merges any number of ranks, identically
            on every rank:  mean = sum_r n_r mean_r / n,
                            M2   = sum_r [M2_r + n_r (mean_r - mean)^2]
  percentiles  the f64 accumulator travels rank 0 -> 1 -> ... -> N-1 and each
            rank adds its own sites in order, reproducing the reference's
            sequential ``_percentiles +=`` bit for bit (a plain all-reduce sum
            would reassociate it); the last rank broadcasts the result.
  histogram  all-reduce(sum) of the pooled 65,536-bin counts (integer sums:
            exact in any order), so every rank's ``OnlineStatistics.histogram``
            is the whole channel's.

Collectives use ``torch.distributed`` (backend "nccl" = RCCL over xGMI on
MI355X) on device buffers; the arithmetic runs in libtmhip kernels through
``StatsOps``.  ``merge_shards`` only sequences collectives, so the same code
is exercised on CPU with the gloo backend and a host-memory ``ops`` test
double (tests/test_distributed_gloo.py).
"""
from __future__ import annotations

import ctypes as C

import numpy as np


class StatsOps(object):
    """libtmhip operations on one rank's ``tmh_stats`` handle (device buffers
    are torch tensors; launches go on torch's current stream)."""

    def __init__(self, lib, handle, npx, n_quantiles, device):
        import torch
        self.torch = torch
        self.L = lib
        self.h = handle
        self.npx = int(npx)
        self.Q = int(n_quantiles)
        self.device = device

    def _stream(self):
        # torch's collectives and copies and these launches must share one
        # ordered stream: the default (null) stream cannot be named through
        # the C-ABI (NULL there means the handle's own stream, which does not
        # synchronise with it), so the merge must run under a created stream
        h = self.torch.cuda.current_stream(self.device).cuda_stream
        if not h:
            raise RuntimeError("StatsOps: run the merge under a non-default torch stream "
                               "(with torch.cuda.stream(...)): the default stream does not "
                               "order against the statistics handle's stream")
        return C.c_void_p(h)

    def _chk(self, rc):
        from tmlibrary_amd import hip
        hip.check(rc)

    def empty_plane(self):
        return self.torch.empty(self.npx, dtype=self.torch.float64, device=self.device)

    def empty_acc(self):
        return self.torch.zeros(self.Q, dtype=self.torch.float64, device=self.device)

    def n_local(self):
        n = C.c_int64()
        self._chk(self.L.tmh_stats_get_n(self.h, C.byref(n)))
        return n.value

    def stage1(self, buf):
        self._chk(self.L.tmh_stats_merge_stage1(self.h, C.c_void_p(buf.data_ptr()), self._stream()))

    def stage2(self, sum_nmean, n_total, m2c):
        self._chk(self.L.tmh_stats_merge_stage2(self.h, C.c_void_p(sum_nmean.data_ptr()), n_total,
                                                C.c_void_p(m2c.data_ptr()), self._stream()))

    def stage3(self, n_total, sum_m2c):
        self._chk(self.L.tmh_stats_merge_stage3(self.h, n_total, C.c_void_p(sum_m2c.data_ptr()),
                                                self._stream()))

    def pct_accumulate(self, acc):
        self._chk(self.L.tmh_stats_pct_accumulate(self.h, C.c_void_p(acc.data_ptr()),
                                                  self._stream()))

    def pct_accumulate_range(self, acc_range, q_begin, q_count):
        self._chk(self.L.tmh_stats_pct_accumulate_range(
            self.h, C.c_void_p(acc_range.data_ptr()), int(q_begin), int(q_count), self._stream()))

    def set_pct_sum(self, acc):
        self._chk(self.L.tmh_stats_set_pct_sum(self.h, C.c_void_p(acc.data_ptr()), self._stream()))

    def empty_hist(self):
        # int64 on the wire (counts < 2**63; RCCL/gloo sum int64 exactly)
        return self.torch.empty(65536, dtype=self.torch.int64, device=self.device)

    def get_hist(self, buf):
        self._chk(self.L.tmh_stats_get_hist_device(self.h, C.c_void_p(buf.data_ptr()),
                                                   self._stream()))

    def set_hist(self, buf):
        self._chk(self.L.tmh_stats_set_hist_device(self.h, C.c_void_p(buf.data_ptr()),
                                                   self._stream()))


class HostStagedDist(object):
    """``torch.distributed`` facade that runs the merge collectives of device
    buffers on a CPU (gloo) process group: each call copies the buffer to
    host memory (``Tensor.cpu()`` waits for torch's current stream, where the
    StatsOps launches were queued), runs the gloo collective and copies the
    result back on the current stream.  For ranks that share one GPU -- RCCL
    needs a GPU per rank -- and for hosts without RCCL; ``merge_welford`` /
    ``merge_counts`` / ``merge_shards`` take it in place of the module."""

    def __init__(self, dist):
        self._d = dist
        self.ReduceOp = dist.ReduceOp

    def get_rank(self, group=None):
        return self._d.get_rank(group)

    def get_world_size(self, group=None):
        return self._d.get_world_size(group)

    def barrier(self, group=None):
        self._d.barrier(group=group)

    def all_reduce(self, t, op=None, group=None):
        h = t.cpu()
        self._d.all_reduce(h, op=self._d.ReduceOp.SUM if op is None else op, group=group)
        t.copy_(h)

    def send(self, t, dst, group=None):
        self._d.send(t.cpu(), dst=dst, group=group)

    def recv(self, t, src, group=None):
        import torch
        h = torch.empty(t.shape, dtype=t.dtype)
        self._d.recv(h, src=src, group=group)
        t.copy_(h)

    def broadcast(self, t, src, group=None):
        h = t.cpu()
        self._d.broadcast(h, src=src, group=group)
        t.copy_(h)


class _NoTimer(object):
    def __call__(self, name):
        return self

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


_NO_TIMER = _NoTimer()


def merge_welford(ops, dist, group=None, int_device=None, n_total=None, timer=None):
    """All-reduce merge of every rank's Welford state (identical on all ranks).
    Returns the global site count.  ``n_total`` (optional) is the global site
    count when the caller already knows it (e.g. from the shard bounds): it
    saves the count all-reduce, whose host read would block the issuing
    thread until this rank's statistics pass has finished.  ``timer(name)``
    (optional) is a context manager wrapped around each collective (bench.py
    times them one by one)."""
    import torch
    timer = timer or _NO_TIMER
    if n_total is None:
        dev = int_device if int_device is not None else getattr(ops, "device", "cpu")
        n_t = torch.tensor([ops.n_local()], dtype=torch.int64, device=dev)
        with timer("allreduce_n"):
            dist.all_reduce(n_t, group=group)
        n_total = int(n_t.item())
    n_total = int(n_total)
    if n_total > 0:
        buf = ops.empty_plane()
        ops.stage1(buf)
        with timer("allreduce_nmean"):
            dist.all_reduce(buf, group=group)
        m2c = ops.empty_plane()
        ops.stage2(buf, n_total, m2c)
        with timer("allreduce_m2c"):
            dist.all_reduce(m2c, group=group)
        ops.stage3(n_total, m2c)
    return n_total


def chain_chunks(n_quantiles, world, chunks=None):
    """Even-aligned quantile ranges for the pipelined rank chain: with C
    chunks the chain takes (N + C - 1) chunk-steps instead of N full steps."""
    Q = int(n_quantiles)
    if chunks is None:
        # a chunk's pass is bounded below by the in-order f64 chain over the
        # rank's sites (~0.06 ms at 3,456 sites), so more chunks than ranks
        # only lengthen the pipeline's fill
        chunks = 1 if world <= 1 else min(max(2, world), 16)
    chunks = max(1, min(int(chunks), max(1, Q // 2)))
    edges = [((Q * i // chunks) // 2) * 2 for i in range(chunks)] + [Q]
    return [(a, b - a) for a, b in zip(edges[:-1], edges[1:]) if b > a]


def merge_percentiles(ops, dist, group=None, chunks=None, timer=None):
    """Ordered percentile chain: the f64 accumulator travels rank 0 -> N-1,
    each rank adding its own sites in order (bit-exact sequential sum), and
    the last rank broadcasts it.  The accumulator is split into quantile
    chunks that flow down the chain as a pipeline (rank r adds chunk c while
    rank r-1 adds chunk c+1); every quantile still sees the ranks' sites in
    global site order."""
    timer = timer or _NO_TIMER
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    acc = ops.empty_acc()
    ranged = getattr(ops, "pct_accumulate_range", None) is not None
    spans = chain_chunks(acc.numel(), world, chunks) if ranged else [(0, acc.numel())]
    for q0, qn in spans:
        part = acc[q0:q0 + qn]
        if rank > 0:
            with timer("chain_recv"):
                dist.recv(part, src=rank - 1, group=group)
        if ranged:
            ops.pct_accumulate_range(part, q0, qn)
        else:
            ops.pct_accumulate(acc)
        if rank < world - 1:
            with timer("chain_send"):
                dist.send(part, dst=rank + 1, group=group)
    with timer("broadcast_pct"):
        dist.broadcast(acc, src=world - 1, group=group)
    ops.set_pct_sum(acc)


def merge_histogram(ops, dist, group=None, timer=None):
    """All-reduce of the pooled per-site histograms (exact integer sums)."""
    timer = timer or _NO_TIMER
    buf = ops.empty_hist()
    ops.get_hist(buf)
    with timer("allreduce_hist"):
        dist.all_reduce(buf, group=group)
    ops.set_hist(buf)


def merge_counts(ops, dist, group=None, chunks=None, timer=None):
    """The merges that need every site's histogram: the ordered percentile
    chain and the pooled-histogram all-reduce (after the fused correct pass
    in the split pipeline)."""
    merge_percentiles(ops, dist, group, chunks, timer)
    merge_histogram(ops, dist, group, timer)


def merge_shards(ops, dist, group=None, int_device=None):
    """Merge every rank's partial statistics into identical global state
    (Welford all-reduce merge, the ordered percentile chain and the
    histogram all-reduce).

    ``ops`` provides n_local/empty_plane/empty_acc/stage1-3/pct_accumulate/
    set_pct_sum/empty_hist/get_hist/set_hist on this rank's state; ``dist``
    is torch.distributed.  Returns the global site count.
    """
    n_total = merge_welford(ops, dist, group, int_device)
    merge_counts(ops, dist, group)
    return n_total


def _rows(plane, n):
    """[n, *plane.shape] buffer like ``plane`` (dtype, device): one row per job."""
    import torch
    return torch.empty((n,) + tuple(plane.shape), dtype=plane.dtype, device=plane.device)


def merge_welford_multi(ops_list, dist, group=None, n_totals=None, timer=None, int_device=None):
    """``merge_welford`` for several jobs at once (a rank's channels, each
    sharded over the same ranks): every job's stage output is a row of one
    buffer, so the merge is TWO all-reduces for all jobs (C x 44 MB each at
    2160 x 2560) instead of two per job -- fewer, larger collectives over
    xGMI.  Arithmetic and results are merge_welford's, job by job.  Returns
    the jobs' global site counts."""
    import torch
    timer = timer or _NO_TIMER
    C = len(ops_list)
    if n_totals is None:
        dev = int_device if int_device is not None else getattr(ops_list[0], "device", "cpu")
        n_t = torch.tensor([ops.n_local() for ops in ops_list], dtype=torch.int64, device=dev)
        with timer("allreduce_n"):
            dist.all_reduce(n_t, group=group)
        n_totals = [int(v) for v in n_t.tolist()]
    n_totals = [int(v) for v in n_totals]
    live = [c for c in range(C) if n_totals[c] > 0]
    if live:
        buf = _rows(ops_list[0].empty_plane(), C)
        for c in live:
            ops_list[c].stage1(buf[c])
        with timer("allreduce_nmean"):
            dist.all_reduce(buf, group=group)
        m2c = _rows(ops_list[0].empty_plane(), C)
        for c in live:
            ops_list[c].stage2(buf[c], n_totals[c], m2c[c])
        with timer("allreduce_m2c"):
            dist.all_reduce(m2c, group=group)
        for c in live:
            ops_list[c].stage3(n_totals[c], m2c[c])
    return n_totals


def merge_counts_multi(ops_list, dist, group=None, chunks=None, timer=None):
    """``merge_counts`` for several jobs at once: one ordered percentile chain
    whose messages carry every job's quantile chunk (a [C, chunk] buffer per
    step, each job's sites added in its own site order: bit-exact per job),
    one broadcast of the [C, Q] sums and one all-reduce of the [C, 65,536]
    pooled histograms -- instead of a chain and two collectives per job."""
    timer = timer or _NO_TIMER
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    C = len(ops_list)
    acc0 = ops_list[0].empty_acc()
    Q = acc0.numel()
    acc = _rows(acc0, C)
    acc.zero_()
    ranged = getattr(ops_list[0], "pct_accumulate_range", None) is not None
    spans = chain_chunks(Q, world, chunks) if ranged else [(0, Q)]
    for q0, qn in spans:
        part = _rows(acc0[:qn], C)
        part.zero_()
        if rank > 0:
            with timer("chain_recv"):
                dist.recv(part, src=rank - 1, group=group)
        for c, ops in enumerate(ops_list):
            if ranged:
                ops.pct_accumulate_range(part[c], q0, qn)
            else:
                ops.pct_accumulate(part[c])
        if rank < world - 1:
            with timer("chain_send"):
                dist.send(part, dst=rank + 1, group=group)
        acc[:, q0:q0 + qn].copy_(part)
    with timer("broadcast_pct"):
        dist.broadcast(acc, src=world - 1, group=group)
    for c, ops in enumerate(ops_list):
        ops.set_pct_sum(acc[c])
    h = _rows(ops_list[0].empty_hist(), C)
    for c, ops in enumerate(ops_list):
        ops.get_hist(h[c])
    with timer("allreduce_hist"):
        dist.all_reduce(h, group=group)
    for c, ops in enumerate(ops_list):
        ops.set_hist(h[c])


def shard_bounds(n_sites, world, rank):
    """Contiguous block of sites for ``rank`` (site order preserved)."""
    base, extra = divmod(int(n_sites), int(world))
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)
