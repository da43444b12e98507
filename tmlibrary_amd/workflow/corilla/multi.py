"""corilla as ONE multi-GPU job over all channels.

The reference schedules one single-process GC3Pie job per channel
(tmlib/workflow/corilla/api.py:45-105 ``create_run_batches``, :115-146
``run_job``) and the site order inside a channel is whatever the database
query returns.  Here every rank of one ``torchrun`` job walks the same list of
channel batches (``IllumstatsCalculator.create_run_batches`` order) and, per
channel:

1. takes the contiguous block ``shard_bounds(n, world, rank)`` of the batch's
   file list -- the list itself is the recorded site order, so the merged
   result is the reference's sequential result over that order;
2. decodes its block and accumulates it: with ``decode`` "auto" (default)
   or "gpu" the rank's compressed chunks are read by the host, inflated on
   the rank's own GPU and fed to the statistics in place
   (models/device_decode.py ``DeviceSiteFeeder``, as ``run_job``), with
   "host" (or files the GPU path cannot read, from the first such file on)
   by the parallel host inflate reader (``update_batch``);
3. merges the partial statistics (Welford all-reduce, ordered percentile
   chain, histogram all-reduce: ``sharded.merge_shards``), so every rank
   holds identical results (``stats.histogram``: the channel's pooled counts);
4. rank 0 writes the ``IllumstatsFile`` (4-dataset HDF5 layout).

The per-channel statistics object is pluggable (``stats_factory``): the
default runs on the GPU through libtmhip; tests plug a CPU double in to check
the orchestration (tests/test_multi_job.py).
"""
from __future__ import annotations

import logging

import numpy as np

from tmlibrary_amd.image import IllumstatsContainer
from tmlibrary_amd.models.file import (RawChunksUnsupported, channel_image_shape,
                                       read_channel_images)
from tmlibrary_amd.workflow.corilla.sharded import merge_shards, shard_bounds

logger = logging.getLogger(__name__)


class GpuChannelStats(object):
    """One rank's share of one channel on the GPU: ``OnlineStatistics`` in
    deferred-percentile mode + ``StatsOps`` for the merge."""

    def __init__(self, image_dimensions, world, device=None, batch_size=32, merge_single=False):
        from tmlibrary_amd import hip
        from tmlibrary_amd.workflow.corilla.stats import OnlineStatistics
        # merge_single: run the deferred-percentile merge path even with one
        # rank (exercises the multi-GPU code on a one-GPU box)
        self.merging = world > 1 or merge_single
        flags = hip.TMH_STATS_DEFERRED_PCT if self.merging else 0
        self.st = OnlineStatistics(image_dimensions, batch_size=batch_size, flags=flags)
        self.world = world
        self.device = device

    @property
    def image_dimensions(self):
        return self.st.image_dimensions

    def update_batch(self, sites):
        self.st.update_batch(sites)

    def update_device(self, dev_sites, n_sites, stream=None, zero_counts=None):
        """Device-resident sites (the GPU inflate's output), in order."""
        self.st.update_device(dev_sites, n_sites, stream=stream, zero_counts=zero_counts)

    def merge(self, dist, group=None):
        if not self.merging or dist is None:
            self.histogram = self.st.histogram
            return self.st.n
        import torch
        from tmlibrary_amd import hip
        from tmlibrary_amd.workflow.corilla.sharded import StatsOps
        st = self.st
        st._flush()
        h, w = st.image_dimensions
        dev = self.device if self.device is not None else torch.device("cuda",
                                                                         torch.cuda.current_device())
        ops = StatsOps(hip.lib(), st._h, h * w, len(st._q), dev)
        # one created stream for the merge's launches, copies and collectives
        # (sharded.StatsOps: the default stream does not order against them)
        ms = torch.cuda.Stream(dev)
        ms.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(ms):
            n_total = merge_shards(ops, dist, group, int_device=dev)
        ms.synchronize()
        st.refresh()  # the handle holds the whole channel's merged state (n = n_total)
        self.histogram = st.histogram  # pooled over every rank's sites
        return n_total

    def container(self):
        return IllumstatsContainer(self.st.mean, self.st.std, self.st.percentiles)

    def close(self):
        self.st.close()


def run_channels_sharded(store, batches, dist=None, group=None, stats_factory=None,
                         block=32, decode_threads=None, device=None, decode="auto",
                         device_block=64, timing=None):
    """Run every channel batch as one sharded job; returns {channel_id:
    IllumstatsContainer} (identical on every rank).  ``dist`` is
    torch.distributed (or None for one process).  ``decode``: "auto" / "gpu"
    (GPU inflate of the rank's shard, ``device_block`` files per device
    block; "gpu" raises ``RawChunksUnsupported`` for files it cannot read)
    or "host".  The GPU path needs statistics with ``update_device`` (the
    default GpuChannelStats); others decode on the host.  ``timing`` (a
    dict, optional) receives per channel the seconds of the rank's
    input + update phase and of the merge."""
    import time
    if decode not in ("auto", "gpu", "host"):
        raise ValueError('decode must be "auto", "gpu" or "host"')
    world = dist.get_world_size(group) if dist is not None else 1
    rank = dist.get_rank(group) if dist is not None else 0
    if stats_factory is None:
        def stats_factory(dims):
            return GpuChannelStats(dims, world, device=device, batch_size=block)
    feeder = None
    results = {}
    for batch in batches:
        ids = [f[0] if isinstance(f, (list, tuple)) else f
               for f in batch["channel_image_files_ids"]]
        paths = [store.channel_image_file(i).location for i in ids]
        H, W, _ = channel_image_shape(paths[0])  # the dataset's shape: no decode needed
        dims = (H, W)
        a, b = shard_bounds(len(paths), world, rank)
        logger.info("channel %s: rank %d of %d takes sites [%d, %d) of %d",
                    batch["channel_id"], rank, world, a, b, len(paths))
        stats = stats_factory(dims)
        t0 = time.perf_counter()
        try:
            start = a
            if decode != "host" and b > a and hasattr(stats, "update_device"):
                if feeder is None:
                    from tmlibrary_amd.models.device_decode import DeviceSiteFeeder
                    feeder = DeviceSiteFeeder(device=device, block=device_block,
                                              n_threads=decode_threads)
                start = a + feeder.feed(paths[a:b], stats, strict=decode == "gpu")
                if start < b:
                    logger.info("channel %s: files from %d on decoded on the host",
                                batch["channel_id"], start)
            elif decode == "gpu" and not hasattr(stats, "update_device"):
                # (an empty shard -- more ranks than files -- has nothing to
                # decode and goes straight to the merge its peers wait in)
                raise RawChunksUnsupported("decode='gpu' needs statistics with update_device")
            for i in range(start, b, block):
                sites = read_channel_images(paths[i:min(b, i + block)], decode_threads)
                if sites.dtype == np.uint8:
                    sites = sites.astype(np.uint16)
                stats.update_batch(sites)
            t1 = time.perf_counter()
            stats.merge(dist, group)
            cont = stats.container()
            if timing is not None:
                timing[batch["channel_id"]] = {"sites": b - a, "gpu_decoded": start - a,
                                               "input_update_s": t1 - t0,
                                               "merge_s": time.perf_counter() - t1}
        finally:
            stats.close()
        if rank == 0:
            store.illumstats_file(batch["channel_id"]).put(cont)
        results[batch["channel_id"]] = cont
    return results
