"""corilla step: illumination statistics per channel (run phase).

Mirrors tmlib/workflow/corilla/api.py:31-146 ``IllumstatsCalculator``:
``run_job(batch)`` reads the channel's site images in the order of
``batch['channel_image_files_ids']``, takes the image dimensions from the
first file, updates ``OnlineStatistics`` with every site, and writes an
``IllumstatsFile`` with mean, std and the percentile dict.

Differences by design (database/cluster orchestration is out of scope): files
are resolved through an ``ExperimentStore`` (tmlibrary_amd/models/file.py)
instead of SQLAlchemy sessions, and the images are read ahead on a
background thread so HDF5 decode overlaps the GPU updates.
"""
from __future__ import annotations

import logging
import queue
import threading

import numpy as np

from tmlibrary_amd.image import IllumstatsContainer
from tmlibrary_amd.models.file import (ExperimentStore, RawChunksUnsupported,
                                       channel_image_shape, default_decode_threads,
                                       read_channel_images)
from tmlibrary_amd.workflow.corilla.stats import OnlineStatistics

logger = logging.getLogger(__name__)

#: corilla/api.py:69 — sites per channel beyond which the reference subsamples
SITE_LIMIT = 20000


def _block_buffer(n, H, W, dtype):
    """[n, H, W] host buffer for a decoded block: page-locked when torch can
    pin memory (the H2D copy is then pure DMA, no CPU staging), else
    pageable."""
    try:
        import torch
        tdt = torch.int16 if np.dtype(dtype) == np.uint16 else torch.uint8
        t = torch.empty((n, H, W), dtype=tdt, pin_memory=True)
        return t.numpy().view(dtype)
    except Exception:  # no torch, or no pinnable memory (no device)
        return np.empty((n, H, W), dtype)


def _file_id(fid):
    # batch JSON stores SQLAlchemy row tuples as [[id], ...]
    if isinstance(fid, (list, tuple)):
        return fid[0]
    return fid


class IllumstatsCalculator(object):
    """Calculation of illumination statistics (corilla/api.py:31-146)."""

    def __init__(self, experiment_id, store=None, batch_size=32, prefetch=2, decode_threads=None,
                 decode="auto", device_block=64):
        """prefetch: blocks of ``batch_size`` files decoded concurrently ahead of
        the GPU update; decode_threads: inflate workers over all of them (None:
        the cores granted, models/file.py:granted_cores).

        decode: where the sites' gzip chunks are inflated -- "gpu": the host
        reads the compressed chunks, the GPU inflates them into a device
        buffer the statistics pass reads in place (models/device_decode.py;
        ``device_block`` files per block, two blocks in flight; 64 sites of
        h5py's 256 chunks fill the GPU's ~16k resident inflate streams once:
        run_job 2,472 sites/s on 1,536 sites against 2,380 with 128, and a
        0.1 s instead of 0.3 s fixed cost, profiles/r4/run_job_device_block_r4db.txt); "host":
        libhdf5 + zlib on the cores; "auto": the GPU path when the files
        allow it (uint16, chunked with the deflate filter only), else host."""
        self.experiment_id = experiment_id
        if store is None:
            raise ValueError("an ExperimentStore is required (no database in this build)")
        if not isinstance(store, ExperimentStore):
            raise TypeError('Argument "store" must have type ExperimentStore.')
        self.store = store
        self.batch_size = batch_size
        self.prefetch = prefetch
        self.decode_threads = decode_threads
        self._buffers = {}  # (block, H, W, dtype) -> reused block buffers (idle sets)
        self._buffers_lock = threading.Lock()
        if decode not in ("auto", "gpu", "host"):
            raise ValueError('decode must be "auto", "gpu" or "host"')
        self.decode = decode
        self.device_block = max(1, int(device_block))
        self._dev = None  # DeviceSiteFeeder, kept across jobs (buffers, decoder, streams)
        self.last_timing = None  # the last run_job's phases (seconds)

    def create_run_batches(self, args=None, channel_files=None, channel_names=None, seed=None):
        """One job per channel (corilla/api.py:45-105).

        ``channel_files`` maps channel id -> list of channel image file ids
        (the database query of the reference).  More than SITE_LIMIT files:
        a random subset of SITE_LIMIT (the reference orders by
        ``random()``; ``seed`` makes the draw reproducible); fewer than 100:
        warning; none: warning and no batch.  Yields the batch dicts
        ``{'id', 'channel_image_files_ids', 'channel_id'}``.
        """
        import random
        channel_files = channel_files if channel_files is not None else {}
        names = channel_names or {}
        rng = random.Random(seed)
        count = 0
        for ch_id in sorted(channel_files):
            name = names.get(ch_id, str(ch_id))
            file_ids = list(channel_files[ch_id])
            n = len(file_ids)
            if n > SITE_LIMIT:
                logger.info('using a subset of image files (n=%d) to calculate '
                            'illumination statistics for channel "%s"', SITE_LIMIT, name)
                file_ids = rng.sample(file_ids, SITE_LIMIT)
            elif n < 100:
                logger.warning('calculation of illumnation statistics for channel "%s" on '
                               'only %d images - this may introduce artifacts upon '
                               'illumination correction', name, n)
            if not file_ids:
                logger.warning('no image files found for channel "%s"', name)
                continue
            count += 1
            yield {"id": count, "channel_image_files_ids": [[f] for f in file_ids],
                   "channel_id": ch_id}

    def _blocks(self, file_ids):
        """Yield (file ids, [n, H, W] sites) in order, ``batch_size`` files at a
        time.  ``prefetch`` blocks are decoded at once,
        each by its share of ``decode_threads`` inflate workers, into a bounded
        pool of reused (pinned when torch can pin) block buffers, so decode of
        the next blocks overlaps the GPU update of the current one and no
        block pays fresh-page faults.  A worker takes a free buffer BEFORE it
        claims the next block index: buffers then go to blocks in order and a
        run-ahead worker can never hold the buffer the next block needs.

        A yielded array is a view of a reused buffer: it is valid until the
        generator is resumed.  Each live generator owns its buffer set (taken
        from the calculator's idle sets under a lock and given back when it
        ends), so concurrent run_job calls or a caller that keeps an earlier
        generator open never share buffers."""
        step = max(1, self.batch_size)
        blocks = [file_ids[i:i + step] for i in range(0, len(file_ids), step)]
        if not blocks:
            return
        paths = [[self.store.channel_image_file(f).location for f in b] for b in blocks]
        H, W, dt = channel_image_shape(paths[0][0])
        total = self.decode_threads or default_decode_threads()
        inflight = max(1, min(self.prefetch, len(blocks)))
        per = max(1, total // inflight)
        # the block buffers are kept on the calculator: pinning ~0.35 GB per
        # buffer costs more than decoding a short job
        key = (step, H, W, np.dtype(dt).str)
        with self._buffers_lock:  # this generator's own set (another may be live)
            sets = self._buffers.get(key, [])
            bufs = sets.pop() if sets else []
        while len(bufs) < min(inflight + 1, len(blocks)):
            bufs.append(_block_buffer(step, H, W, dt))
        pool = queue.Queue()
        for b in bufs[:min(inflight + 1, len(blocks))]:
            pool.put(b)
        lock = threading.Lock()
        ready = threading.Condition(lock)
        results = {}
        state = {"next": 0, "stop": False}

        def worker():
            while True:
                buf = pool.get()
                with lock:
                    k = state["next"]
                    if state["stop"] or k >= len(blocks):
                        pool.put(buf)
                        return
                    state["next"] = k + 1
                try:
                    item = read_channel_images(paths[k], per, out=buf)
                except BaseException as e:  # surface I/O errors in the caller
                    item = e
                with ready:
                    results[k] = (buf, item)
                    ready.notify_all()

        threads = [threading.Thread(target=worker, daemon=True) for _ in range(inflight)]
        for t in threads:
            t.start()
        try:
            for k in range(len(blocks)):
                with ready:
                    while k not in results:
                        ready.wait()
                    buf, item = results.pop(k)
                if isinstance(item, BaseException):
                    raise item
                yield blocks[k], item
                pool.put(buf)  # the consumer's update has returned: reuse
        finally:
            with lock:
                state["stop"] = True
            for _ in threads:
                pool.put(None)  # wake workers waiting for a buffer
            for t in threads:
                t.join()
            with self._buffers_lock:  # idle again: the next generator may reuse it
                self._buffers.setdefault(key, []).append(bufs)

    def _update_device(self, file_ids, stats):
        """The job's sites through the GPU inflate into the statistics, in order
        (models/device_decode.py DeviceSiteFeeder: block k+1's host chunk read
        and H2D copy overlap block k's inflate and statistics update).

        Returns how many of ``file_ids`` (a prefix) went into ``stats``.  With
        decode="auto" a block the GPU path cannot read (another layout or
        element size: ``RawChunksUnsupported``, raised before anything of the
        block is queued) ends the GPU path there, and the caller continues on
        the host from the first file not taken -- every site is counted once,
        in the job's order."""
        from tmlibrary_amd.models.device_decode import DeviceSiteFeeder
        paths = [self.store.channel_image_file(f).location for f in file_ids]
        if self._dev is None:
            self._dev = DeviceSiteFeeder(block=self.device_block, n_threads=self.decode_threads)

        def on_block(k, n):
            for fid in file_ids[k:k + n]:
                logger.info("update statistics for image: %d", fid)

        done = self._dev.feed(paths, stats, strict=self.decode == "gpu", on_block=on_block)
        if done < len(file_ids):
            logger.info("channel image files from %d on not GPU-decodable: decoding the rest "
                        "on the host", done)
        return done

    def run_job(self, batch, assume_clean_state=False):
        """corilla/api.py:115-146.  The reference reads the first site to learn
        the image dimensions; here the file's dataset shape gives them without
        decoding it (~40 ms per job).  ``last_timing`` holds the job's phases
        in seconds (sites -> statistics, read-back, illumstats write)."""
        import time
        t0 = time.perf_counter()
        file_ids = [_file_id(f) for f in batch["channel_image_files_ids"]]
        logger.info("calculate illumination statistics")
        H, W, _ = channel_image_shape(self.store.channel_image_file(file_ids[0]).location)
        stats = OnlineStatistics(image_dimensions=(H, W), batch_size=self.batch_size)
        timing = {}
        try:
            start = 0  # files already in the statistics (GPU path)
            if self.decode != "host":
                start = self._update_device(file_ids, stats)
            if start < len(file_ids):
                for ids, sites in self._blocks(file_ids[start:]):
                    for fid in ids:
                        logger.info("update statistics for image: %d", fid)
                    stats.update_batch(sites)
            t1 = time.perf_counter()
            timing["sites"] = t1 - t0
            stats_file = self.store.illumstats_file(batch["channel_id"])
            logger.info("write calculated statistics to file")
            illumstats = IllumstatsContainer(stats.mean, stats.std, stats.percentiles)
            t2 = time.perf_counter()
            timing["read_back"] = t2 - t1
            stats_file.put(illumstats)
            timing["write"] = time.perf_counter() - t2
        finally:
            stats.close()
        self.last_timing = timing
        return illumstats
