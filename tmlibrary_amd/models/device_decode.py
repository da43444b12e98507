"""GPU decode of channel image files: HDF5 gzip chunks inflated on the device.

The reference reads every site with h5py (tmlib/models/file.py:322-351,
tmlib/readers.py:367-389), i.e. libhdf5's deflate filter runs zlib's inflate
on the host, one chunk after another -- on the GPU box's 16 granted cores that
caps the corilla job at ~290 sites/s (profiles/r3/input_path_threads_r3l.jsonl).
Here the host only copies the still-compressed chunks out of the files
(libtmh5 ``tmh5_read_raw_chunks``: HDF5 metadata under its lock, the bytes by
parallel ``pread``), the compressed bytes cross PCIe, and libtmhip inflates
every chunk on the GPU (``tmh_inflate_device``: one lane per zlib stream,
byte-identical to zlib, Adler-32 checked) and places the chunks' rows into a
device ``[n, H, W]`` site buffer (``tmh_place_chunks_device``) that the
statistics pass reads in place.

No CPU fallback inside: a file the GPU path cannot take (not chunked with the
deflate filter only) raises ``RawChunksUnsupported`` and the caller decides
(``IllumstatsCalculator`` decodes such blocks on the host, as the reference).
"""
from __future__ import annotations

import ctypes as C
import time

import numpy as np

from tmlibrary_amd import hip
from tmlibrary_amd.models.file import RawChunksUnsupported, read_raw_chunks


class DeviceChunkDecoder(object):
    """Inflate blocks of channel image files into device site buffers.

    Device buffers (compressed bytes, chunk table, raw chunks, statuses) and
    pinned host staging are kept across calls and grown on demand.  ``decode``
    enqueues on ``stream`` and returns; ``check()`` (called by the next
    ``decode`` of the same slot, or explicitly) raises if any chunk failed."""

    def __init__(self, device=None, stream=None, slots=2, n_threads=None):
        import torch
        self.torch = torch
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.stream = stream if stream is not None else torch.cuda.Stream(self.device)
        # the H2D copies on their own stream: block k+1's compressed bytes
        # cross PCIe while block k inflates on ``stream``
        self.copy_stream = torch.cuda.Stream(self.device)
        self.n_threads = n_threads
        self.slots = [dict() for _ in range(max(1, slots))]
        self.k = 0
        # host seconds: waiting for a slot's previous block, reading raw chunks
        # (libhdf5 metadata + pread), the whole decode() call
        self.times = {"slot_wait": 0.0, "read": 0.0, "call": 0.0}

    def _grow(self, slot, name, n, dtype, pinned=False):
        torch = self.torch
        t = slot.get(name)
        if t is None or t.numel() < n:
            n = max(int(n * 1.25), 1)
            if pinned:
                t = torch.empty(n, dtype=dtype, pin_memory=True)
            else:
                t = torch.empty(n, dtype=dtype, device=self.device)
            slot[name] = t
        return t

    def decode(self, paths, out_ptr, n_out=None, expect=None):
        """Decode ``paths`` into the device buffer at ``out_ptr`` ([n, H, W] of
        the files' dtype, contiguous).  Returns (H, W, elem_bytes).  The work is
        queued on ``self.stream``; the slot's buffers are reused two calls later
        (the caller orders its consumers after ``self.stream``).

        ``expect`` = (H, W, elem_bytes) the buffer was sized for: a block of
        another shape raises ValueError (the reference's broadcast error in
        OnlineStatistics.update), of another element size
        RawChunksUnsupported -- both before anything is queued."""
        torch = self.torch
        L = hip.lib()
        t0 = time.perf_counter()
        slot = self.slots[self.k % len(self.slots)]
        self.k += 1
        if slot.get("event") is not None:
            slot["event"].synchronize()  # the slot's previous block is done
            self._raise_failed(slot)
        t1 = time.perf_counter()
        hb = slot.get("h_blob")
        ht = slot.get("h_tab")
        blob, table, geom = read_raw_chunks(
            paths, self.n_threads, None if hb is None else hb.numpy(),
            None if ht is None else ht.numpy().view(hip.ZCHUNK_DTYPE))
        t2 = time.perf_counter()
        H, W, es, cr, cc = geom
        if expect is not None:
            eh, ew, ees = expect
            if (H, W) != (eh, ew):
                raise ValueError("operands could not be broadcast together with shapes (%d,%d) "
                                 "(%d,%d)" % (H, W, eh, ew))
            if es != ees:
                raise RawChunksUnsupported("%d-byte pixels in a %d-byte job" % (es, ees))
        n = len(table)
        if hb is None or blob.ctypes.data != hb.data_ptr():  # grown: pin the new size
            hb = self._grow(slot, "h_blob", blob.nbytes, torch.uint8, pinned=True)
            hb.numpy()[:blob.nbytes] = blob
            slot["h_blob"] = hb
        tb = table.view(np.uint8).reshape(-1)
        if ht is None or table.ctypes.data != ht.data_ptr():
            esz = hip.ZCHUNK_DTYPE.itemsize  # whole entries, so the pinned bytes view as a table
            ht = torch.empty(max(int(n * 1.25), 1) * esz, dtype=torch.uint8, pin_memory=True)
            ht.numpy()[:tb.nbytes] = tb
            slot["h_tab"] = ht
        d_src = self._grow(slot, "d_src", blob.nbytes + 16, torch.uint8)
        d_tab = self._grow(slot, "d_tab", tb.nbytes, torch.uint8)
        raw_bytes = n * cr * cc * es
        d_raw = self._grow(slot, "d_raw", raw_bytes, torch.uint8)
        d_st = self._grow(slot, "d_status", n, torch.int32)
        raw_max = int(table["raw_len"].max()) if n else 0
        scr_bytes = int(L.tmh_inflate_scratch_bytes(n, raw_max))
        d_scr = self._grow(slot, "d_scratch", max(scr_bytes, 4), torch.uint8)
        prev = slot.get("inflated")  # the slot's device buffers are free once its last block inflated
        with torch.cuda.stream(self.copy_stream):
            if prev is not None:
                self.copy_stream.wait_event(prev)
            d_src[:blob.nbytes].copy_(hb[:blob.nbytes], non_blocking=True)
            d_tab[:tb.nbytes].copy_(ht[:tb.nbytes], non_blocking=True)
            copied = torch.cuda.Event()
            copied.record(self.copy_stream)
        self.stream.wait_event(copied)
        sp = C.c_void_p(self.stream.cuda_stream)
        hip.check(L.tmh_inflate_device(C.c_void_p(d_src.data_ptr()), blob.nbytes,
                                       C.c_void_p(d_tab.data_ptr()), n, raw_max,
                                       C.c_void_p(d_raw.data_ptr()), raw_bytes,
                                       C.c_void_p(d_scr.data_ptr()), d_scr.numel(),
                                       C.c_void_p(d_st.data_ptr()), sp))
        hip.check(L.tmh_place_chunks_device(C.c_void_p(d_raw.data_ptr()),
                                            C.c_void_p(d_tab.data_ptr()), n, H, W, es, cr, cc,
                                            C.c_void_p(int(out_ptr)), sp))
        inflated = torch.cuda.Event()
        inflated.record(self.stream)
        slot["inflated"] = inflated
        h_st = self._grow(slot, "h_status", n, torch.int32, pinned=True)
        with torch.cuda.stream(self.stream):
            h_st[:n].copy_(d_st[:n], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        slot["event"] = ev
        slot["n"] = n
        slot["paths"] = list(paths)
        slot["images"] = table["image"].copy()
        t3 = time.perf_counter()
        self.times["slot_wait"] += t1 - t0
        self.times["read"] += t2 - t1
        self.times["call"] += t3 - t0
        return H, W, es

    def _raise_failed(self, slot):
        n = slot.get("n", 0)
        if not n:
            return
        st = slot["h_status"][:n].numpy()
        bad = np.nonzero(st)[0]
        slot["n"] = 0
        if bad.size:
            i = int(bad[0])
            path = slot["paths"][int(slot["images"][i])]
            raise IOError("%s: chunk %d: %s (%d of %d chunks failed to inflate)"
                          % (path, i, hip.Z_STATUS.get(int(st[i]), "error %d" % st[i]),
                             bad.size, n))

    def reset(self):
        """Forget every slot's pending block (after a job aborted part way):
        waits for the queued work, drops the statuses unread, so a later job
        never raises an earlier job's inflate error."""
        for slot in self.slots:
            ev = slot.get("event")
            if ev is not None:
                try:
                    ev.synchronize()
                finally:
                    slot["event"] = None
            slot["n"] = 0

    def check(self):
        """Wait for every queued block; raise if a chunk failed to inflate."""
        for slot in self.slots:
            if slot.get("event") is not None:
                slot["event"].synchronize()
                self._raise_failed(slot)


class DeviceSiteFeeder(object):
    """A run of channel image files into a statistics object through the GPU
    inflate, in file order (the corilla job's input path, SURVEY.md §8(f)
    rank 1; reference: tmlib/workflow/corilla/api.py:131-136 reads and
    updates site by site).

    Two device site buffers of ``block`` sites: block k+1's host chunk read
    and H2D copy overlap block k's inflate (decoder stream) and statistics
    update (statistics stream S, ``stats.update_device``); a buffer is reused
    once S has read it.  Buffers, decoder and streams are kept across calls
    (one feeder per job runner).  ``feed`` returns how many of the files (a
    prefix) went into ``stats``: with ``strict`` False a block the GPU path
    cannot read (``RawChunksUnsupported``, raised before anything of the block
    is queued) ends the GPU run there and the caller decodes the rest on the
    host -- every site counted once, in order."""

    def __init__(self, device=None, block=64, n_threads=None):
        import torch
        self.torch = torch
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.block = max(1, int(block))
        self.n_threads = n_threads
        self._key = None
        self.dec = None
        self.last_zero_counts = None

    def _ensure(self, H, W):
        torch = self.torch
        if self._key != (H, W):
            B = self.block
            self.bufs = [torch.empty((B, H, W), dtype=torch.int16, device=self.device)
                         for _ in range(2)]
            self.dec = DeviceChunkDecoder(device=self.device, slots=2, n_threads=self.n_threads)
            self.S = torch.cuda.Stream(self.device)
            self._key = (H, W)

    def feed(self, paths, stats, strict=False, on_block=None):
        """``stats``: has ``image_dimensions`` and ``update_device(ptr, n,
        stream=, zero_counts=)``.  ``on_block(k, n)`` (optional) is called as
        files [k, k + n) are queued (the caller's per-site logging)."""
        torch = self.torch
        from tmlibrary_amd.models.file import channel_image_shape
        from tmlibrary_amd.workflow.corilla.stats import log_zero_warnings
        if not paths:
            return 0
        H, W, dt = channel_image_shape(paths[0])
        if np.dtype(dt) != np.uint16 or (H, W) != tuple(stats.image_dimensions):
            if strict:
                raise RawChunksUnsupported("GPU decode takes uint16 sites of the job's shape")
            return 0
        self._ensure(H, W)
        dec, S, bufs, B = self.dec, self.S, self.bufs, self.block
        zc = torch.zeros(len(paths), dtype=torch.int64, pin_memory=True).numpy()
        used = [None, None]
        done, ok = 0, False
        try:
            for k in range(0, len(paths), B):
                b = (k // B) % 2
                if used[b] is not None:
                    dec.stream.wait_event(used[b])  # S has read the buffer's previous block
                blk = paths[k:k + B]
                try:
                    dec.decode(blk, bufs[b].data_ptr(), expect=(H, W, 2))
                except RawChunksUnsupported:
                    if strict:
                        raise
                    break
                ready = torch.cuda.Event()
                ready.record(dec.stream)
                S.wait_event(ready)
                if on_block is not None:
                    on_block(k, len(blk))
                stats.update_device(bufs[b].data_ptr(), len(blk), stream=S.cuda_stream,
                                    zero_counts=zc[k:k + len(blk)])
                used[b] = torch.cuda.Event()
                used[b].record(S)
                done = k + len(blk)
            S.synchronize()
            dec.check()  # a chunk that failed to inflate raises here
            ok = True
        finally:
            if not ok:  # aborted: nothing of this run may surface in a later one
                S.synchronize()
                dec.reset()
        log_zero_warnings(zc[:done])
        self.last_zero_counts = zc[:done]
        return done
