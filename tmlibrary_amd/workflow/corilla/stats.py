"""Online illumination statistics on MI355X.

Drop-in for tmlib/workflow/corilla/stats.py:35-121 (``OnlineStatistics``):
per-pixel Welford mean/variance over log10-transformed site images and the
running sum of per-site intensity percentiles.  State lives in HBM inside a
``tmh_stats`` handle; ``update`` stages sites in a host batch and flushes
them to the GPU in one launch group (Welford pass + histogram/percentile
pass + in-order percentile accumulation).

Behavioural notes vs the reference
  * ``update`` raises ``ValueError`` for an image whose shape differs from
    ``image_dimensions`` before touching any state (the reference fails in
    numpy broadcasting after the percentile sum was already updated).
  * The 'image contains zero values' warning (stats.py:81-82) is logged when
    the site is flushed to the GPU, not at the ``update`` call.
  * The inf-skip branch (stats.py:86-88) cannot trigger for unsigned-integer
    images, the only type ``ChannelImage`` admits; it is not modelled.
"""
from __future__ import annotations

import ctypes as C
import functools
import logging

import numpy as np

from tmlibrary_amd import hip
from tmlibrary_amd.image import ChannelImage, IllumstatsImage
from tmlibrary_amd.workflow.corilla.quantiles import quantile_table, stats_log10_lut

logger = logging.getLogger(__name__)

#: sites staged on the host per GPU flush
DEFAULT_BATCH = 32


def log_zero_warnings(zero_counts):
    """stats.py:81-82: one 'image contains zero values' warning per site with a
    zero pixel (log-transformed updates)."""
    for _ in range(int(np.count_nonzero(np.asarray(zero_counts)))):
        logger.warning("image contains zero values")


@functools.lru_cache(maxsize=8)
def _percentile_keys(decimals):
    """The percentile keys as the reference builds them (Python's round of
    each np.linspace(0, 100, 10**(decimals + 2)) value, stats.py:44-47):
    100,000 rounds cost ~0.16 s, so once per process, not per job."""
    q = np.linspace(0, 100, 10 ** (decimals + 2))
    q.setflags(write=False)  # shared by every OnlineStatistics of the process
    return q, tuple(round(x, decimals) for x in q)


class OnlineStatistics(object):
    """Welford mean/variance + percentile accumulator (stats.py:35-121)."""

    def __init__(self, image_dimensions, decimals=3, batch_size=DEFAULT_BATCH, flags=0,
                 options=None):
        self.image_dimensions = tuple(int(d) for d in image_dimensions)
        if len(self.image_dimensions) != 2:
            raise ValueError("image_dimensions must be (height, width)")
        if not (0 <= decimals <= 3):
            raise ValueError('Argument "decimals" must lie in range [0, 3].')
        self.decimals = decimals
        precision = 10 ** (decimals + 2)
        self._q, self._keys = _percentile_keys(decimals)
        h, w = self.image_dimensions
        self._npx = h * w
        lo, hi, gamma = quantile_table(self._npx, self._q)
        self._lut = stats_log10_lut()
        self._batch_size = max(1, int(batch_size))
        self._stage = np.empty((self._batch_size, h, w), dtype=np.uint16)
        self._staged = 0
        self._staged_log = None
        self._cache = None
        L = hip.lib()
        handle = C.c_void_p()
        hip.check(L.tmh_stats_create(h, w, precision, hip.ptr(lo), hip.ptr(hi), hip.ptr(gamma),
                                     hip.ptr(self._lut), self._batch_size, int(flags),
                                     C.byref(handle)))
        self._h = handle
        for opt, val in (options or {}).items():  # launch shapes only (tmh_stats_set_option)
            hip.check(L.tmh_stats_set_option(handle, int(opt), int(val)))

    # -- reference attributes ---------------------------------------------------
    @property
    def n(self):
        """Number of sites accumulated (stats.py:53, :89): the handle's count
        plus the sites still staged on the host."""
        c = C.c_int64()
        hip.check(hip.lib().tmh_stats_get_n(self._h, C.byref(c)))
        return c.value + self._staged

    @n.setter
    def n(self, value):
        """The reference's ``n`` is a plain attribute (stats.py:53): setting
        it changes the count later updates continue from and the divisor of
        ``var`` / ``percentiles``.  Staged sites are flushed first."""
        self._flush()
        hip.check(hip.lib().tmh_stats_set_n(self._h, int(value)))
        self._cache = None

    def refresh(self):
        """Forget cached results: the handle's state was changed through the
        C-ABI (e.g. the multi-GPU merge, sharded.merge_shards)."""
        self._flush()
        self._cache = None

    def update(self, image, log_transform=True):
        """Add one site (stats.py:64-92)."""
        if not isinstance(image, ChannelImage):
            raise TypeError('Argument "image" must have type tmlib.image.ChannelImage.')
        arr = image.array
        if arr.shape != self.image_dimensions:
            raise ValueError("operands could not be broadcast together with shapes %s %s"
                             % (arr.shape, self.image_dimensions))
        log_transform = bool(log_transform)
        if self._staged and self._staged_log != log_transform:
            self._flush()
        self._stage[self._staged] = arr  # uint8 widens exactly to uint16
        self._staged += 1
        self._staged_log = log_transform
        self._cache = None
        if self._staged == self._batch_size:
            self._flush()

    def update_batch(self, sites: np.ndarray, log_transform=True):
        """Add a contiguous [n, H, W] uint16 stack of sites, in order."""
        sites = np.ascontiguousarray(sites)
        if sites.ndim != 3 or sites.shape[1:] != self.image_dimensions:
            raise ValueError("sites must be [n, %d, %d]" % self.image_dimensions)
        if sites.dtype == np.uint8:
            sites = sites.astype(np.uint16)
        if sites.dtype != np.uint16:
            raise ValueError("sites must be uint8 or uint16")
        self._flush()
        self._push(sites, bool(log_transform))

    def update_device(self, dev_sites, n_sites, log_transform=True, stream=None,
                      zero_counts=None):
        """Add ``n_sites`` sites that already sit in device memory ([n, H, W]
        uint16 at address ``dev_sites``, e.g. decoded by the GPU inflate), in
        order, on ``stream`` (a HIP stream handle; None: the handle's).
        ``zero_counts``: a host int64 array (pinned: asynchronous) that receives
        the sites' zero-pixel counts; the caller logs the warnings
        (``log_zero_warnings``) once the stream has reached them.  Without it
        the counts are read back here (synchronising) and logged at once."""
        n = int(n_sites)
        if n <= 0:
            return
        self._flush()
        L = hip.lib()
        sp = None if stream is None else C.c_void_p(int(stream))
        own = zero_counts is None
        if own:
            zero_counts = np.zeros(n, dtype=np.int64)
        # calls of <= 4,096 sites: the handle keeps one such chunk's zero
        # counts (tmh_stats_zero_counts).  On another stream than the handle's
        # the handle's stream waits for the work (tmhip.h stream contract).
        site_bytes = 2 * self.image_dimensions[0] * self.image_dimensions[1]
        for c0 in range(0, n, 4096):
            nc = min(4096, n - c0)
            hip.check(L.tmh_stats_update_device(self._h,
                                                C.c_void_p(int(dev_sites) + c0 * site_bytes), nc,
                                                int(bool(log_transform)), sp))
            hip.check(L.tmh_stats_zero_counts(self._h, hip.ptr(zero_counts[c0:c0 + nc]), nc, sp))
        self._cache = None
        if own:
            hip.check(L.tmh_synchronize(sp))
            if log_transform:
                log_zero_warnings(zero_counts)

    def _push(self, sites, log_transform):
        n = sites.shape[0]
        if n == 0:
            return
        zeros = np.zeros(n, dtype=np.int64)
        hip.check(hip.lib().tmh_stats_update(self._h, hip.ptr(sites), n, int(log_transform),
                                             hip.ptr(zeros)))
        self._cache = None
        if log_transform:
            for _ in range(int(np.count_nonzero(zeros))):
                logger.warning("image contains zero values")

    def _flush(self):
        if self._staged:
            n = self._staged
            self._staged = 0
            self._push(self._stage[:n], self._staged_log)

    def _finalize(self):
        self._flush()
        if self._cache is None:
            h, w = self.image_dimensions
            mean = np.empty((h, w), dtype=np.float64)
            std = np.empty((h, w), dtype=np.float64)
            acc = np.empty(len(self._q), dtype=np.float64)
            hist = np.empty(65536, dtype=np.uint64)
            n = C.c_int64()
            hip.check(hip.lib().tmh_stats_finalize(self._h, C.byref(n), hip.ptr(mean),
                                                   hip.ptr(std), hip.ptr(acc), hip.ptr(hist)))
            self._cache = dict(n=n.value, mean=mean, std=std, acc=acc, hist=hist)
        return self._cache

    # -- results (stats.py:94-121) ----------------------------------------------
    @property
    def var(self):
        """M2 / (n - 1), NaN where n < 2 (stats.py:94-102)."""
        c = self._finalize()
        if c.get("var") is None:
            v = np.empty(self.image_dimensions, dtype=np.float64)
            hip.check(hip.lib().tmh_stats_variance(self._h, hip.ptr(v)))
            c["var"] = v
        return c["var"].copy()

    @property
    def mean(self):
        return IllumstatsImage(self._finalize()["mean"].copy())

    @property
    def std(self):
        return IllumstatsImage(self._finalize()["std"].copy())

    @property
    def percentile_sums(self):
        """The raw f64 accumulator ``_percentiles`` (sum over sites, in order)."""
        return self._finalize()["acc"].copy()

    @property
    def histogram(self):
        """Pooled 65,536-bin histogram of all sites (sum of per-site counts)."""
        return self._finalize()["hist"].copy()

    @property
    def percentiles(self):
        c = self._finalize()
        n = c["n"]
        return {self._keys[i]: int(x / n) for i, x in enumerate(c["acc"].tolist())}

    def close(self):
        if getattr(self, "_h", None):
            hip.lib().tmh_stats_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
