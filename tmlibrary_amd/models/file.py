"""HDF5 files of the illumination path (no h5py, no database).

Mirrors the storage half of tmlib/models/file.py with the on-disk layout
unchanged:
  ``ChannelImageFile``  (:207-379) ``/array`` u8/u16, gzip; ``get`` (:322-351),
                        ``put`` (:353-363); FILENAME_FORMAT ``channel_image_file_{id}.h5``
  ``IllumstatsFile``    (:383-472) ``/mean``, ``/std`` f64, ``/percentiles/keys`` f64,
                        ``/percentiles/values`` i64; ``get`` smooths on read
                        (:420-438), ``put`` (:440-456); FILENAME_FORMAT
                        ``illumstats_file_{id}.h5``

The SQLAlchemy/PostgreSQL part of the reference models (ids, sessions,
locations from the channel rows) is out of scope: here a file is addressed by
its path, and ``ExperimentStore`` maps ids to paths.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

from tmlibrary_amd.image import ChannelImage, IllumstatsContainer, IllumstatsImage
from tmlibrary_amd.metadata import ChannelImageMetadata, IllumstatsImageMetadata

_LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hip",
                         "libtmh5.so")
_lib = None
_lock = threading.Lock()

_SIGS = {
    "tmh5_last_error": (C.c_char_p, []),
    "tmh5_write_illumstats": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                        C.c_int64, C.c_void_p, C.c_void_p]),
    "tmh5_illumstats_shape": (C.c_int, [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                        C.POINTER(C.c_int64)]),
    "tmh5_read_illumstats": (C.c_int, [C.c_char_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p]),
    "tmh5_write_channel_image": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                           C.c_int]),
    "tmh5_channel_image_shape": (C.c_int, [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                           C.POINTER(C.c_int)]),
    "tmh5_read_channel_image": (C.c_int, [C.c_char_p, C.c_void_p]),
    "tmh5_write_channel_image_chunked": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int,
                                                   C.c_void_p, C.c_int, C.c_int, C.c_int]),
    "tmh5_read_channel_images": (C.c_int, [C.POINTER(C.c_char_p), C.c_int64, C.c_void_p,
                                           C.c_int]),
    "tmh5_read_raw_chunks": (C.c_int, [C.POINTER(C.c_char_p), C.c_int64, C.c_int, C.c_void_p,
                                       C.c_int64, C.c_void_p, C.c_int64, C.POINTER(C.c_int64),
                                       C.POINTER(C.c_int64), C.c_void_p]),
}

#: struct tmh5_chunk (include/tmh5.h) = struct tmh_zchunk (include/tmhip.h)
CHUNK_DTYPE = np.dtype([("src_off", np.int64), ("src_len", np.int64), ("raw_off", np.int64),
                        ("raw_len", np.int64), ("image", np.int64), ("row0", np.int32),
                        ("col0", np.int32), ("flags", np.int32), ("reserved", np.int32)])


class RawChunksUnsupported(IOError):
    """A file's /array is not chunked with the deflate filter only (contiguous,
    shuffle, other filters, unwritten chunks): decode it on the host."""


def h5lib():
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(_LIB_PATH):
                raise RuntimeError("libtmh5.so not built (make -C tmlibrary_amd/csrc h5; "
                                   "needs libhdf5)")
            lib = C.CDLL(_LIB_PATH)
            for name, (res, args) in _SIGS.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
        return _lib


def _check(rc, path):
    if rc == 0:
        return
    msg = h5lib().tmh5_last_error().decode()
    if rc == -2:
        raise KeyError(msg)
    if rc == -22:
        raise ValueError("%s: %s" % (path, msg))
    raise IOError("%s: %s" % (path, msg))


def _b(path):
    return os.fsencode(path)


def write_illumstats(path, mean, std, percentiles):
    """The four datasets of IllumstatsFile.put (file.py:451-456).  Keys and
    values are written in dict order, as ``percentiles.keys()/values()``."""
    L = h5lib()
    m = np.ascontiguousarray(mean, dtype=np.float64)
    s = np.ascontiguousarray(std, dtype=np.float64)
    keys = np.ascontiguousarray(list(percentiles.keys()), dtype=np.float64)
    vals = np.ascontiguousarray(list(percentiles.values()), dtype=np.int64)
    _check(L.tmh5_write_illumstats(_b(path), m.shape[0], m.shape[1], m.ctypes.data, s.ctypes.data,
                                   keys.size, keys.ctypes.data, vals.ctypes.data), path)


def read_illumstats(path):
    L = h5lib()
    h, w, q = C.c_int(), C.c_int(), C.c_int64()
    _check(L.tmh5_illumstats_shape(_b(path), C.byref(h), C.byref(w), C.byref(q)), path)
    mean = np.empty((h.value, w.value), np.float64)
    std = np.empty_like(mean)
    keys = np.empty(q.value, np.float64)
    vals = np.empty(q.value, np.int64)
    _check(L.tmh5_read_illumstats(_b(path), mean.ctypes.data, std.ctypes.data, keys.ctypes.data,
                                  vals.ctypes.data), path)
    return mean, std, keys, vals


def h5py_chunk_shape(shape, itemsize):
    """The chunk shape h5py picks for a gzip dataset created without explicit
    chunks -- what the reference's files carry: DatasetWriter.write(...,
    compression=True) calls ``create_dataset(path, data=data,
    compression='gzip')`` (tmlib/writers.py:384-387), and h5py chunks such a
    dataset with its ``guess_chunk`` (h5py/_hl/filters.py, a dependency not
    vendored in the reference; the algorithm, unchanged across h5py 2.x-3.x,
    is restated here): a target of 16 KiB x 2^log10(dataset MiB), clamped to
    [8 KiB, 1 MiB]; halve the axes in turn until the chunk is below the target
    or within 50% of it (and below 1 MiB).  A 2160 x 2560 uint16 site: 135 x
    160 (43,200 bytes, 256 chunks per site)."""
    chunks = [float(x if x != 0 else 1024) for x in shape]
    dset = float(np.prod(chunks)) * itemsize
    target = 16 * 1024 * (2 ** np.log10(dset / (1024.0 * 1024)))
    target = min(max(target, 8 * 1024), 1024 * 1024)
    i = 0
    while True:
        cb = float(np.prod(chunks)) * itemsize
        if (cb < target or abs(cb - target) / target < 0.5) and cb < 1024 * 1024:
            break
        if np.prod(chunks) == 1:
            break
        chunks[i % len(chunks)] = float(np.ceil(chunks[i % len(chunks)] / 2.0))
        i += 1
    return tuple(int(x) for x in chunks)


def write_channel_image(path, array, gzip_level=4, chunks=None):
    """``/array`` gzip-compressed (gzip_level < 0: contiguous, uncompressed);
    ``chunks`` = (rows, cols), "rows" for whole-row ~256 KiB chunks, or None
    for h5py's own choice (h5py_chunk_shape: the reference's layout)."""
    L = h5lib()
    a = np.ascontiguousarray(array)
    if a.dtype not in (np.uint8, np.uint16) or a.ndim != 2:
        raise ValueError("channel images are 2-D uint8/uint16")
    if chunks is None:
        chunks = h5py_chunk_shape(a.shape, a.itemsize)
    cr, cc = (0, 0) if chunks == "rows" else (int(chunks[0]), int(chunks[1]))
    _check(L.tmh5_write_channel_image_chunked(_b(path), a.shape[0], a.shape[1], 8 * a.itemsize,
                                              a.ctypes.data, int(gzip_level), cr, cc), path)


def read_channel_image(path):
    L = h5lib()
    h, w, bits = C.c_int(), C.c_int(), C.c_int()
    _check(L.tmh5_channel_image_shape(_b(path), C.byref(h), C.byref(w), C.byref(bits)), path)
    out = np.empty((h.value, w.value), np.uint8 if bits.value == 8 else np.uint16)
    _check(L.tmh5_read_channel_image(_b(path), out.ctypes.data), path)
    return out


def granted_cores():
    """CPUs this process may actually use: the affinity mask, capped by a
    cgroup v2/v1 CPU quota when one is set (a GPU box shows every core of the
    host but grants a share of them)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(period)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                period = int(f.read())
            if q > 0:
                quota = q / period
        except (OSError, ValueError):
            pass
    if quota is not None:
        n = min(n, max(1, int(quota)))
    return max(1, n)


def default_decode_threads():
    """Inflate workers: the cores granted, at most 64 (one file each)."""
    return max(1, min(64, granted_cores()))


def channel_image_shape(path):
    """(height, width, numpy dtype) of a channel image file, from its header."""
    L = h5lib()
    h, w, bits = C.c_int(), C.c_int(), C.c_int()
    _check(L.tmh5_channel_image_shape(_b(path), C.byref(h), C.byref(w), C.byref(bits)), path)
    return h.value, w.value, (np.uint8 if bits.value == 8 else np.uint16)


def read_channel_images(paths, n_threads=None, out=None):
    """Decode many channel image files (same shape/dtype) into one [n, H, W]
    array with ``n_threads`` parallel inflate workers (libtmh5; the HDF5
    layout of tmlib/models/file.py:322-363).  ``out``: a C-contiguous
    [>= n, H, W] array of the files' dtype to decode into (reused buffers
    skip the page faults of a fresh allocation); returns its first n planes."""
    paths = list(paths)
    L = h5lib()
    if not paths:
        return np.empty((0, 0, 0), np.uint16)
    h, w, bits = C.c_int(), C.c_int(), C.c_int()
    _check(L.tmh5_channel_image_shape(_b(paths[0]), C.byref(h), C.byref(w), C.byref(bits)),
           paths[0])
    dt = np.uint8 if bits.value == 8 else np.uint16
    if out is None:
        out = np.empty((len(paths), h.value, w.value), dt)
    else:
        if (out.dtype != dt or out.ndim != 3 or out.shape[0] < len(paths) or
                out.shape[1:] != (h.value, w.value) or not out.flags.c_contiguous):
            raise ValueError("out must be a C-contiguous [>= %d, %d, %d] %s array"
                             % (len(paths), h.value, w.value, np.dtype(dt).name))
        out = out[:len(paths)]
    arr = (C.c_char_p * len(paths))(*[_b(p) for p in paths])
    nt = default_decode_threads() if n_threads is None else int(n_threads)
    _check(L.tmh5_read_channel_images(arr, len(paths), out.ctypes.data, nt), paths[0])
    return out


def read_raw_chunks(paths, n_threads=None, blob=None, table=None):
    """The still-compressed chunks of channel image files for the GPU inflate
    (libtmh5 tmh5_read_raw_chunks): returns (blob, table, geom) -- blob a
    uint8 view holding every chunk's zlib stream, table a CHUNK_DTYPE array
    (one entry per chunk: its bytes in blob, its decompressed bytes in a raw
    buffer of len(table) full chunks, file index, origin), geom =
    (height, width, elem_bytes, chunk_rows, chunk_cols).  ``blob`` / ``table``:
    buffers to fill (e.g. pinned memory reused across calls); grown (fresh
    numpy arrays) when too small.  Raises RawChunksUnsupported for files the
    GPU path cannot take."""
    paths = list(paths)
    L = h5lib()
    arr = (C.c_char_p * len(paths))(*[_b(p) for p in paths])
    nt = default_decode_threads() if n_threads is None else int(n_threads)
    geom = np.zeros(5, np.int32)
    used, nch = C.c_int64(), C.c_int64()
    for attempt in range(2):
        bcap = 0 if blob is None else blob.nbytes
        tcap = 0 if table is None else len(table)
        rc = L.tmh5_read_raw_chunks(arr, len(paths), nt, None if blob is None else blob.ctypes.data,
                                    bcap, None if table is None else table.ctypes.data, tcap,
                                    C.byref(used), C.byref(nch), geom.ctypes.data)
        if rc == -28 and attempt == 0:  # too small: size them and read again
            if blob is None or blob.nbytes < used.value:
                blob = np.empty(max(used.value, 1), np.uint8)
            if table is None or len(table) < nch.value:
                table = np.empty(max(nch.value, 1), CHUNK_DTYPE)
            continue
        if rc == -95:
            raise RawChunksUnsupported(h5lib().tmh5_last_error().decode())
        _check(rc, paths[0] if paths else "")
        break
    return blob[:used.value], table[:nch.value], tuple(int(x) for x in geom)


class ChannelImageFile(object):
    """One site/channel plane on disk (tmlib/models/file.py:207-379)."""

    FILENAME_FORMAT = "channel_image_file_{id}.h5"

    def __init__(self, location, channel_id=0, site_id=0, cycle_id=0, tpoint=0, zplane=0):
        self.location = location
        self.channel_id = channel_id
        self.site_id = site_id
        self.cycle_id = cycle_id
        self.tpoint = tpoint
        self.zplane = zplane

    def get(self):
        md = ChannelImageMetadata(channel_id=self.channel_id, site_id=self.site_id,
                                  tpoint=self.tpoint, zplane=self.zplane, cycle_id=self.cycle_id)
        return ChannelImage(read_channel_image(self.location), md)

    def put(self, image):
        if not isinstance(image, ChannelImage):
            raise TypeError('Argument "image" must have type tmlib.image.ChannelImage.')
        write_channel_image(self.location, image.array, gzip_level=4)


class IllumstatsFile(object):
    """Illumination statistics of one channel (tmlib/models/file.py:383-472)."""

    FILENAME_FORMAT = "illumstats_file_{id}.h5"

    def __init__(self, location, channel_id=0):
        self.location = location
        self.channel_id = channel_id

    def get(self):
        """Read the four datasets, then smooth (file.py:420-438).  mean and std
        share ONE metadata object, as in the reference (:431-434)."""
        mean, std, keys, vals = read_illumstats(self.location)
        md = IllumstatsImageMetadata(channel_id=self.channel_id)
        percentiles = dict(zip(keys.tolist(), vals.tolist()))
        cont = IllumstatsContainer(IllumstatsImage(mean, md), IllumstatsImage(std, md),
                                   percentiles)
        return cont.smooth()

    def put(self, data):
        if not isinstance(data, IllumstatsContainer):
            raise TypeError('Argument "data" must have type tmlib.image.IllumstatsContainer.')
        write_illumstats(self.location, data.mean.array, data.std.array, data.percentiles)


class ExperimentStore(object):
    """Id -> file mapping standing in for the experiment database:
    ``<root>/channel_image_files/channel_image_file_{id}.h5`` and
    ``<root>/illumstats/illumstats_file_{channel_id}.h5``.  ``file_info``
    optionally maps a file id to (channel_id, site_id, cycle_id, tpoint, zplane)."""

    def __init__(self, root, file_info=None):
        self.root = root
        self.file_info = file_info or {}

    def channel_image_file(self, file_id):
        info = self.file_info.get(file_id, (0, int(file_id), 0, 0, 0))
        path = os.path.join(self.root, "channel_image_files",
                            ChannelImageFile.FILENAME_FORMAT.format(id=file_id))
        return ChannelImageFile(path, *info)

    def illumstats_file(self, channel_id):
        d = os.path.join(self.root, "illumstats")
        os.makedirs(d, exist_ok=True)
        return IllumstatsFile(os.path.join(d, IllumstatsFile.FILENAME_FORMAT.format(id=channel_id)),
                              channel_id)
