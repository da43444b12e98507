"""Image classes of the illumination-correction path, computed on MI355X.

Mirrors the hot-path subset of tmlib/image.py:
  ``Image``                (:35-454; array/metadata checks, ``smooth`` :287-311,
                            ``_shift_and_crop`` / ``align`` :345-454)
  ``ChannelImage``         (:455-670; ``_map_to_uint8`` / ``scale`` :493-568,
                            ``clip`` :570-597, ``_correct_illumination`` :599-631,
                            ``correct`` :633-670)
  ``IllumstatsImage``      (:1097-1136)
  ``IllumstatsContainer``  (:1139-1213; ``smooth`` :1172-1193,
                            ``get_closest_percentile`` :1195-1213)

plus the illuminati post-correct chain (illuminati/api.py:396-405) as one
fused pass, ``Corrector.chain_u8``.

Smoothing, correction, clipping, alignment and scaling run in libtmhip.so
(no CPU fallback); the host only evaluates numpy slice bounds and LUT
parameters.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import hip
from .metadata import ImageMetadata, IllumstatsImageMetadata

#: np.log10(1e-10) on this host: the log of a zero pixel in the correction
#: (image.py:624-626 replaces 0 by 10**-10 before the log10)
ZERO_LOG10 = float(np.log10(np.float64(10 ** -10)))


class Image(object):
    """2-D pixel array + optional metadata (tmlib/image.py:35-311)."""

    __slots__ = ("_array", "_metadata")

    def __init__(self, array, metadata=None):
        self.array = array
        self.metadata = metadata

    @property
    def metadata(self):
        return self._metadata

    @metadata.setter
    def metadata(self, value):
        if value is not None and not isinstance(value, ImageMetadata):
            raise TypeError('Argument "metadata" must have type tmlib.metadata.ImageMetadata.')
        self._metadata = value

    @property
    def array(self):
        return self._array

    @array.setter
    def array(self, value):
        if not isinstance(value, np.ndarray):
            raise TypeError('Argument "array" must have type numpy.ndarray.')
        if value.ndim != 2:
            raise ValueError('Argument "array" must be two dimensional.')
        self._array = value

    @property
    def dimensions(self):
        return self.array.shape

    @property
    def dtype(self):
        return self.array.dtype

    @property
    def is_int(self):
        return issubclass(self.array.dtype.type, np.integer)

    @property
    def is_float(self):
        return issubclass(self.array.dtype.type, np.floating)

    @property
    def is_uint(self):
        return issubclass(self.array.dtype.type, np.unsignedinteger)

    @property
    def is_uint8(self):
        return self.array.dtype == np.uint8

    @property
    def is_uint16(self):
        return self.array.dtype == np.uint16

    def align(self, crop=True, inplace=True):
        """Image.align (tmlib/image.py:412-454): shift by the metadata's
        (y_shift, x_shift) and crop, or zero-pad with crop=False (on the GPU)."""
        if self.metadata is None:
            raise AttributeError('Image requires attribute "metadata" for alignment.')
        md = self.metadata
        w, shape = align_window(self.array.shape, md.y_shift, md.x_shift, md.bottom_residue,
                                md.top_residue, md.right_residue, md.left_residue, crop=crop)
        array = align_array(self.array, w, shape)
        if inplace:
            self.metadata.is_aligned = True
            self.array = array
            return self
        new_object = self.__class__(array, self.metadata)
        new_object.metadata.is_aligned = True
        return new_object

    def smooth(self, sigma, inplace=True):
        """Gaussian smoothing (image.py:287-311 -> mahotas.gaussian_filter),
        'reflect' border, radius int(4*sigma+0.5), float64, on the GPU."""
        array = smooth_f64(self.array, sigma)
        if inplace:
            self.array = array
            self.metadata.is_smoothed = True
            return self
        new_img = self.__class__(array, self.metadata)
        new_img.metadata.is_smoothed = True
        return new_img


def align_window(shape, y, x, bottom, top, right, left, crop=True):
    """The numpy slicing of tmlib/image.py:345-410 as a tmh_window: the source
    slice ``[top-y : -(bottom+y) or H, left-x : -(right+x) or W]`` and, for
    crop=False, its destination at (top, left).  Returns (window, out_shape);
    raises like the reference when the pasted window does not fit."""
    H, W = int(shape[0]), int(shape[1])
    row_start, row_end = top - y, bottom + y
    row_end = H if row_end == 0 else -row_end
    col_start, col_end = left - x, right + x
    col_end = W if col_end == 0 else -col_end
    rs, re_, _ = slice(row_start, row_end).indices(H)
    cs, ce, _ = slice(col_start, col_end).indices(W)
    rows, cols = max(0, re_ - rs), max(0, ce - cs)
    w = np.zeros((), dtype=hip.WINDOW_DTYPE)
    w["src_r0"], w["src_c0"], w["rows"], w["cols"] = rs, cs, rows, cols
    if crop:
        return w, (rows, cols)
    # aligned_im[top:top+rows, left:left+cols] = extracted (numpy assignment,
    # negative starts included)
    dr = range(H)[top:top + rows]
    dc = range(W)[left:left + cols]
    # numpy broadcasting: equal extents, or a 1-extent source into an empty slice
    ok = all(n == len(t) or (n == 1 and len(t) == 0) for n, t in ((rows, dr), (cols, dc)))
    if not ok:
        raise Exception("Shifting and cropping of the image failed!\n"
                        "Reason: could not broadcast input array from shape (%d,%d) into "
                        "shape (%d,%d)" % (rows, cols, len(dr), len(dc)))
    if len(dr) == 0 or len(dc) == 0:
        w["rows"] = w["cols"] = 0  # nothing pasted
        return w, (H, W)
    w["dst_r0"], w["dst_c0"] = dr.start, dc.start
    return w, (H, W)


def align_array(array: np.ndarray, window, out_shape) -> np.ndarray:
    a = np.ascontiguousarray(array)
    if a.dtype not in (np.uint8, np.uint16):
        raise TypeError("only uint8/uint16 images are aligned on the device")
    out = np.empty(out_shape, dtype=a.dtype)
    win = np.ascontiguousarray(np.asarray(window, dtype=hip.WINDOW_DTYPE).reshape(1))
    hip.check(hip.lib().tmh_align(hip.ptr(a), hip.ptr(out), a.itemsize, 1, a.shape[0],
                                  a.shape[1], hip.ptr(win), out_shape[0], out_shape[1]))
    return out


def smooth_f64(array: np.ndarray, sigma) -> np.ndarray:
    L = hip.lib()
    a = np.ascontiguousarray(array, dtype=np.float64)
    if a.ndim != 2:
        raise ValueError("smoothing needs a 2-D array")
    out = np.empty_like(a)
    hip.check(L.tmh_smooth_f64(hip.ptr(a), hip.ptr(out), a.shape[0], a.shape[1], float(sigma)))
    return out


class ChannelImage(Image):
    """Grayscale uint8/uint16 site image (tmlib/image.py:455-670)."""

    @staticmethod
    def _map_to_uint8(img, lower_bound=None, upper_bound=None):
        """tmlib/image.py:493-531: uint16 -> uint8 through the reference's numpy
        LUT (evaluated bit-exactly per pixel on the GPU).  Bounds default to the
        image's min / max (the reference's intent; its py3 range check would
        raise on None)."""
        if img.dtype != np.uint16:
            raise TypeError('"img" must have 16-bit unsigned integer type.')
        if lower_bound is not None and not (0 <= lower_bound < 2 ** 16):
            raise ValueError('"lower_bound" must be in the range [0, 65535]')
        if upper_bound is not None and not (0 <= upper_bound < 2 ** 16):
            raise ValueError('"upper_bound" must be in the range [0, 65535]')
        if lower_bound is None:
            lower_bound = np.min(img)
        if upper_bound is None:
            upper_bound = np.max(img)
        if lower_bound >= upper_bound:
            raise ValueError('"lower_bound" must be smaller than "upper_bound"')
        a = np.ascontiguousarray(img)
        out = np.empty(a.shape, dtype=np.uint8)
        hip.check(hip.lib().tmh_map_u16_to_u8(hip.ptr(a), hip.ptr(out), a.size, int(lower_bound),
                                               int(upper_bound)))
        return out

    def scale(self, lower, upper, inplace=True):
        """tmlib/image.py:533-568: map [lower, upper] to [0, 255] (uint16 only;
        uint8 images are returned unchanged)."""
        if self.is_uint16:
            array = self._map_to_uint8(self.array, lower, upper)
            if inplace:
                self.array = array
                self.metadata.is_rescaled = True
                return self
            new_image = self.__class__(array, self.metadata)
            new_image.metadata.is_rescaled = True
            return new_image
        return self

    def __init__(self, array, metadata=None):
        super(ChannelImage, self).__init__(array, metadata)
        if not self.is_uint:
            raise TypeError("Image must have unsigned integer type.")

    @property
    def array(self):
        return self._array

    @array.setter
    def array(self, value):
        if not isinstance(value, np.ndarray):
            raise TypeError('Argument "array" must have type numpy.ndarray.')
        if value.ndim != 2:
            raise ValueError('Argument "array" must be two dimensional.')
        if not (value.dtype == np.uint16 or value.dtype == np.uint8):
            raise ValueError('Argument "array" must have numpy.uint8 or numpy.uint16 data type.')
        self._array = value

    def clip(self, lower, upper, inplace=True):
        """np.clip of the pixels (image.py:570-597), on the GPU."""
        array = clip_array(self.array, lower, upper)
        if inplace:
            self.array = array
            self.metadata.is_clipped = True
            return self
        new_image = self.__class__(array, self.metadata)
        new_image.metadata.is_clipped = True
        return new_image

    @staticmethod
    def _correct_illumination(img, mean, std, log_transform=True):
        """image.py:599-631: log10 -> z-score -> rescale by mean(std),
        mean(mean) -> 10** -> cast to the input dtype (x86 astype rule)."""
        corr = Corrector(mean, std, log_transform=log_transform)
        try:
            return corr.apply(img)
        finally:
            corr.close()

    def correct(self, stats, inplace=True):
        """image.py:633-670: correct with the container's (smoothed) stats."""
        if not isinstance(stats, IllumstatsContainer):
            raise TypeError('Argument "stats" must have type tmlib.image.IllumstatsContainer.')
        if (stats.mean.metadata.channel_id != self.metadata.channel_id or
                stats.std.metadata.channel_id != self.metadata.channel_id):
            raise ValueError("Channels don't match!")
        array = stats.corrector().apply(self.array)
        if inplace:
            self.array = array
            self.metadata.is_corrected = True
            return self
        new_object = ChannelImage(array, self.metadata)
        new_object.metadata.is_corrected = True
        return new_object


def clip_array(array: np.ndarray, lower, upper) -> np.ndarray:
    info = np.iinfo(array.dtype)
    for b in (lower, upper):
        if not (info.min <= int(b) <= info.max):
            raise OverflowError("Python integer %d out of bounds for %s" % (int(b), array.dtype))
    L = hip.lib()
    a = np.ascontiguousarray(array)
    if a.dtype == np.uint8:
        wide = a.astype(np.uint16)
        out = np.empty_like(wide)
        hip.check(L.tmh_clip_u16(hip.ptr(wide), hip.ptr(out), wide.size, int(lower), int(upper)))
        return out.astype(np.uint8)
    out = np.empty_like(a)
    hip.check(L.tmh_clip_u16(hip.ptr(a), hip.ptr(out), a.size, int(lower), int(upper)))
    return out


class Corrector(object):
    """Device-resident correction for one (mean, std) pair.

    Holds tmh_corrector: per-pixel coefficients and the two global means
    (np.mean(std), np.mean(mean), image.py:627) computed once, so a loop of
    ``correct`` calls (illuminati/api.py:389-405) does not redo them.
    """

    def __init__(self, mean, std, log_transform=True):
        L = hip.lib()
        m = np.ascontiguousarray(mean, dtype=np.float64)
        s = np.ascontiguousarray(std, dtype=np.float64)
        if m.shape != s.shape or m.ndim != 2:
            raise ValueError("mean and std must be 2-D arrays of the same shape")
        self.shape = m.shape
        self.log_transform = bool(log_transform)
        h = C.c_void_p()
        hip.check(L.tmh_corrector_create(hip.ptr(m), hip.ptr(s), m.shape[0], m.shape[1],
                                         int(self.log_transform), ZERO_LOG10, C.byref(h)))
        self._h = h

    def means(self):
        a, b = C.c_double(), C.c_double()
        hip.check(hip.lib().tmh_corrector_means(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def apply(self, img: np.ndarray, clip=None, out=None) -> np.ndarray:
        """Correct one image [H,W] or a stack [n,H,W] (uint8/uint16).

        ``out``: optional C-contiguous array of the same shape and dtype to
        write into (a reused buffer skips the first-touch page faults of a
        fresh result, which bound the host path's rate)."""
        img = np.asarray(img)
        if img.shape[-2:] != self.shape:
            raise ValueError("operands could not be broadcast together with shapes %s %s"
                             % (img.shape, self.shape))
        a = np.ascontiguousarray(img)
        if out is None:
            out = np.empty_like(a)
        elif (not isinstance(out, np.ndarray) or out.shape != a.shape or out.dtype != a.dtype
              or not out.flags.c_contiguous or not out.flags.writeable):
            raise ValueError("out must be a writeable C-contiguous %s array of shape %s"
                             % (a.dtype, a.shape))
        elif np.shares_memory(out, a):
            raise ValueError("out must not overlap the input")
        n = 1 if a.ndim == 2 else int(np.prod(a.shape[:-2]))
        lo, hi = (-1, -1) if clip is None else (int(clip[0]), int(clip[1]))
        L = hip.lib()
        if a.dtype == np.uint16:
            hip.check(L.tmh_correct_u16(self._h, hip.ptr(a), hip.ptr(out), n, lo, hi))
        elif a.dtype == np.uint8:
            hip.check(L.tmh_correct_u8(self._h, hip.ptr(a), hip.ptr(out), n, lo, hi))
        else:
            raise TypeError("only uint8/uint16 images can be corrected")
        return out

    def chain_u8(self, sites: np.ndarray, windows, clip_lo: int, clip_hi: int) -> np.ndarray:
        """illuminati/api.py:396-405 for a stack of uint16 sites [n,H,W] in one
        pass: correct -> align(crop=False) with each site's window (see
        ``align_window``) -> clip(clip_lo, clip_hi) -> scale -> uint8."""
        a = np.ascontiguousarray(sites)
        if a.dtype != np.uint16:
            raise TypeError("the chain takes uint16 sites")
        if a.ndim == 2:
            a = a[None]
        if a.shape[-2:] != self.shape:
            raise ValueError("site shape %s does not match the statistics %s"
                             % (a.shape[-2:], self.shape))
        win = np.ascontiguousarray(np.asarray(windows, dtype=hip.WINDOW_DTYPE).reshape(-1))
        if win.size != a.shape[0]:
            raise ValueError("one alignment window per site is required")
        out = np.empty(a.shape, dtype=np.uint8)
        hip.check(hip.lib().tmh_correct_chain_u8(self._h, hip.ptr(a), hip.ptr(out), a.shape[0],
                                                  hip.ptr(win), int(clip_lo), int(clip_hi)))
        return out

    def close(self):
        if getattr(self, "_h", None):
            hip.lib().tmh_corrector_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class IllumstatsImage(Image):
    """float64 statistics plane (tmlib/image.py:1097-1136)."""

    def __init__(self, array, metadata=None):
        if metadata is not None and not isinstance(metadata, IllumstatsImageMetadata):
            raise TypeError('Argument "metadata" must have type '
                            'tmlib.metadata.IllumstatsImageMetadata.')
        super(IllumstatsImage, self).__init__(array, metadata)
        if not self.is_float:
            raise TypeError("Image must have data type float.")

    @property
    def array(self):
        return self._array

    @array.setter
    def array(self, value):
        if not isinstance(value, np.ndarray):
            raise TypeError('Argument "array" must have type numpy.ndarray.')
        if value.ndim != 2:
            raise ValueError('Argument "array" must be two dimensional.')
        if not value.dtype == np.float64:
            raise ValueError('Argument "array" must have numpy.float data type.')
        self._array = value


class IllumstatsContainer(object):
    """mean/std planes + percentile dict of one channel (tmlib/image.py:1139-1213)."""

    def __init__(self, mean, std, percentiles):
        if not isinstance(mean, IllumstatsImage):
            raise TypeError('Argument "mean" must have type tmlib.image.IllumstatsImage.')
        if not isinstance(std, IllumstatsImage):
            raise TypeError('Argument "std" must have type tmlib.image.IllumstatsImage.')
        self.mean = mean
        self.std = std
        self.percentiles = percentiles
        self._corr = None
        self._corr_key = None
        self._corr_arrays = None
        self._corr_locked = []

    def smooth(self, sigma=5):
        """Gaussian-smooth mean and std in place (image.py:1172-1193)."""
        self.mean.array = self.mean.smooth(sigma).array
        self.mean.metadata.is_smoothed = True
        self.std.array = self.std.smooth(sigma).array
        self.std.metadata.is_smoothed = True
        return self

    def get_closest_percentile(self, value):
        """Value of the percentile whose key is closest to ``value``; the first
        key (in dict order) wins ties (image.py:1195-1213)."""
        keys = np.array(list(self.percentiles.keys()))
        idx = np.abs(keys - value).argmin()
        return self.percentiles[keys[idx]]

    def corrector(self, log_transform=True) -> Corrector:
        """Cached device corrector for the current mean/std planes.

        The cache is keyed on the plane objects AND their contents: building
        the corrector marks both arrays read-only (those that were writeable),
        so an in-place write into ``mean.array`` / ``std.array`` raises
        instead of leaving stale device coefficients behind.  Replacing a
        plane (``smooth`` does) or making it writeable again
        (``arr.flags.writeable = True``, then writing) makes the next call
        rebuild the corrector from the current values.  ``release()`` (also
        run when the container is collected) drops the corrector and makes
        the arrays this container locked writeable again.  Neither closes the
        Corrector itself: a caller may hold it past the container (its own
        ``__del__``/``close`` frees the device handle)."""
        m, s = self.mean.array, self.std.array
        key = (id(m), id(s), bool(log_transform))
        if (self._corr is None or self._corr_key != key or m.flags.writeable or
                s.flags.writeable):
            self.release()
            self._corr = Corrector(m, s, log_transform)
            self._corr_key = key
            self._corr_arrays = (m, s)  # keep the ids valid while cached
            self._corr_locked = [a for a in (m, s) if a.flags.writeable]
            for a in self._corr_locked:
                a.flags.writeable = False
        return self._corr

    def release(self):
        """Drop the cache's reference to the device corrector (a caller that
        still holds it keeps a working handle; the last reference frees it);
        the planes it locked are writeable again (the reference's planes are
        plain arrays)."""
        self._corr = None
        self._corr_key = None
        self._corr_arrays = None
        for a in self._corr_locked:
            try:
                a.flags.writeable = True
            except ValueError:  # a view of a read-only base: leave it
                pass
        self._corr_locked = []

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass
