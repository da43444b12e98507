"""Image metadata used on the illumination-correction path.

Mirrors the hot-path subset of tmlib/metadata.py: ``ImageMetadata``
(:28-58), ``SiteImageMetadata`` (:61-113), ``ChannelImageMetadata``
(:163-336) and ``IllumstatsImageMetadata`` (:477-522).  Every attribute is
type-checked on assignment and raises ``TypeError`` like the reference.
"""
from __future__ import annotations


def _typed(name: str, kind: type, label: str = None):
    label = label or name
    slot = "_" + name

    def fget(self):
        return getattr(self, slot)

    def fset(self, value):
        # bool is an int subclass in Python; the reference's isinstance checks
        # accept it for int fields, and so do we
        if not isinstance(value, kind):
            raise TypeError('Attribute "%s" must have type %s.' % (label, kind.__name__))
        setattr(self, slot, value)

    return property(fget, fset)


class ImageMetadata(object):
    """Base metadata (tmlib/metadata.py:28-58)."""

    __slots__ = ("_is_aligned", "_is_omitted")
    is_aligned = _typed("is_aligned", bool)
    is_omitted = _typed("is_omitted", bool, "omit")

    def __init__(self):
        self.is_aligned = False
        self.is_omitted = False


class SiteImageMetadata(ImageMetadata):
    """Metadata of an image that maps to one site (tmlib/metadata.py:61-113)."""

    __slots__ = ("_site_id", "_tpoint", "_zplane")
    site_id = _typed("site_id", int)
    tpoint = _typed("tpoint", int)
    zplane = _typed("zplane", int)

    def __init__(self, site_id, tpoint, zplane):
        super(SiteImageMetadata, self).__init__()
        self.tpoint = tpoint
        self.zplane = zplane
        self.site_id = site_id


class ChannelImageMetadata(SiteImageMetadata):
    """Metadata of a ``ChannelImage`` (tmlib/metadata.py:163-336)."""

    __slots__ = ("_channel_id", "_cycle_id", "_is_corrected", "_is_rescaled", "_is_clipped",
                 "_bottom_residue", "_top_residue", "_left_residue", "_right_residue",
                 "_x_shift", "_y_shift")
    channel_id = _typed("channel_id", int)
    cycle_id = _typed("cycle_id", int)
    is_corrected = _typed("is_corrected", bool)
    is_rescaled = _typed("is_rescaled", bool)
    is_clipped = _typed("is_clipped", bool)
    bottom_residue = _typed("bottom_residue", int)
    top_residue = _typed("top_residue", int)
    left_residue = _typed("left_residue", int)
    right_residue = _typed("right_residue", int)
    x_shift = _typed("x_shift", int)
    y_shift = _typed("y_shift", int)

    def __init__(self, channel_id, site_id, cycle_id, tpoint, zplane):
        super(ChannelImageMetadata, self).__init__(site_id, tpoint, zplane)
        self.channel_id = channel_id
        self.cycle_id = cycle_id
        self.is_corrected = False
        self.is_rescaled = False
        self.is_clipped = False
        self.bottom_residue = 0
        self.top_residue = 0
        self.left_residue = 0
        self.right_residue = 0
        self.x_shift = 0
        self.y_shift = 0

    def __repr__(self):
        return "<%s(channel_id=%r, site_id=%r, cycle_id=%r, tpoint=%r)" % (
            self.__class__.__name__, self.channel_id, self.site_id, self.cycle_id, self.tpoint)


class IllumstatsImageMetadata(ImageMetadata):
    """Metadata of an ``IllumstatsImage`` (tmlib/metadata.py:477-522)."""

    __slots__ = ("_channel_id", "_is_smoothed")
    channel_id = _typed("channel_id", int)
    is_smoothed = _typed("is_smoothed", bool)

    def __init__(self, channel_id):
        super(IllumstatsImageMetadata, self).__init__()
        self.channel_id = channel_id
        self.is_smoothed = False

    def __repr__(self):
        return "%s(channel_id=%r)" % (self.__class__.__name__, self.channel_id)
