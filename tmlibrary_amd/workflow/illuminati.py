"""The illuminati step's use of this path's statistics.

illuminati builds the display pyramid from corrected site images; per
channel layer it derives the intensity clip bounds from the channel's
illumination statistics -- the percentiles ``OnlineStatistics`` accumulated
(corilla/stats.py:114-121) -- and then runs every site through correct ->
align -> clip -> scale (illuminati/api.py:396-405; here
``Corrector.chain_u8``, one fused pass).
"""
from __future__ import annotations


def clip_bounds(stats, clip=True, clip_value=None, clip_percent=99.9, bit_depth=16):
    """(clip_min, clip_max) of a channel layer, tmlib/workflow/illuminati/
    api.py:119-164 (``layer.min_intensity`` / ``layer.max_intensity``):

    * ``clip`` with no ``clip_value``: clip_max = the channel's percentile
      closest to ``clip_percent`` (IllumstatsContainer.get_closest_percentile,
      image.py:1195-1213), raised to 700 (255 for 8-bit channels) -- a dim,
      probably "empty" channel is not stretched further (api.py:142-153);
      clip_min = the percentile closest to 0.001 (api.py:155);
    * ``clip`` with a ``clip_value``: (0, clip_value) (api.py:156-160);
    * no ``clip``: (0, 2**bit_depth - 1) (api.py:161-164).

    ``stats``: an IllumstatsContainer (or anything with
    ``get_closest_percentile``); ignored unless the bounds come from it."""
    if not clip:
        return 0, 2 ** int(bit_depth) - 1
    if clip_value is not None:
        return 0, clip_value
    clip_max = stats.get_closest_percentile(clip_percent)
    floor = 255 if int(bit_depth) == 8 else 700
    if clip_max < floor:
        clip_max = floor
    clip_min = stats.get_closest_percentile(0.001)
    return clip_min, clip_max


def correct_chain_u8(stats, sites, windows, clip=True, clip_value=None, clip_percent=99.9,
                     bit_depth=16, log_transform=True):
    """illuminati/api.py:389-405 for a stack of uint16 sites of one channel
    layer: the layer's clip bounds from the channel's statistics
    (``clip_bounds``), then correct (``stats``' smoothed planes) -> align
    (``windows``, image.align_window) -> clip -> scale to uint8 in one device
    pass.  Returns (uint8 sites, (clip_min, clip_max))."""
    lo, hi = clip_bounds(stats, clip, clip_value, clip_percent, bit_depth)
    out = stats.corrector(log_transform).chain_u8(sites, windows, int(lo), int(hi))
    return out, (lo, hi)
