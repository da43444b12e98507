"""tmlibrary_amd — MI355X-native corilla illumination statistics + correction.

A drop-in for TmLibrary's ``tmlib.workflow.corilla`` (``OnlineStatistics``,
``IllumstatsCalculator.run_job``) and the apply step in ``tmlib.image``
(``IllumstatsContainer.smooth``, ``ChannelImage.correct``/``clip``), computed
by hand-written gfx950 HIP kernels behind the C-ABI in ``include/tmhip.h``.
"""
__version__ = "0.1.0"
