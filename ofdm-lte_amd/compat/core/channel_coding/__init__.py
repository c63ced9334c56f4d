"""Alias of core/channel_coding (core/channel_coding/__init__.py:15-40) ->
lte_phy.channel_coding: all 18 names + set_decoder_mode; the submodules
(crc, segmentation, turbo_encoder, turbo_decoder, rate_matching) re-export
the same functions."""
from lte_phy.channel_coding import *  # noqa: F401,F403
from lte_phy.channel_coding import __all__, LogMAPDecoder, find_interleaver_size, set_decoder_mode  # noqa: F401
from . import crc, rate_matching, segmentation, turbo_decoder, turbo_encoder  # noqa: F401
