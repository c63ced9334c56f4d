"""Alias of core/channel_coding/turbo_decoder.py -> lte_phy.channel_coding."""
from lte_phy.channel_coding import LogMAPDecoder, set_decoder_mode, turbo_decode  # noqa: F401
