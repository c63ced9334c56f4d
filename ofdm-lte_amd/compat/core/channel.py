"""Alias of core/channel.py (ChannelSimulator) -> lte_phy.ofdm_core."""
from lte_phy.ofdm_core import ChannelSimulator  # noqa: F401
