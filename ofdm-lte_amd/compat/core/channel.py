"""Alias of core/channel.py -> lte_phy.channel (AWGNChannel,
RayleighMultiPathChannel, FadingChannel) and lte_phy.ofdm_core
(ChannelSimulator)."""
from lte_phy.channel import AWGNChannel, FadingChannel, RayleighMultiPathChannel  # noqa: F401
from lte_phy.config import ITU_CHANNEL_MODELS  # noqa: F401
from lte_phy.ofdm_core import ChannelSimulator  # noqa: F401
from lte_phy.rayleighchannel import RayleighChannel  # noqa: F401
