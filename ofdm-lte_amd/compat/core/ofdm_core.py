"""Alias of core/ofdm_core.py -> lte_phy.ofdm_core."""
from lte_phy.ofdm_core import (ChannelSimulator, OFDMChannel, OFDMReceiver, OFDMSimulator,  # noqa: F401
                               OFDMTransmitter, simulate_spatial_multiplexing)
