"""Alias of core/channel_coding/turbo_encoder.py -> lte_phy.channel_coding."""
from lte_phy.channel_coding import (qpp_deinterleave, qpp_interleave, rsc_encode, turbo_encode,  # noqa: F401
                                    turbo_encode_block_list)
