"""Alias of core/channel_coding/rate_matching.py -> lte_phy.channel_coding."""
from lte_phy.channel_coding import (rate_dematching_turbo, rate_match_turbo, sub_block_deinterleaver,  # noqa: F401
                                    sub_block_deinterleaver_llr, sub_block_interleaver)
