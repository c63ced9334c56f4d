"""Alias of core/channel_coding/turbo_decoder.py -> lte_phy.channel_coding."""
from lte_phy.channel_coding import (LogMAPDecoder, log_sum_exp, max_star, set_decoder_mode,  # noqa: F401
                                    turbo_decode)
