"""Alias of core/channel_coding/segmentation.py -> lte_phy.channel_coding."""
from lte_phy.channel_coding import (desegment_code_blocks, find_interleaver_size,  # noqa: F401
                                    get_segmentation_info, segment_code_blocks)
