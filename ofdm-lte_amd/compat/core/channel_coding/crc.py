"""Alias of core/channel_coding/crc.py -> lte_phy.channel_coding."""
from lte_phy.channel_coding import (attach_crc24a, attach_crc24b, calculate_crc24a, calculate_crc24b,  # noqa: F401
                                    check_crc24a, check_crc24b)
