"""Alias of core/channel_coding/crc.py -> lte_phy.channel_coding."""
from lte_phy.channel_coding import (CRC16_POLYNOMIAL, CRC24A_POLYNOMIAL, CRC24B_POLYNOMIAL,  # noqa: F401
                                    attach_crc16, attach_crc24a, attach_crc24b, calculate_crc16, calculate_crc24a,
                                    calculate_crc24b, check_crc16, check_crc24a, check_crc24b,
                                    get_test_vectors_crc24a)
