"""Alias of the reference's config.py -> lte_phy.config."""
import _boot  # noqa: F401
from lte_phy.config import *  # noqa: F401,F403
from lte_phy.config import (CP_VALUES, ITU_CHANNEL_MODELS, LTE_PROFILES, MODULATION_SCHEMES,  # noqa: F401
                            SUBCARRIER_SPACING, LTEConfig, create_config_5MHz_QPSK, create_config_10MHz_64QAM,
                            create_config_20MHz_16QAM)
