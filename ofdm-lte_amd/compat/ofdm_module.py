"""Alias of the reference's ofdm_module.py -> lte_phy.ofdm_module."""
import _boot  # noqa: F401
from lte_phy.config import LTEConfig  # noqa: F401
from lte_phy.ofdm_module import *  # noqa: F401,F403
from lte_phy.ofdm_module import OFDMModule  # noqa: F401
