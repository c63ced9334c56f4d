"""Alias of core/dft_precoding.py -> lte_phy.dft_precoding."""
from lte_phy.dft_precoding import DFTPrecodifier, IDFTDecodifier, SC_FDMPrecodifier, SC_FDMDecodifier  # noqa: F401
