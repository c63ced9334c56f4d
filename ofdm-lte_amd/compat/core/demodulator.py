"""Alias of core/demodulator.py -> lte_phy.demodulator."""
from lte_phy.demodulator import OFDMDemodulator, SymbolDetector  # noqa: F401
from lte_phy.modulator import QAMModulator  # noqa: F401
from lte_phy.dft_precoding import SC_FDMDecodifier  # noqa: F401
