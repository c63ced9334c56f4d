"""Alias of core/modulator.py -> lte_phy.modulator."""
from lte_phy.modulator import (OFDMModulator, QAMModulator, qam16_to_llrs, qam64_to_llrs,  # noqa: F401
                                qpsk_to_llrs)
from lte_phy.resource_mapper import ResourceMapper  # noqa: F401
from lte_phy.dft_precoding import SC_FDMPrecodifier  # noqa: F401
from lte_phy.config import LTEConfig  # noqa: F401
