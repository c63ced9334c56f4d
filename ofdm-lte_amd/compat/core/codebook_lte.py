"""Alias of core/codebook_lte.py -> lte_phy.tm4."""
from lte_phy.tm4 import LTECodebook  # noqa: F401
