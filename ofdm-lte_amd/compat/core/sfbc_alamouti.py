"""Alias of core/sfbc_alamouti.py -> lte_phy.sfbc_alamouti."""
from lte_phy.sfbc_alamouti import SFBCAlamouti, SFBCResourceMapper  # noqa: F401
