"""Alias of core/rayleighchannel.py -> lte_phy.rayleighchannel."""
from lte_phy.rayleighchannel import RayleighChannel  # noqa: F401
