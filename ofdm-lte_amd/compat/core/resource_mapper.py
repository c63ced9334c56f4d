"""Alias of core/resource_mapper.py -> lte_phy.resource_mapper."""
from lte_phy.resource_mapper import LTEResourceGrid, PilotPattern, ResourceMapper, EnhancedOFDMModulator  # noqa: F401
