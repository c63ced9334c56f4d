"""Alias of core/layer_mapper.py -> lte_phy.tm4."""
from lte_phy.tm4 import LayerDemapper, LayerMapper  # noqa: F401
