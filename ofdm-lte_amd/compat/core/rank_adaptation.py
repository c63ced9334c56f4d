"""Alias of core/rank_adaptation.py -> lte_phy.tm4."""
from lte_phy.tm4 import RankAdaptation  # noqa: F401
