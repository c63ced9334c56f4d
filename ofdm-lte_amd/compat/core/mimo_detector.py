"""Alias of core/mimo_detector.py -> lte_phy.tm4."""
from lte_phy.tm4 import MIMODetector  # noqa: F401
