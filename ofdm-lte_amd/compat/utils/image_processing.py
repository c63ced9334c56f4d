"""Alias of utils/image_processing.py -> lte_phy.image_processing."""
from lte_phy.image_processing import *  # noqa: F401,F403
from lte_phy.image_processing import ImageProcessor  # noqa: F401
