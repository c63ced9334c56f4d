"""Alias of core/csi_feedback.py -> lte_phy.beamforming."""
from lte_phy.beamforming import CSIFeedback  # noqa: F401
