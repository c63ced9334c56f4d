"""Alias of core/beamforming_precoder.py -> lte_phy.beamforming."""
from lte_phy.beamforming import AdaptiveBeamforming, BeamformingPrecoder  # noqa: F401
