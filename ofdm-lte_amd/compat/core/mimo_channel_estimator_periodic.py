"""Alias of core/mimo_channel_estimator_periodic.py -> lte_phy.mimo_channel_estimator_periodic."""
from lte_phy.mimo_channel_estimator_periodic import MIMOChannelEstimatorPeriodic  # noqa: F401
from lte_phy.lte_receiver import LTEChannelEstimator  # noqa: F401
from lte_phy.resource_mapper import LTEResourceGrid, PilotPattern  # noqa: F401
