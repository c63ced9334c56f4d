"""Alias of core/lte_receiver.py -> lte_phy.lte_receiver."""
from lte_phy.lte_receiver import LTEChannelEstimator, LTEEqualizerZF, LTEReceiver  # noqa: F401
from lte_phy.resource_mapper import LTEResourceGrid, PilotPattern  # noqa: F401
from lte_phy.modulator import QAMModulator  # noqa: F401
