"""lte_phy -- MI355X-native LTE PHY link-level engine.

Drop-in for Darioxavierl/OFDM-LTE's public API (LTEConfig, OFDMModule,
OFDMSimulator, OFDMTransmitter, OFDMReceiver, OFDMChannel): same names,
arguments and result dictionaries; the per-OFDM-symbol chain and the turbo
decoder run as hand-written gfx950 HIP kernels in liblte_hip.so.
"""
from .config import (CP_VALUES, ITU_CHANNEL_MODELS, LTE_PROFILES, MODULATION_SCHEMES, SUBCARRIER_SPACING,
                     LTEConfig)
from .ofdm_core import (ChannelSimulator, OFDMChannel, OFDMReceiver, OFDMSimulator, OFDMTransmitter,
                        simulate_spatial_multiplexing)
from .ofdm_module import OFDMModule
from . import channel_coding
from .tm4 import LTECodebook, LayerMapper, MIMODetector, RankAdaptation
from .beamforming import AdaptiveBeamforming, BeamformingPrecoder, CSIFeedback
from .image_processing import ImageProcessor
from .sfbc_alamouti import SFBCAlamouti, SFBCResourceMapper

__version__ = '0.1.0'
__all__ = ['LTEConfig', 'OFDMModule', 'OFDMSimulator', 'OFDMTransmitter', 'OFDMReceiver', 'OFDMChannel',
           'ChannelSimulator', 'simulate_spatial_multiplexing', 'channel_coding', 'LTECodebook', 'LayerMapper',
           'MIMODetector', 'RankAdaptation', 'BeamformingPrecoder', 'AdaptiveBeamforming', 'CSIFeedback',
           'ImageProcessor', 'SFBCAlamouti', 'SFBCResourceMapper', 'MODULATION_SCHEMES', 'ITU_CHANNEL_MODELS',
           'LTE_PROFILES', 'CP_VALUES', 'SUBCARRIER_SPACING']
