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
from .resource_mapper import EnhancedOFDMModulator, LTEResourceGrid, PilotPattern, ResourceMapper
from .modulator import OFDMModulator, QAMModulator, qam16_to_llrs, qam64_to_llrs, qpsk_to_llrs
from .dft_precoding import DFTPrecodifier, IDFTDecodifier, SC_FDMDecodifier, SC_FDMPrecodifier
from .lte_receiver import LTEChannelEstimator, LTEEqualizerZF, LTEReceiver
from .demodulator import OFDMDemodulator, SymbolDetector
from .rayleighchannel import RayleighChannel
from .channel import AWGNChannel, FadingChannel, RayleighMultiPathChannel
from .mimo_channel_estimator_periodic import MIMOChannelEstimatorPeriodic

__version__ = '0.1.0'
__all__ = ['LTEConfig', 'OFDMModule', 'OFDMSimulator', 'OFDMTransmitter', 'OFDMReceiver', 'OFDMChannel',
           'ChannelSimulator', 'simulate_spatial_multiplexing', 'channel_coding', 'LTECodebook', 'LayerMapper',
           'MIMODetector', 'RankAdaptation', 'BeamformingPrecoder', 'AdaptiveBeamforming', 'CSIFeedback',
           'ImageProcessor', 'SFBCAlamouti', 'SFBCResourceMapper', 'MODULATION_SCHEMES', 'ITU_CHANNEL_MODELS',
           'LTE_PROFILES', 'CP_VALUES', 'SUBCARRIER_SPACING',
           'LTEResourceGrid', 'PilotPattern', 'ResourceMapper', 'EnhancedOFDMModulator', 'QAMModulator',
           'OFDMModulator', 'qpsk_to_llrs', 'qam16_to_llrs', 'qam64_to_llrs', 'DFTPrecodifier', 'IDFTDecodifier',
           'SC_FDMPrecodifier', 'SC_FDMDecodifier', 'LTEChannelEstimator', 'LTEEqualizerZF', 'LTEReceiver',
           'OFDMDemodulator', 'SymbolDetector', 'RayleighChannel', 'AWGNChannel', 'RayleighMultiPathChannel',
           'FadingChannel', 'MIMOChannelEstimatorPeriodic']
