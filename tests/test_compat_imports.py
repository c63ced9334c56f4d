"""CPU: the reference's import paths resolve to lte_phy with only a PYTHONPATH
change (ofdm-lte_amd/compat): `from module import OFDMModule, LTEConfig`
(examples/example_basic.py:17), `from core.sfbc_alamouti import SFBCAlamouti`
(test/test_alamouti_unit.py:11), core.ofdm_core, core.channel_coding (+ its
submodules), config, ofdm_module.  Runs in a fresh interpreter whose
sys.path holds the compat directory only (no repo paths)."""
import os
import subprocess
import sys

from conftest import ROOT

CODE = r'''
import sys
from module import OFDMModule, LTEConfig
import lte_phy   # importable once an alias has run (compat/_boot.py)
from config import LTEConfig as C2, LTE_PROFILES
from ofdm_module import OFDMModule as M2
from core.ofdm_core import OFDMSimulator, simulate_spatial_multiplexing, OFDMChannel
from core.channel import ChannelSimulator
from core.sfbc_alamouti import SFBCAlamouti, SFBCResourceMapper
from core.channel_coding import turbo_decode, rate_match_turbo, set_decoder_mode, calculate_crc24a
from core.channel_coding.turbo_decoder import turbo_decode as td2, LogMAPDecoder
from core.channel_coding.segmentation import segment_code_blocks, find_interleaver_size
from core.mimo_detector import MIMODetector
from core.layer_mapper import LayerMapper
from core.codebook_lte import LTECodebook
from core.rank_adaptation import RankAdaptation
from core.beamforming_precoder import BeamformingPrecoder
from core.csi_feedback import CSIFeedback
from utils.image_processing import ImageProcessor
import module.core.ofdm_core as mc
assert OFDMModule is lte_phy.OFDMModule is M2 and LTEConfig is lte_phy.LTEConfig is C2
assert OFDMSimulator is lte_phy.OFDMSimulator is mc.OFDMSimulator
assert SFBCAlamouti is lte_phy.SFBCAlamouti
assert turbo_decode is td2 is lte_phy.channel_coding.turbo_decode
assert MIMODetector is lte_phy.MIMODetector and ImageProcessor is lte_phy.ImageProcessor
assert find_interleaver_size(5000) == lte_phy.channel_coding.find_interleaver_size(5000)
assert LTE_PROFILES[20.0]['N'] == 2048 and len(lte_phy.channel_coding.__all__) >= 18
assert SFBCAlamouti().get_statistics()['diversity_order'] == 2
print('ok')
'''


def test_reference_import_paths_resolve_to_lte_phy():
    env = dict(os.environ)
    env['PYTHONPATH'] = os.path.join(ROOT, 'ofdm-lte_amd', 'compat')
    r = subprocess.run([sys.executable, '-c', CODE], env=env, capture_output=True, text=True, timeout=120,
                       cwd='/tmp')
    assert r.returncode == 0 and r.stdout.strip().endswith('ok'), r.stderr[-3000:]
