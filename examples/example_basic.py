"""Example 1 of the reference (examples/example_basic.py) on the MI355X engine:
OFDMModule with the default configuration, 10 000 random bits through the
GPU chain at SNR 5 / 10 / 15 / 20 dB.  Only the import changes.

    python examples/example_basic.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ofdm-lte_amd'))

from lte_phy import LTEConfig, OFDMModule  # noqa: E402


def main():
    config = LTEConfig()
    print(config)
    module = OFDMModule(config=config, channel_type='awgn')
    bits = np.random.randint(0, 2, 10000)
    for snr in (5, 10, 15, 20):
        r = module.transmit(bits, snr_db=snr)
        print(f"SNR {snr:>2} dB: BER {r['ber']:.4e} ({r['bit_errors']} errors), PAPR {r['papr_db']:.2f} dB")


if __name__ == '__main__':
    main()
