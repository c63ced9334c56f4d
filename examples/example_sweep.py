"""Example 2 of the reference (examples/example_sweep.py) on the MI355X engine:
BER sweep OFDM vs SC-FDM with OFDMModule.run_ber_sweep (one GPU call per
(SNR, trial), identical semantics to the reference), then the same comparison
as a device-resident Monte-Carlo grid (run_grid: Philox randomness, thousands
of frames per launch).

    python examples/example_sweep.py
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ofdm-lte_amd'))

from lte_phy import OFDMModule  # noqa: E402


def main():
    snr_range = np.arange(0, 21, 5)
    res = {}
    for name, kw in [('OFDM (QPSK)', {'enable_sc_fdm': False}), ('SC-FDM (QPSK)', {'enable_sc_fdm': True})]:
        m = OFDMModule(**kw)
        res[name] = m.run_ber_sweep(num_bits=50000, snr_range=snr_range)
        print(name, ' '.join(f'{b:.3e}' for b in res[name]['ber_mean']))
    print(f"{'SNR (dB)':<10} {'OFDM BER':<12} {'SC-FDM BER':<12}")
    for s, a, b in zip(snr_range, res['OFDM (QPSK)']['ber_mean'], res['SC-FDM (QPSK)']['ber_mean']):
        print(f'{s:<10.1f} {a:<12.4e} {b:<12.4e}')
    for name, kw in [('OFDM', {'enable_sc_fdm': False}), ('SC-FDM', {'enable_sc_fdm': True})]:
        sim = OFDMModule(**kw).simulator
        t = time.time()
        g = sim.run_grid(snr_range, num_trials=2000, seed=1)
        el = time.time() - t
        print(f'run_grid {name}: {len(snr_range) * 2000} frames in {el:.2f} s, BER', ' '.join(f'{b:.3e}' for b in g['ber']))


if __name__ == '__main__':
    main()
