"""Coded config-2 BER-curve fixture from the float64 ORACLE (oracle/lte_oracle.py
+ oracle/coding_oracle.c, pinned bit-exact to the reference by
tests/test_oracle_golden.py and, for this chain, by golden_r2's cod_curve).

Workload: OFDMSimulator.simulate_siso_coded (core/ofdm_core.py:925-1338) on
config 2 (20 MHz, 64-QAM, Rayleigh ITU Pedestrian-A, TB 27 760) at SNR
0:2:30 dB, FRAMES frames per SNR point.  Frame f of SNR point s draws, from
np.random.RandomState(SEED0 + 1000 * s + f) in this order: the TB bits
(randint(0, 2, TB)), the Jakes phases of the 4 paths (2 pi rand(4, 16)), the
real then imaginary unit normals of the noise (randn(L) twice).  The GPU test
regenerates exactly these draws (RandomState is stable across NumPy versions)
and injects them, so only the expected per-frame bit errors and CRC verdicts
are stored.

usage:  python tests/golden/make_fixture_ber_curve.py [--procs 8]
"""
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(ROOT, 'tests', 'golden', 'fixture_ber_curve.npz')
SNRS = list(range(0, 31, 2))
FRAMES = 32
SEED0 = 777
TB = 27760


def draws(s, f, L):
    rs = np.random.RandomState(SEED0 + 1000 * s + f)
    bits = rs.randint(0, 2, TB)
    ph = 2 * np.pi * rs.rand(4, 16)
    z_re = rs.randn(L)
    z_im = rs.randn(L)
    return bits, ph, z_re, z_im


def one(job):
    s, f = job
    sys.path.insert(0, ROOT)
    from oracle import lte_oracle as O
    O.lib()
    num = O.Numerology(bandwidth=20.0, modulation='64-QAM')
    L = 14 * (num.N + num.cp)
    bits, ph, zr, zi = draws(s, f, L)
    r = O.simulate_siso_coded(num, bits, float(SNRS[s]), 'rayleigh_mp',
                              draws=[{'phases': list(ph), 'z_re': zr, 'z_im': zi}])
    return s, f, int(r['bit_errors']), int(r['crc_pass'])


def main():
    procs = int(sys.argv[sys.argv.index('--procs') + 1]) if '--procs' in sys.argv else 8
    t0 = time.time()
    jobs = [(s, f) for s in range(len(SNRS)) for f in range(FRAMES)]
    with mp.get_context('spawn').Pool(procs) as pool:
        res = pool.map(one, jobs)
    err = np.zeros((len(SNRS), FRAMES), dtype=np.int64)
    crc = np.zeros((len(SNRS), FRAMES), dtype=np.uint8)
    for s, f, e, c in res:
        err[s, f], crc[s, f] = e, c
    np.savez_compressed(OUT, snrs=np.array(SNRS, dtype=np.float64), frames=np.array([FRAMES]),
                        seed0=np.array([SEED0]), tb=np.array([TB]), bit_errors=err, crc_ok=crc)
    ber = err.sum(1) / (FRAMES * TB)
    with open(OUT.replace('.npz', '_manifest.json'), 'w') as f:
        json.dump({'generated_by': 'tests/golden/make_fixture_ber_curve.py (float64 oracle)',
                   'numpy': np.__version__, 'ber': ber.tolist(), 'bler': (1 - crc.mean(1)).tolist()}, f, indent=1)
    print('BER', np.array2string(ber, precision=4), f'({time.time() - t0:.0f}s)')


if __name__ == '__main__':
    main()
