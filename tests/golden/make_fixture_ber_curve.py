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

--config 4: the config-4 curve (fixture_ber_curve_c4.npz) -- SFBC 2x2 Alamouti
+ the coding chain (oracle/mimo_oracle.py simulate_sfbc_coded: the build's
composition, simulate_mimo with the Q19 estimator fix around
simulate_siso_coded's coding), 20 MHz 64-QAM, Rayleigh PedA,
TB 27 760, 0:2:30 dB x 32 frames.  Frame f of SNR point s draws from
np.random.RandomState(SEED0_C4 + 1000 * s + f): the TB bits, then
transmit_mimo's draws in the reference's order (core/ofdm_core.py:468-541):
per RX r, per TX t: the 4 paths' Jakes phases (2 pi rand(16) each), the link's
100 dB noise (randn(L) real, randn(L) imaginary); then the RX noise (randn(L)
twice).

usage:  python tests/golden/make_fixture_ber_curve.py [--procs 8] [--config 2|4]
"""
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(ROOT, 'tests', 'golden', 'fixture_ber_curve.npz')
OUT_C4 = os.path.join(ROOT, 'tests', 'golden', 'fixture_ber_curve_c4.npz')
SNRS = list(range(0, 31, 2))
FRAMES = 32
SEED0 = 777
SEED0_C4 = 4444
TB = 27760
NUM_RX_C4 = 2


def draws(s, f, L):
    rs = np.random.RandomState(SEED0 + 1000 * s + f)
    bits = rs.randint(0, 2, TB)
    ph = 2 * np.pi * rs.rand(4, 16)
    z_re = rs.randn(L)
    z_im = rs.randn(L)
    return bits, ph, z_re, z_im


def draws_c4(s, f, L, num_rx=NUM_RX_C4, n_paths=4):
    """bits, then transmit_mimo's draws: per RX [per TX (phases [P][16], link z_re, z_im)], RX z_re, z_im."""
    rs = np.random.RandomState(SEED0_C4 + 1000 * s + f)
    bits = rs.randint(0, 2, TB)
    ph = np.zeros((num_rx, 2, n_paths, 16))
    lz = np.zeros((num_rx, 2, 2, L))
    z = np.zeros((num_rx, 2, L))
    for r in range(num_rx):
        for t in range(2):
            for p in range(n_paths):
                ph[r, t, p] = 2 * np.pi * rs.rand(16)
            lz[r, t, 0] = rs.randn(L)
            lz[r, t, 1] = rs.randn(L)
        z[r, 0] = rs.randn(L)
        z[r, 1] = rs.randn(L)
    return bits, ph, lz, z


def one_c4(job):
    s, f = job
    sys.path.insert(0, ROOT)
    from oracle import lte_oracle as O, mimo_oracle as M
    O.lib()
    num = O.Numerology(bandwidth=20.0, modulation='64-QAM')
    L = 14 * (num.N + num.cp)
    bits, ph, lz, z = draws_c4(s, f, L)
    d = [{'links': [{'phases': list(ph[r, t]), 'z_re': lz[r, t, 0], 'z_im': lz[r, t, 1]} for t in range(2)],
          'z_re': z[r, 0], 'z_im': z[r, 1]} for r in range(NUM_RX_C4)]
    r = M.simulate_sfbc_coded(num, bits, float(SNRS[s]), NUM_RX_C4, 'rayleigh_mp', draws=d)
    return s, f, int(r['bit_errors']), int(r['crc_pass'])


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
    c4 = '--config' in sys.argv and sys.argv[sys.argv.index('--config') + 1] == '4'
    out = OUT_C4 if c4 else OUT
    t0 = time.time()
    jobs = [(s, f) for s in range(len(SNRS)) for f in range(FRAMES)]
    with mp.get_context('spawn').Pool(procs) as pool:
        res = pool.map(one_c4 if c4 else one, jobs)
    err = np.zeros((len(SNRS), FRAMES), dtype=np.int64)
    crc = np.zeros((len(SNRS), FRAMES), dtype=np.uint8)
    for s, f, e, c in res:
        err[s, f], crc[s, f] = e, c
    extra = {'num_rx': np.array([NUM_RX_C4])} if c4 else {}
    np.savez_compressed(out, snrs=np.array(SNRS, dtype=np.float64), frames=np.array([FRAMES]),
                        seed0=np.array([SEED0_C4 if c4 else SEED0]), tb=np.array([TB]), bit_errors=err, crc_ok=crc,
                        **extra)
    ber = err.sum(1) / (FRAMES * TB)
    with open(out.replace('.npz', '_manifest.json'), 'w') as f:
        man = {'generated_by': 'tests/golden/make_fixture_ber_curve.py' + (' --config 4' if c4 else '') +
               ' (float64 oracle)', 'numpy': np.__version__, 'ber': ber.tolist(),
               'bler': (1 - crc.mean(1)).tolist()}
        if c4:
            man['parity'] = ('unpinned by the reference: the reference has no function that composes SFBC with '
                             'the coding chain; this fixture is the float64 oracle\'s composition '
                             '(oracle/mimo_oracle.py simulate_sfbc_coded, DESIGN.md 3a), each of whose components '
                             'is pinned to the reference\'s goldens')
        json.dump(man, f, indent=1)
    print('BER', np.array2string(ber, precision=4), f'({time.time() - t0:.0f}s)')


if __name__ == '__main__':
    main()
