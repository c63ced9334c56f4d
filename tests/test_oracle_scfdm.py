"""CPU: the SC-FDM rows of the oracle (oracle/lte_oracle.py dft_matrix,
modulate_stream / receive / simulate_siso / simulate_simo with sc_fdm; SURVEY
§8(f) rank 2) against vectors from running the reference
(tests/golden/make_golden_scfdm.py).  Exact equality unless stated."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import ROOT, unpack

MAN = json.load(open(os.path.join(ROOT, 'tests', 'golden', 'golden_scfdm_manifest.json')))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize('M', [62, 249, 499, 999])
def test_dft_precoding(golden_scfdm, oracle, M):
    g = golden_scfdm
    X = oracle.dft_matrix(M) @ g[f'dft{M}_x']
    assert np.array_equal(X, g[f'dft{M}_X'])
    assert np.array_equal(oracle.dft_matrix(M, inverse=True) @ X, g[f'dft{M}_inv'])
    assert np.max(np.abs(g[f'dft{M}_inv'] - g[f'dft{M}_x'])) < 1e-12      # unitary round trip
    assert np.max(np.abs(g[f'dft{M}_fftX'] - X)) < 1e-12                  # precoding_ifft == matrix


def test_transmitter_sc_fdm(golden_scfdm, oracle):
    g = golden_scfdm
    num = oracle.Numerology(bandwidth=1.25, modulation='QPSK')
    bits = unpack(g['tx_bits'], int(g['tx_nbits'][0])).astype(np.int64)
    sig, syms, _ = oracle.modulate_stream(num, bits, sc_fdm=True)
    assert np.array_equal(sig, g['tx_signal'])
    assert np.array_equal(np.array(syms), g['tx_syms'])
    assert oracle.papr(sig)['papr_db'] == g['tx_papr'][0]


E2E = [('sc_c1', 1.25, 'QPSK', 'awgn', [0, 5, 10], 'siso'),
       ('sc_c1odd', 1.25, '16-QAM', 'awgn', [12], 'siso'),
       ('sc_c5m', 5.0, 'QPSK', 'awgn', [3], 'siso'),
       ('sc_c2', 20.0, '64-QAM', 'rayleigh_mp', [10, 20, 30], 'siso'),
       ('sc_c3', 10.0, '16-QAM', 'rayleigh_mp', [15], 'siso'),
       ('sc_simo', 1.25, 'QPSK', 'awgn', [10], 'simo'),
       ('noeq_c1', 1.25, 'QPSK', 'awgn', [5, 10], 'noeq'),
       ('noeq_c2', 20.0, '16-QAM', 'rayleigh_mp', [20], 'noeq'),
       ('noeq_sc', 1.25, 'QPSK', 'awgn', [10], 'noeq_sc')]


@pytest.mark.parametrize('name,bw,mod,chan,snrs,fn', E2E)
def test_end_to_end_sc_fdm(golden_scfdm, oracle, name, bw, mod, chan, snrs, fn):
    g = golden_scfdm
    num = oracle.Numerology(bandwidth=bw, modulation=mod)
    n = int(g[f'{name}_nbits'][0])
    bits = unpack(g[f'{name}_bits'], n).astype(np.int64)
    for snr in snrs:
        k = f'{name}_snr{snr}'
        if fn == 'siso':
            r = oracle.simulate_siso(num, bits, snr, channel=chan, sc_fdm=True)
        elif fn.startswith('noeq'):
            r = oracle.simulate_siso(num, bits, snr, channel=chan, sc_fdm=fn == 'noeq_sc', equalize=False)
        else:
            r = oracle.simulate_simo(num, bits, snr, num_rx=2, channel=chan, sc_fdm=True)
        assert r['bit_errors'] == g[k + '_errors'][0], (k, r['bit_errors'], g[k + '_errors'][0])
        assert np.array_equal(r['bits_received_array'], unpack(g[k + '_rx'], n))
        assert r['papr_db'] == g[k + '_papr'][0]
        assert sha(r['signal_tx']) == MAN[k + '_sigtx_sha']
        assert np.array_equal(np.array(np.random.get_state()[1][:8], dtype=np.uint32), g[k + '_state'])


def test_ber_sweep_sc_fdm(golden_scfdm, oracle):
    """OFDMModule(enable_sc_fdm=True).run_ber_sweep: bits drawn once from the
    global RNG, then simulate_siso per (SNR, trial) (ofdm_core.py:1795-1846)."""
    g = golden_scfdm
    num = oracle.Numerology(bandwidth=5.0, modulation='QPSK')
    np.random.seed(777)
    bits = np.random.randint(0, 2, 4000)
    ber, pap = [], []
    for snr in [0.0, 5.0, 10.0]:
        rr = [oracle.simulate_siso(num, bits, snr, sc_fdm=True) for _ in range(2)]
        ber.append(np.mean([r['ber'] for r in rr]))
        pap.append(np.mean([r['papr_db'] for r in rr]))
    assert np.array_equal(np.array(ber), g['sweep_ber'])
    assert np.array_equal(np.array(pap), g['sweep_papr'])
