"""CPU: the beamforming oracle (oracle/bf_oracle.py)
against vectors from running the reference (tests/golden/make_golden_bf.py):
MRT / eigen precoders, beamforming gain, CSI feedback (PMI / CQI / RI / SINR),
the adaptive update period and simulate_beamforming end to end.  Exact
equality unless stated."""
import numpy as np
import pytest

from conftest import unpack

MODS = {2: 'QPSK', 4: '16-QAM', 6: '64-QAM'}


def test_precoders_and_feedback(golden_bf, bf_oracle):
    g = golden_bf
    for i in range(int(g['p_n'][0])):
        ntx, nrx, tm4 = (int(v) for v in g[f'p{i}_cfg'])
        H = g[f'p{i}_H']
        wm = bf_oracle.mrt_weights(H)
        assert np.array_equal(wm, g[f'p{i}_wmrt'])
        we = bf_oracle.eigen_weights(H)
        assert np.array_equal(we, g[f'p{i}_weig'])
        assert [bf_oracle.bf_gain_db(H, wm), bf_oracle.bf_gain_db(H, we)] == list(g[f'p{i}_gain'])
        assert np.array_equal(wm @ g[f'p{i}_s'].reshape(1, -1), g[f'p{i}_x'])
        fb = bf_oracle.csi_feedback(H, ntx, 'TM4' if tm4 else 'TM6', 0.3)
        assert [fb['pmi'], fb['cqi'], fb['ri'], fb['sinr_db']] == list(g[f'p{i}_fb']), i
        assert np.array_equal(fb['precoder'], g[f'p{i}_fbW'])


def test_update_period(golden_bf, bf_oracle):
    assert [bf_oracle.update_period(v) for v in (0.0, 3.0, 30.0, 120.0, 500.0)] == list(golden_bf['update_period'])


@pytest.mark.parametrize('name', ['bf_21a', 'bf_42s', 'bf_81a', 'bf_24s', 'bf_44a'])
def test_simulate_beamforming_e2e(golden_bf, oracle, bf_oracle, name):
    g = golden_bf
    bw, bps, snr, ntx, nrx, tm4, adaptive, v, seed = g[f'{name}_cfg']
    num = oracle.Numerology(bandwidth=float(bw), modulation=MODS[int(bps)])
    n = int(g[f'{name}_nbits'][0])
    bits = unpack(g[f'{name}_bits'], n).astype(np.int64)
    np.random.seed(int(seed))
    r = bf_oracle.simulate_beamforming(num, bits, float(snr), int(ntx), int(nrx), 'TM4' if tm4 else 'TM6',
                                       'adaptive' if adaptive else 'static')
    assert r['bit_errors'] == g[f'{name}_errors'][0]
    assert np.array_equal(r['bits_received_array'], unpack(g[f'{name}_rx'], n))
    assert np.array_equal(r['channel_matrix'], g[f'{name}_H'])
    assert np.array_equal(np.array(r['pmi_history']), g[f'{name}_pmi'])
    assert [r['beamforming_gain_db'], r['unique_pmis']] == list(g[f'{name}_gain'])
    assert np.array_equal(np.array(np.random.get_state()[1][:8], dtype=np.uint32), g[f'{name}_state'])
