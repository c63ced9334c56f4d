"""Pin the CPU oracle to the reference: every check below compares the oracle
with golden vectors produced by running the reference itself
(tests/golden/make_golden.py).  Equalities are exact (the oracle restates the
reference's float64 arithmetic operation-for-operation)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import unpack

MAN = json.load(open(os.path.join(os.path.dirname(__file__), 'golden', 'golden_manifest.json')))
MODS = ['QPSK', '16-QAM', '64-QAM']


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize('bw', [1.25, 2.5, 5.0, 10.0, 15.0, 20.0])
@pytest.mark.parametrize('cpt', ['normal', 'extended'])
def test_numerology(golden, oracle, bw, cpt):
    n = oracle.Numerology(bandwidth=bw, modulation='QPSK', cp_type=cpt)
    key = f'num_{bw}_{cpt}'
    sc = golden[key + '_scalars']
    assert [n.N, n.Nc, n.fs, n.cp, n.N + n.cp] == list(sc)
    assert np.array_equal(n.data_idx, golden[key + '_data'])
    assert np.array_equal(n.pilot_idx, golden[key + '_pilot'])


@pytest.mark.parametrize('cell', range(4))
def test_pilots(golden, oracle, cell):
    assert np.array_equal(oracle.pilots(cell, 200), golden[f'pilots_cell{cell}'])


@pytest.mark.parametrize('mod', MODS)
def test_qam_map_and_hard(golden, oracle, mod):
    bits = golden[f'qam_{mod}_bits'].astype(np.int64)
    assert np.array_equal(oracle.bits_to_symbols(bits, mod), golden[f'qam_{mod}_syms'])
    hard = oracle.symbols_to_bits(golden[f'qam_{mod}_pts'], mod)
    assert np.array_equal(hard, golden[f'qam_{mod}_hard'])


def test_modulate_c1(golden, oracle):
    n = oracle.Numerology(bandwidth=1.25, modulation='QPSK')
    sig, _, _ = oracle.modulate_stream(n, golden['mod_c1_bits'].astype(np.int64))
    assert np.array_equal(sig, golden['mod_c1_signal'])


@pytest.mark.parametrize('fD', [0.0, 5.5555555556, 55.555555556])
def test_jakes_filter(golden, oracle, fD):
    x = golden[f'jakes_fD{fD:.3f}_x']
    delays = [int(np.round(d * 1.92e6)) for d in [0.0, 0.11e-6 * 10, 0.41e-6 * 10]]
    gains = 10 ** (np.array(10 ** (np.array([0.0, -9.7, -22.8]) / 20)) / 20)
    np.random.seed(321)
    ph = [2 * np.pi * np.random.rand(16) for _ in delays]
    y = oracle.multipath(x, delays, gains, ph, fD, 1.92e6)
    assert np.array_equal(y, golden[f'jakes_fD{fD:.3f}_y'])


def test_channel_estimate_zf(golden, oracle):
    n = oracle.Numerology(bandwidth=20.0, modulation='64-QAM')
    H, snr = oracle.estimate_channel(n, golden['chest_Y'])
    assert np.array_equal(H, golden['chest_H'])
    assert snr == golden['chest_snr_db'][0]
    assert np.array_equal(golden['chest_Y'] / (H + 1e-6), golden['zf_out'])


@pytest.mark.parametrize('mod', MODS)
def test_llrs(golden, oracle, mod):
    out = oracle.llrs(golden['llr_pts'], golden['llr_nv'], mod)
    assert np.array_equal(out, golden[f'llr_{mod}'])


@pytest.mark.parametrize('vec', ['zeros40', 'ones40', 'alt40', 'rand27760'])
def test_crc(golden, oracle, vec):
    v = golden[f'crc_{vec}_in']
    assert np.array_equal(oracle.crc_bits(v, oracle.CRC24A_POLY, 24), golden[f'crc_{vec}_24a'])
    assert np.array_equal(oracle.crc_bits(v, oracle.CRC24B_POLY, 24), golden[f'crc_{vec}_24b'])
    assert np.array_equal(oracle.crc_bits(v, oracle.CRC16_POLY, 16), golden[f'crc_{vec}_16'])


@pytest.mark.parametrize('B', [40, 6144, 6145, 9232, 27784])
def test_segmentation(golden, oracle, B):
    tb = unpack(golden[f'seg_{B}_tb'], B)
    blocks, plan = oracle.segment(tb)
    assert [p[0] for p in plan] == list(golden[f'seg_{B}_sizes'])
    cat = np.concatenate(blocks)
    assert np.array_equal(cat, unpack(golden[f'seg_{B}_blocks'], len(cat)))
    assert np.array_equal(oracle.desegment(blocks, plan), tb)


@pytest.mark.parametrize('K', [40, 1024, 5568, 5632, 6144])
def test_turbo_encode_rate_match(golden, oracle, K):
    cb = unpack(golden[f'enc_{K}_in'], K)
    enc = oracle.turbo_encode(cb)
    assert np.array_equal(enc, unpack(golden[f'enc_{K}_out'], 3 * K + 12))
    E = 3 * K + 12
    assert np.array_equal(oracle.rate_match(enc, E, K, 0), unpack(golden[f'rm_{K}_out'], E))
    assert np.array_equal(oracle.rate_dematch(golden[f'dm_{K}_in'], K, 0), golden[f'dm_{K}_out'])
    for E2 in [K + 17, 4 * K]:
        assert np.array_equal(oracle.rate_match(enc, E2, K, 2), unpack(golden[f'rm_{K}_E{E2}'], E2))
        assert np.array_equal(oracle.rate_dematch(golden[f'dm_{K}_E{E2}_in'], K, 2), golden[f'dm_{K}_E{E2}_out'])


@pytest.mark.parametrize('K,its', [(40, 8), (1024, 1), (1024, 8), (5568, 2)])
def test_turbo_decode(golden, oracle, K, its):
    key = f'td_{K}_{its}'
    if key + '_llr' not in golden:
        pytest.skip('slow vector not generated')
    dec = oracle.turbo_decode(golden[key + '_llr'], K, its)
    assert np.array_equal(dec, unpack(golden[key + '_dec'], K))


def test_bcjr_app(golden, oracle):
    app = oracle.bcjr_app(golden['bcjr_ls'], golden['bcjr_lp'], golden['bcjr_la'])
    assert np.array_equal(app, golden['bcjr_app'])


def _state_head():
    return np.array(np.random.get_state()[1][:8], dtype=np.uint32)


E2E = [('e2e_c1', 1.25, 'QPSK', 'awgn', [0, 5, 10], 'siso'),
       ('e2e_c1odd', 1.25, 'QPSK', 'awgn', [3], 'siso'),
       ('e2e_c2', 20.0, '64-QAM', 'rayleigh_mp', [0, 10, 20, 30], 'siso'),
       ('e2e_c2awgn', 20.0, '16-QAM', 'awgn', [12], 'siso'),
       ('e2e_c3', 10.0, '16-QAM', 'rayleigh_mp', [5, 15], 'simo'),
       ('e2e_c1simo', 1.25, 'QPSK', 'awgn', [2], 'simo'),
       ('e2e_cod_small', 1.25, 'QPSK', 'awgn', [0, 6], 'coded'),
       ('e2e_cod_c2s', 20.0, '64-QAM', 'rayleigh_mp', [8, 20], 'coded'),
       ('e2e_cod_c2', 20.0, '64-QAM', 'rayleigh_mp', [20], 'coded')]


@pytest.mark.parametrize('name,bw,mod,chan,snrs,fn', E2E)
def test_end_to_end(golden, oracle, name, bw, mod, chan, snrs, fn):
    if name + '_nbits' not in golden:
        pytest.skip('slow vector not generated')
    nb = int(golden[name + '_nbits'][0])
    bits = unpack(golden[name + '_bits'], nb).astype(np.int64)
    num = oracle.Numerology(bandwidth=bw, modulation=mod)
    for snr in snrs:
        k = f'{name}_snr{snr}'
        if fn == 'siso':
            r = oracle.simulate_siso(num, bits, snr, chan)
        elif fn == 'simo':
            r = oracle.simulate_simo(num, bits, snr, num_rx=4 if name == 'e2e_c3' else 2, channel=chan)
        else:
            r = oracle.simulate_siso_coded(num, bits, snr, chan)
        assert r['bit_errors'] == int(golden[k + '_errors'][0]), k
        assert np.array_equal(r['bits_received_array'], unpack(golden[k + '_rx'], nb)), k
        assert r['papr_db'] == golden[k + '_papr'][0]
        assert np.array_equal(_state_head(), golden[k + '_state']), 'global RNG side effects differ'
        assert sha(r['signal_tx']) == MAN[k + '_sigtx_sha']
        if fn == 'simo':
            assert sha(r['symbols_rx_combined']) == MAN[k + '_comb_sha']
        else:
            assert sha(r['signal_rx']) == MAN[k + '_sigrx_sha']
        if fn == 'coded':
            assert int(r['crc_pass']) == int(golden[k + '_crc'][0])
            assert r['channel_snr_db'] == golden[k + '_chsnr'][0]
            assert r['noise_var_mean'] == golden[k + '_nvmean'][0]
            assert sha(r['symbols_rx']) == MAN[k + '_symbols_rx_sha']


def test_ref_compat_draws_reproduce(golden, oracle):
    """Injected draws (what the GPU path consumes) reproduce the frozen-RNG call."""
    num = oracle.Numerology(bandwidth=20.0, modulation='64-QAM')
    bits = unpack(golden['e2e_c2_bits'], int(golden['e2e_c2_nbits'][0])).astype(np.int64)
    L = 14 * (num.N + num.cp)
    d = oracle.ref_compat_draws(num, 'rayleigh_mp', L)
    r = oracle.simulate_siso(num, bits, 20, 'rayleigh_mp', draws=d)
    assert r['bit_errors'] == int(golden['e2e_c2_snr20_errors'][0])
    assert sha(r['signal_rx']) == MAN['e2e_c2_snr20_sigrx_sha']
