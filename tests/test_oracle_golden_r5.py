"""CPU: the float64 oracle against the round-5 reference goldens
(tests/golden/make_golden_r5.py): every chain at an SNR float32 cannot
represent (7.3, 9.7, 18.6, 12.1, 13.7, 27.3, 21.9 dB and a 0.1-dB
run_ber_sweep).  All exact; signal_rx to the last bit."""
import numpy as np
import pytest

from conftest import unpack


def _state_head():
    return np.array(np.random.get_state()[1][:8], dtype=np.uint32)


def _bits(g, name):
    nb = int(g[name + '_nbits'][0])
    return unpack(g[name + '_bits'], nb).astype(np.int64), nb


def test_float32_cannot_hold_these_snrs():
    for s in (7.3, 9.7, 18.6, 12.1, 13.7, 27.3, 21.9, 0.1):
        assert float(np.float32(s)) != s
        assert 10 ** (float(np.float32(s)) / 10) != 10 ** (s / 10)


def test_siso_c2_7p3(golden_r5, oracle):
    num = oracle.Numerology(bandwidth=20.0, modulation='64-QAM')
    bits, nb = _bits(golden_r5, 'siso_c2')
    r = oracle.simulate_siso(num, bits, 7.3, 'rayleigh_mp')
    k = 'siso_c2_snr7.3'
    assert r['bit_errors'] == int(golden_r5[k + '_errors'][0])
    assert np.array_equal(r['bits_received_array'], unpack(golden_r5[k + '_rx'], nb))
    assert np.array_equal(r['signal_rx'], golden_r5[k + '_sigrx'])
    assert np.array_equal(_state_head(), golden_r5[k + '_state'])


@pytest.mark.parametrize('snr', [9.7, 18.6])
def test_coded_tb2000(golden_r5, oracle, snr):
    num = oracle.Numerology(bandwidth=20.0, modulation='64-QAM')
    bits, nb = _bits(golden_r5, 'cod_c2s')
    r = oracle.simulate_siso_coded(num, bits, snr, 'rayleigh_mp')
    k = f'cod_c2s_snr{snr}'
    assert r['bit_errors'] == int(golden_r5[k + '_errors'][0])
    assert int(r['crc_pass']) == int(golden_r5[k + '_crc'][0])
    assert np.array_equal(r['bits_received_array'], unpack(golden_r5[k + '_rx'], nb))
    assert r['channel_snr_db'] == golden_r5[k + '_chsnr'][0]
    assert r['noise_var_mean'] == golden_r5[k + '_nvmean'][0]
    assert np.array_equal(r['signal_rx'], golden_r5[k + '_sigrx'])
    assert np.array_equal(_state_head(), golden_r5[k + '_state'])


def test_simo_c3_12p1(golden_r5, oracle):
    num = oracle.Numerology(bandwidth=10.0, modulation='16-QAM')
    bits, nb = _bits(golden_r5, 'c3')
    r = oracle.simulate_simo(num, bits, 12.1, num_rx=4, channel='rayleigh_mp', profile='Vehicular_A')
    k = 'c3_snr12.1'
    assert r['bit_errors'] == int(golden_r5[k + '_errors'][0])
    assert np.array_equal(r['symbols_rx_combined'], golden_r5[k + '_comb'])
    assert np.array_equal(_state_head(), golden_r5[k + '_state'])


def test_sweep_tenth_db(golden_r5, oracle):
    """run_ber_sweep (core/ofdm_core.py:1795-1846): one bit draw, then
    simulate_siso per (SNR, trial) in order, mean per SNR; restated on the
    oracle."""
    num = oracle.Numerology(bandwidth=1.25, modulation='QPSK')
    snrs = np.arange(0, 1.0, 0.1)
    assert np.array_equal(snrs, golden_r5['sweep01_snr'])
    np.random.seed(0)
    bits = np.random.randint(0, 2, 14 * 62 * 2)      # drawn once (:1816), every trial reuses it
    vals = np.array([np.mean([oracle.simulate_siso(num, bits, snr, 'awgn')['ber'] for _ in range(2)])
                     for snr in snrs])
    assert np.array_equal(vals, golden_r5['sweep01_ber_values'])
    assert np.array_equal(vals, golden_r5['sweep01_ber_mean'])
    assert np.array_equal(_state_head(), golden_r5['sweep01_state'])


def test_sfbc_c4_13p7(golden_r5, oracle, mimo_oracle):
    num = oracle.Numerology(bandwidth=20.0, modulation='64-QAM')
    bits, nb = _bits(golden_r5, 'sfbc_c4')
    r = mimo_oracle.simulate_sfbc(num, bits, 13.7, num_rx=2, channel='rayleigh_mp')
    k = 'sfbc_c4_snr13.7'
    assert r['bit_errors'] == int(golden_r5[k + '_errors'][0])
    assert np.array_equal(r['bits_received_array'], unpack(golden_r5[k + '_rx'], nb))
    assert np.array_equal(r['channel_matrix'], golden_r5[k + '_H'])
    assert np.array_equal(_state_head(), golden_r5[k + '_state'])


@pytest.mark.parametrize('name,chan,snr', [('sm_c5ray', 'rayleigh_mp', 27.3), ('sm_c5awgn', 'awgn', 21.9)])
def test_spatial(golden_r5, oracle, mimo_oracle, name, chan, snr):
    num = oracle.Numerology(bandwidth=20.0, modulation='64-QAM')
    bits, nb = _bits(golden_r5, name)
    r = mimo_oracle.simulate_spatial(num, bits, snr, channel=chan)
    k = f'{name}_snr{snr}'
    assert r['bit_errors'] == int(golden_r5[k + '_errors'][0])
    assert np.array_equal(r['bits_received_array'], unpack(golden_r5[k + '_rx'], nb))
    assert np.array_equal(r['channel_matrix'], golden_r5[k + '_H'])
    assert np.array_equal(_state_head(), golden_r5[k + '_state'])
