"""CPU: the float64 oracle against the round-2 reference goldens
(tests/golden/make_golden_r2.py): the coded config-2 BER curve at every SNR of
0:2:30 dB, config 3 with the Vehicular-A profile, and run_ber_sweep.  All
exact (the oracle restates the reference's float64 operations in order)."""
import json
import os

import numpy as np
import pytest

from conftest import ROOT, unpack

MAN = json.load(open(os.path.join(ROOT, 'tests', 'golden', 'golden_r2_manifest.json')))


def sha(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _state_head():
    return np.array(np.random.get_state()[1][:8], dtype=np.uint32)


@pytest.mark.parametrize('snr', [0, 8, 16, 18, 20, 30])
def test_coded_curve_points(golden_r2, oracle, snr):
    num = oracle.Numerology(bandwidth=20.0, modulation='64-QAM')
    nb = int(golden_r2['cod_curve_nbits'][0])
    bits = unpack(golden_r2['cod_curve_bits'], nb).astype(np.int64)
    r = oracle.simulate_siso_coded(num, bits, snr, 'rayleigh_mp')
    k = f'cod_curve_snr{snr}'
    assert r['bit_errors'] == int(golden_r2[k + '_errors'][0])
    assert int(r['crc_pass']) == int(golden_r2[k + '_crc'][0])
    assert np.array_equal(r['bits_received_array'], unpack(golden_r2[k + '_rx'], nb))
    assert r['channel_snr_db'] == golden_r2[k + '_chsnr'][0]
    assert r['noise_var_mean'] == golden_r2[k + '_nvmean'][0]
    assert sha(r['signal_rx']) == MAN[k + '_sigrx_sha']
    assert np.array_equal(_state_head(), golden_r2[k + '_state'])


@pytest.mark.parametrize('snr', [5, 15])
def test_config3_vehicular_a(golden_r2, oracle, snr):
    num = oracle.Numerology(bandwidth=10.0, modulation='16-QAM')
    nb = int(golden_r2['c3veha_nbits'][0])
    bits = unpack(golden_r2['c3veha_bits'], nb).astype(np.int64)
    r = oracle.simulate_simo(num, bits, snr, num_rx=4, channel='rayleigh_mp', profile='Vehicular_A')
    k = f'c3veha_snr{snr}'
    assert r['bit_errors'] == int(golden_r2[k + '_errors'][0])
    assert np.array_equal(r['symbols_rx_combined'], golden_r2[k + '_comb'])
    assert sha(r['signal_tx']) == MAN[k + '_sigtx_sha']
    assert np.array_equal(_state_head(), golden_r2[k + '_state'])


def test_fixture_curve_covers_cliff(fixture_curve):
    """The oracle BER-curve fixture spans the turbo cliff: failing frames at low
    SNR, clean frames at high SNR (so the GPU comparison exercises both)."""
    crc = fixture_curve['crc_ok']
    assert crc[0].sum() == 0 and crc[-1].all()
    assert fixture_curve['bit_errors'].shape == (16, int(fixture_curve['frames'][0]))
