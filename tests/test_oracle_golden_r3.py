"""CPU: the float64 oracle against the round-3 reference goldens
(tests/golden/make_golden_r3.py): the SISO / SIMO chains with the UE at 3 km/h
(fD = 5.556 Hz at 2 GHz, the GUI default): coded config 2, uncoded config 2,
config 3 (Vehicular-A).  All exact."""
import json
import os

import numpy as np
import pytest

from conftest import ROOT, unpack

MAN = json.load(open(os.path.join(ROOT, 'tests', 'golden', 'golden_r3_manifest.json')))


def sha(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _state_head():
    return np.array(np.random.get_state()[1][:8], dtype=np.uint32)


def _fd(oracle):
    return oracle.doppler_hz(2.0, MAN['velocity_kmh'])


@pytest.mark.parametrize('snr', [8, 20])
def test_coded_3kmh(golden_r3, oracle, snr):
    num = oracle.Numerology(bandwidth=20.0, modulation='64-QAM')
    nb = int(golden_r3['v3cod_nbits'][0])
    bits = unpack(golden_r3['v3cod_bits'], nb).astype(np.int64)
    r = oracle.simulate_siso_coded(num, bits, snr, 'rayleigh_mp', fD=_fd(oracle))
    k = f'v3cod_snr{snr}'
    assert r['bit_errors'] == int(golden_r3[k + '_errors'][0])
    assert int(r['crc_pass']) == int(golden_r3[k + '_crc'][0])
    assert np.array_equal(r['bits_received_array'], unpack(golden_r3[k + '_rx'], nb))
    assert r['channel_snr_db'] == golden_r3[k + '_chsnr'][0]
    assert r['noise_var_mean'] == golden_r3[k + '_nvmean'][0]
    assert sha(r['signal_rx']) == MAN[k + '_sigrx_sha']
    assert np.array_equal(_state_head(), golden_r3[k + '_state'])


@pytest.mark.parametrize('snr', [10, 20])
def test_uncoded_3kmh(golden_r3, oracle, snr):
    num = oracle.Numerology(bandwidth=20.0, modulation='64-QAM')
    nb = int(golden_r3['v3siso_nbits'][0])
    bits = unpack(golden_r3['v3siso_bits'], nb).astype(np.int64)
    r = oracle.simulate_siso(num, bits, snr, 'rayleigh_mp', fD=_fd(oracle))
    k = f'v3siso_snr{snr}'
    assert r['bit_errors'] == int(golden_r3[k + '_errors'][0])
    assert np.array_equal(r['bits_received_array'], unpack(golden_r3[k + '_rx'], nb))
    assert sha(r['signal_rx']) == MAN[k + '_sigrx_sha']
    assert np.array_equal(_state_head(), golden_r3[k + '_state'])


@pytest.mark.parametrize('snr', [5, 15])
def test_config3_vehicular_a_3kmh(golden_r3, oracle, snr):
    num = oracle.Numerology(bandwidth=10.0, modulation='16-QAM')
    nb = int(golden_r3['v3c3_nbits'][0])
    bits = unpack(golden_r3['v3c3_bits'], nb).astype(np.int64)
    r = oracle.simulate_simo(num, bits, snr, num_rx=4, channel='rayleigh_mp', profile='Vehicular_A',
                             fD=_fd(oracle))
    k = f'v3c3_snr{snr}'
    assert r['bit_errors'] == int(golden_r3[k + '_errors'][0])
    assert np.array_equal(r['symbols_rx_combined'], golden_r3[k + '_comb'])
    assert np.array_equal(_state_head(), golden_r3[k + '_state'])
