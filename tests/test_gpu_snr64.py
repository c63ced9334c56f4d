"""GPU: the float64 chains at SNRs float32 cannot represent, against the
reference's own outputs (tests/golden/golden_r5.npz, tests/golden/make_golden_r5.py).

The reference holds snr_db as a Python float and forms 10 ** (snr_db / 10)
(core/channel.py:32,191), 1 / 10 ** (snr_db / 10) (core/ofdm_core.py:1224) and
10 ** (-snr_db / 10) (:2397, :2737) in float64; lte_run_args.snr_db is double
since ABI 3 (include/lte_phy.h).  Bars (float64): identical bit errors,
received bits, CRC verdicts and global-RNG state; signal_rx within 1e-13
relative (L2); combined symbols 1e-12.  A control run at the float32-rounded
SNR shows the signal bar can see the difference."""
import numpy as np
import pytest

from conftest import unpack

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def C():
    from lte_phy import _capi
    _capi.device_init(0)
    return _capi


def _state():
    return np.array(np.random.get_state()[1][:8], dtype=np.uint32)


def _rel(a, b):
    return np.linalg.norm(np.asarray(a) - b) / np.linalg.norm(b)


def _bits(g, name):
    nb = int(g[name + '_nbits'][0])
    return unpack(g[name + '_bits'], nb).astype(np.int64), nb


def _sim(bw, mod, chan='rayleigh_mp', **kw):
    import lte_phy
    return lte_phy.OFDMSimulator(lte_phy.LTEConfig(bandwidth=bw, modulation=mod), channel_type=chan, **kw)


def test_siso_c2_7p3(C, golden_r5):
    sim = _sim(20.0, '64-QAM')
    bits, nb = _bits(golden_r5, 'siso_c2')
    k = 'siso_c2_snr7.3'
    r = sim.simulate_siso(bits, 7.3)
    assert np.array_equal(_state(), golden_r5[k + '_state'])
    assert r['bit_errors'] == int(golden_r5[k + '_errors'][0])
    assert np.array_equal(r['bits_received_array'], unpack(golden_r5[k + '_rx'], nb))
    assert _rel(r['signal_rx'], golden_r5[k + '_sigrx']) < 1e-13
    g = golden_r5[k + '_symrx']
    assert _rel(np.asarray(r['symbols_rx'])[:len(g)], g) < 1e-12
    assert abs(r['papr_db'] - golden_r5[k + '_papr'][0]) < 1e-9
    # control: the float32-rounded SNR moves the noise scale by ~1e-8
    r32 = sim.simulate_siso(bits, float(np.float32(7.3)))
    assert _rel(r32['signal_rx'], golden_r5[k + '_sigrx']) > 1e-10


@pytest.mark.parametrize('snr', [9.7, 18.6])
def test_coded_tb2000(C, golden_r5, snr):
    sim = _sim(20.0, '64-QAM')
    bits, nb = _bits(golden_r5, 'cod_c2s')
    k = f'cod_c2s_snr{snr}'
    r = sim.simulate_siso_coded(bits, snr)
    assert np.array_equal(_state(), golden_r5[k + '_state'])
    assert r['bit_errors'] == int(golden_r5[k + '_errors'][0])
    assert int(r['crc_pass']) == int(golden_r5[k + '_crc'][0])
    assert np.array_equal(r['bits_received_array'], unpack(golden_r5[k + '_rx'], nb))
    assert abs(r['channel_snr_db'] - golden_r5[k + '_chsnr'][0]) < 1e-9
    assert abs(r['noise_var_mean'] / golden_r5[k + '_nvmean'][0] - 1) < 1e-12
    assert _rel(r['signal_rx'], golden_r5[k + '_sigrx']) < 1e-13


def test_simo_c3_12p1(C, golden_r5):
    sim = _sim(10.0, '16-QAM', itu_profile='Vehicular_A')
    bits, nb = _bits(golden_r5, 'c3')
    k = 'c3_snr12.1'
    r = sim.simulate_simo(bits, 12.1, num_rx=4, parallel=False)
    assert np.array_equal(_state(), golden_r5[k + '_state'])
    assert r['bit_errors'] == int(golden_r5[k + '_errors'][0])
    assert np.array_equal(r['bits_received_array'], unpack(golden_r5[k + '_rx'], nb))
    g = golden_r5[k + '_comb']
    assert _rel(np.asarray(r['symbols_rx_combined'])[:len(g)], g) < 1e-12


def test_sweep_tenth_db(C, golden_r5):
    """OFDMModule.run_ber_sweep over np.arange(0, 1.0, 0.1): one batched call,
    every (SNR, trial) frame at its own float64 SNR."""
    import lte_phy
    m = lte_phy.OFDMModule(lte_phy.LTEConfig(bandwidth=1.25, modulation='QPSK'))
    np.random.seed(0)
    res = m.run_ber_sweep(14 * 62 * 2, np.arange(0, 1.0, 0.1), num_trials=2)
    assert np.array_equal(np.asarray(res['snr_db'], dtype=np.float64), golden_r5['sweep01_snr'])
    assert np.array_equal(res['ber_mean'], golden_r5['sweep01_ber_mean'])
    assert np.array_equal(res['ber_values'], golden_r5['sweep01_ber_values'])
    assert np.max(np.abs(res['papr_values'] - golden_r5['sweep01_papr'])) < 1e-9
    assert np.array_equal(_state(), golden_r5['sweep01_state'])


def test_sfbc_c4_13p7(C, golden_r5):
    sim = _sim(20.0, '64-QAM')
    bits, nb = _bits(golden_r5, 'sfbc_c4')
    k = 'sfbc_c4_snr13.7'
    r = sim.simulate_mimo(bits, 13.7, num_rx=2)
    assert np.array_equal(_state(), golden_r5[k + '_state'])
    assert r['bit_errors'] == int(golden_r5[k + '_errors'][0])
    assert np.array_equal(r['bits_received_array'], unpack(golden_r5[k + '_rx'], nb))
    H = golden_r5[k + '_H']
    assert np.max(np.abs(r['channel_matrix'] - H)) < 1e-12 * (1 + np.max(np.abs(H)))
    assert np.allclose([r['papr_db_tx0'], r['papr_db_tx1'], r['papr_db']], golden_r5[k + '_papr'], rtol=0,
                       atol=1e-9)


@pytest.mark.parametrize('name,chan,snr', [('sm_c5ray', 'rayleigh_mp', 27.3), ('sm_c5awgn', 'awgn', 21.9)])
def test_spatial(C, golden_r5, name, chan, snr):
    import lte_phy
    bits, nb = _bits(golden_r5, name)
    k = f'{name}_snr{snr}'
    r = lte_phy.simulate_spatial_multiplexing(bits, num_tx=4, num_rx=4, rank=4, detector_type='MMSE',
                                              modulation='64-QAM', snr_db=snr,
                                              config=lte_phy.LTEConfig(bandwidth=20.0, modulation='64-QAM'),
                                              channel_type=chan, itu_profile='Pedestrian_A', velocity_kmh=3,
                                              enable_csi_feedback=False)
    assert np.array_equal(_state(), golden_r5[k + '_state'])
    assert r['bit_errors'] == int(golden_r5[k + '_errors'][0])
    assert np.array_equal(r['bits_received_array'], unpack(golden_r5[k + '_rx'], nb))
    assert np.array_equal(r['channel_matrix'], golden_r5[k + '_H'])
