"""GPU parity of SC-FDM (DFT-precoded OFDM,
core/dft_precoding.py) against the reference's own outputs
(tests/golden/golden_scfdm.npz, frozen global RNG) and the oracle.

Bars: the Bluestein M-point DFT (float32 on the device) within 2e-6 relative
L2 of the reference's float64 DFT matrix; TX stream within 1e-5 relative;
end to end BER within the north_star 1e-3 of the reference, PAPR within
1e-3 dB, identical global-RNG side effects."""
import numpy as np
import pytest

from conftest import unpack

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def C():
    from lte_phy import _capi
    _capi.device_init(0)
    return _capi


def _state_head():
    return np.array(np.random.get_state()[1][:8], dtype=np.uint32)


def _rel(a, b):
    return np.linalg.norm(a - b) / np.linalg.norm(b)


@pytest.mark.parametrize('M', [62, 249, 499, 999])
def test_dft_stage_vs_reference(C, golden_scfdm, M):
    g = golden_scfdm
    X = C.dft(g[f'dft{M}_x'][None])[0]
    assert _rel(X, g[f'dft{M}_X']) < 2e-6
    x = C.dft(g[f'dft{M}_X'][None], inverse=True)[0]
    assert _rel(x, g[f'dft{M}_inv']) < 2e-6


def test_dft_stage_batch_and_sizes(C):
    """Batched transforms of every size the Bluestein path accepts (M <= 1024)."""
    rs = np.random.RandomState(3)
    for M in (1, 2, 3, 17, 64, 300, 1024):
        x = rs.randn(5, M) + 1j * rs.randn(5, M)
        X = C.dft(x)
        ref = np.fft.fft(x, axis=1) / np.sqrt(M)
        assert _rel(X, ref) < 3e-6, M
        assert _rel(C.dft(X, inverse=True), x) < 3e-6, M
    with pytest.raises(ValueError):
        C.dft(np.zeros((1, 1025)))


def test_transmitter_sc_fdm(C, golden_scfdm):
    import lte_phy
    g = golden_scfdm
    tx = lte_phy.OFDMTransmitter(lte_phy.LTEConfig(bandwidth=1.25, modulation='QPSK'), enable_sc_fdm=True)
    bits = unpack(g['tx_bits'], int(g['tx_nbits'][0])).astype(np.int64)
    sig, syms, infos = tx.modulate(bits)
    assert _rel(sig, g['tx_signal']) < 1e-5
    assert np.max(np.abs(np.array(syms) - g['tx_syms'])) < 1e-7
    assert abs(tx.calculate_papr(sig)['papr_db'] - g['tx_papr'][0]) < 1e-3
    assert 'SC-FDM' in repr(tx)
    tx2 = lte_phy.OFDMTransmitter(lte_phy.LTEConfig(bandwidth=1.25, modulation='QPSK'), mode='sc-fdm')
    assert _rel(tx2.modulate(bits)[0], g['tx_signal']) < 1e-5


@pytest.mark.parametrize('name,bw,mod,chan,snrs,fn', [
    ('sc_c1', 1.25, 'QPSK', 'awgn', [0, 5, 10], 'siso'),
    ('sc_c1odd', 1.25, '16-QAM', 'awgn', [12], 'siso'),
    ('sc_c5m', 5.0, 'QPSK', 'awgn', [3], 'siso'),
    ('sc_c2', 20.0, '64-QAM', 'rayleigh_mp', [10, 20, 30], 'siso'),
    ('sc_c3', 10.0, '16-QAM', 'rayleigh_mp', [15], 'siso'),
    ('sc_simo', 1.25, 'QPSK', 'awgn', [10], 'simo'),
    ('noeq_c1', 1.25, 'QPSK', 'awgn', [5, 10], 'noeq'),
    ('noeq_c2', 20.0, '16-QAM', 'rayleigh_mp', [20], 'noeq'),
    ('noeq_sc', 1.25, 'QPSK', 'awgn', [10], 'noeq_sc')])
def test_sc_fdm_ref_compat(C, golden_scfdm, name, bw, mod, chan, snrs, fn):
    """SC-FDM drivers, and the receiver without equalisation (noeq*:
    enable_equalization=False, with and without SC-FDM)."""
    import lte_phy
    g = golden_scfdm
    sim = lte_phy.OFDMSimulator(lte_phy.LTEConfig(bandwidth=bw, modulation=mod), channel_type=chan,
                                enable_sc_fdm=fn != 'noeq', enable_equalization=not fn.startswith('noeq'))
    fn = 'siso' if fn.startswith('noeq') else fn
    nb = int(g[name + '_nbits'][0])
    bits = unpack(g[name + '_bits'], nb).astype(np.int64)
    for snr in snrs:
        k = f'{name}_snr{snr}'
        r = sim.simulate_siso(bits, snr) if fn == 'siso' else sim.simulate_simo(bits, snr, num_rx=2, parallel=False)
        ref_err = int(g[k + '_errors'][0])
        assert abs(r['bit_errors'] - ref_err) / nb < 1e-3, (k, r['bit_errors'], ref_err)
        diff = np.mean(r['bits_received_array'] != unpack(g[k + '_rx'], nb))
        assert diff < 1e-3, (k, diff)
        assert abs(r['papr_db'] - g[k + '_papr'][0]) < 1e-3
        assert np.array_equal(_state_head(), g[k + '_state'])
        if k + '_sigtx' in g:
            assert _rel(r['signal_tx'], g[k + '_sigtx']) < 1e-5
        if k + '_symrx' in g:
            assert np.median(np.abs(r['symbols_rx'] - g[k + '_symrx'])) < 1e-4


def test_ber_sweep_sc_fdm(C, golden_scfdm):
    import lte_phy
    g = golden_scfdm
    m = lte_phy.OFDMModule(enable_sc_fdm=True)
    np.random.seed(777)
    sw = m.run_ber_sweep(num_bits=4000, snr_range=np.array([0.0, 5.0, 10.0]), num_trials=2)
    assert np.max(np.abs(sw['ber_mean'] - g['sweep_ber'])) < 1e-3
    assert np.max(np.abs(sw['papr_values'] - g['sweep_papr'])) < 1e-3
    assert np.array_equal(_state_head(), g['sweep_state'])


def test_run_grid_sc_fdm(C):
    """Philox grid with SC-FDM: BER falls with SNR and SC-FDM changes the chain."""
    import lte_phy
    cfg = lte_phy.LTEConfig(bandwidth=5.0, modulation='16-QAM')
    a = lte_phy.OFDMSimulator(cfg, enable_sc_fdm=True).run_grid([0.0, 10.0, 20.0], 8, seed=1, frames_per_call=8)
    b = lte_phy.OFDMSimulator(cfg).run_grid([0.0, 10.0, 20.0], 8, seed=1, frames_per_call=8)
    assert a['ber'][0] > a['ber'][1] > a['ber'][2]
    assert not np.array_equal(a['counts'], b['counts'])
