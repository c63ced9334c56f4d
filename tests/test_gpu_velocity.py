"""GPU: the SISO / SIMO chains with a moving UE (fD > 0), against the
reference's own outputs at 3 km/h (tests/golden/golden_r3.npz, made by
tests/golden/make_golden_r3.py): OFDMSimulator(velocity_kmh=3) gives fD =
5.556 Hz at 2 GHz (core/channel.py:113-143) and a time-varying Jakes sum over
the whole stream (core/rayleighchannel.py:20-42), evaluated per sample on the
device.

Bars: float64 (default) -- identical bit errors, received bits, CRC verdict,
RNG state; measured SNR to 1e-9 dB, noise variance and received symbols to
1e-12 relative.  float32 fast mode -- |dBER| < 1e-3 (north_star) and the same
CRC verdicts."""
import numpy as np
import pytest

from conftest import unpack

pytestmark = pytest.mark.gpu

V = 3.0


@pytest.fixture(scope='module')
def C():
    from lte_phy import _capi
    _capi.device_init()
    return _capi


def _sim(bw, mod, prec, **kw):
    import lte_phy
    return lte_phy.OFDMSimulator(lte_phy.LTEConfig(bandwidth=bw, modulation=mod), channel_type='rayleigh_mp',
                                 velocity_kmh=V, precision=prec, **kw)


def _state_head():
    return np.array(np.random.get_state()[1][:8], dtype=np.uint32)


@pytest.mark.parametrize('prec', ['f64', 'f32'])
def test_coded_3kmh_vs_reference(C, golden_r3, prec):
    """simulate_siso_coded, config 2 (TB 27 760) at 3 km/h, 8 dB (past the
    cliff) and 20 dB."""
    import json
    import os
    from conftest import ROOT
    sim = _sim(20.0, '64-QAM', prec)
    man = json.load(open(os.path.join(ROOT, 'tests', 'golden', 'golden_r3_manifest.json')))
    assert sim.channels[0].fD == man['v3cod_snr8_fD']          # the reference's own fD, bit for bit
    nb = int(golden_r3['v3cod_nbits'][0])
    bits = unpack(golden_r3['v3cod_bits'], nb).astype(np.int64)
    for snr in (8, 20):
        k = f'v3cod_snr{snr}'
        r = sim.simulate_siso_coded(bits, float(snr))
        ref = int(golden_r3[k + '_errors'][0])
        assert bool(r['crc_pass']) == bool(golden_r3[k + '_crc'][0]), k
        assert np.array_equal(_state_head(), golden_r3[k + '_state']), k
        if prec == 'f64':
            assert r['bit_errors'] == ref, (k, r['bit_errors'], ref)
            assert np.array_equal(r['bits_received_array'], unpack(golden_r3[k + '_rx'], nb)), k
            assert abs(r['channel_snr_db'] - golden_r3[k + '_chsnr'][0]) < 1e-9, k
            assert abs(r['noise_var_mean'] / golden_r3[k + '_nvmean'][0] - 1) < 1e-12, k
        elif golden_r3[k + '_crc'][0]:
            assert abs(r['bit_errors'] - ref) / nb < 1e-3, (k, r['bit_errors'], ref)


@pytest.mark.parametrize('prec', ['f64', 'f32'])
def test_uncoded_3kmh_vs_reference(C, golden_r3, prec):
    """simulate_siso, config 2 uncoded (14 OFDM symbols) at 3 km/h, 10 / 20 dB."""
    sim = _sim(20.0, '64-QAM', prec)
    nb = int(golden_r3['v3siso_nbits'][0])
    bits = unpack(golden_r3['v3siso_bits'], nb).astype(np.int64)
    for snr in (10, 20):
        k = f'v3siso_snr{snr}'
        r = sim.simulate_siso(bits, snr)
        ref = int(golden_r3[k + '_errors'][0])
        g = golden_r3[k + '_symrx']
        rel = np.linalg.norm(np.asarray(r['symbols_rx'])[:len(g)] - g) / np.linalg.norm(g)
        assert np.array_equal(_state_head(), golden_r3[k + '_state']), k
        if prec == 'f64':
            assert r['bit_errors'] == ref, (k, r['bit_errors'], ref)
            assert np.array_equal(r['bits_received_array'], unpack(golden_r3[k + '_rx'], nb)), k
            assert rel < 1e-12, (k, rel)
        else:
            assert abs(r['bit_errors'] - ref) / nb < 1e-3, (k, r['bit_errors'], ref)
            assert rel < 1e-5, (k, rel)


@pytest.mark.parametrize('prec', ['f64', 'f32'])
def test_simo_config3_3kmh_vs_reference(C, golden_r3, prec):
    """simulate_simo, config 3 (SIMO 1x4 MRC, 10 MHz 16-QAM, Vehicular-A) at 3 km/h."""
    sim = _sim(10.0, '16-QAM', prec, itu_profile='Vehicular_A')
    nb = int(golden_r3['v3c3_nbits'][0])
    bits = unpack(golden_r3['v3c3_bits'], nb).astype(np.int64)
    for snr in (5, 15):
        k = f'v3c3_snr{snr}'
        r = sim.simulate_simo(bits, snr, num_rx=4, parallel=False)
        ref = int(golden_r3[k + '_errors'][0])
        g = golden_r3[k + '_comb']
        comb = np.asarray(r['symbols_rx_combined'])
        rel = np.linalg.norm(comb[:len(g)] - g) / np.linalg.norm(g)
        assert np.array_equal(_state_head(), golden_r3[k + '_state']), k
        if prec == 'f64':
            assert r['bit_errors'] == ref, (k, r['bit_errors'], ref)
            assert np.array_equal(r['bits_received_array'], unpack(golden_r3[k + '_rx'], nb)), k
            assert rel < 1e-12, (k, rel)
        else:
            assert abs(r['bit_errors'] - ref) / nb < 1e-3, (k, r['bit_errors'], ref)
            assert rel < 1e-5, (k, rel)


@pytest.mark.parametrize('prec', ['f64', 'f32'])
def test_run_grid_3kmh_sharding_invariant(C, prec):
    """Philox grid of the coded chain at 3 km/h: sharded counts sum to the
    unsharded ones, and BER falls with SNR."""
    sim = _sim(20.0, '64-QAM', prec)
    a = sim.run_grid([10.0, 24.0], 24, seed=7, coded=True)
    b0 = sim.run_grid([10.0, 24.0], 24, seed=7, coded=True, rank=0, world_size=2)
    b1 = sim.run_grid([10.0, 24.0], 24, seed=7, coded=True, rank=1, world_size=2)
    assert np.array_equal(a['counts'], b0['counts'] + b1['counts'])
    assert a['ber'][1] <= a['ber'][0]


# Faster UEs than the 3 km/h goldens cover: the channel stages against the
# oracle's per-sample Jakes sum (oracle/lte_oracle.py multipath / jakes,
# core/rayleighchannel.py:20-58) on the same global-RNG draws.  20 MHz,
# fs = 30.72 MHz, 2 GHz: 30 km/h (fD 55.6 Hz), 120 km/h (222 Hz) and 500 km/h
# (926 Hz).  SISO: the Taylor sub-intervals shrink to 64 samples by 120 km/h
# and give way to the per-sample sum past ~227 km/h (k_channel); the 4x4
# spatial links take the per-symbol Taylor sets up to ~6.5 km/h, the
# per-sample exact sum beyond (k_channel_mimo<.., EX>); float32's per-symbol
# quadratic holds to ~20 km/h ((|W| S / 2)^3 / 6 under its half ulp), the
# per-sample sum (float64 arithmetic, rounded) beyond.
@pytest.mark.parametrize('prec,tol', [('f64', 1e-12), ('f32', 1e-5)])
@pytest.mark.parametrize('kmh', [30.0, 120.0, 500.0])
def test_ofdm_channel_transmit_moving_vs_oracle(C, oracle, kmh, prec, tol):
    import lte_phy
    num = oracle.Numerology(bandwidth=20.0, modulation='64-QAM')
    rs = np.random.RandomState(5)
    x = (rs.randn(30000) + 1j * rs.randn(30000)) / np.sqrt(2)
    ch = lte_phy.OFDMChannel('rayleigh_mp', 15.0, num.fs, itu_profile='Pedestrian_A', frequency_ghz=2.0,
                             velocity_kmh=kmh, precision=prec)
    np.random.seed(1234)
    y = ch.transmit(x)
    st = _state_head()
    np.random.seed(1234)
    assert ch.fD == oracle.doppler_hz(2.0, kmh)
    ref = oracle.channel_transmit(num, x, 'rayleigh_mp', 15.0, 'Pedestrian_A', fD=ch.fD)
    assert np.array_equal(st, _state_head())
    assert np.linalg.norm(y - ref) / np.linalg.norm(ref) < tol


# (3 and 6 km/h: the per-symbol sets evaluated at degree 4 after Chebyshev
# economisation, k_channel_tay EC -- inside its 1e-17 bound for this stage's
# 1024-sample symbols up to ~6.5 km/h)
@pytest.mark.parametrize('prec,tol,kmh', [('f64', 1e-12, 3.0), ('f64', 1e-12, 6.0), ('f64', 1e-12, 30.0),
                                          ('f64', 1e-12, 120.0), ('f64', 1e-12, 500.0),
                                          ('f32', 1e-5, 30.0), ('f32', 1e-5, 120.0), ('f32', 1e-5, 500.0)])
def test_spatial_multiplexing_channel_moving_vs_oracle(C, mimo_oracle, oracle, kmh, prec, tol):
    import lte_phy
    num = oracle.Numerology(bandwidth=20.0, modulation='64-QAM')
    rs = np.random.RandomState(6)
    xs = [(rs.randn(8 * 2192) + 1j * rs.randn(8 * 2192)) / np.sqrt(2) for _ in range(4)]
    cs = lte_phy.ChannelSimulator(channel_type='rayleigh_mp', snr_db=18.0, fs=num.fs, itu_profile='Pedestrian_A',
                                  frequency_ghz=2.0, velocity_kmh=kmh, verbose=False, precision=prec)
    np.random.seed(4321)
    ys, Hm = cs.transmit_spatial_multiplexing(list(xs), num_rx=4)
    st = _state_head()
    np.random.seed(4321)
    ref, Href = mimo_oracle.transmit_sm(num, xs, 4, 'rayleigh_mp', 18.0, 'Pedestrian_A',
                                        fD=oracle.doppler_hz(2.0, kmh))
    assert np.array_equal(st, _state_head())
    for r in range(4):
        assert np.linalg.norm(ys[r] - ref[r]) / np.linalg.norm(ref[r]) < tol, r
    assert np.allclose(Hm, Href, rtol=1e-9 if prec == 'f64' else 1e-5, atol=1e-12 if prec == 'f64' else 1e-6)


def test_channel_economised_sets_match_degree5(C, monkeypatch):
    """k_channel_tay's degree-4 economised sets (LTE_CHT_ECON, on by default
    where the bound holds) against the degree-5 sets: the 4x4 PedA links at
    3 km/h, the same draws, streams equal to 1e-14."""
    import lte_phy
    rs = np.random.RandomState(7)
    xs = [(rs.randn(8 * 2192) + 1j * rs.randn(8 * 2192)) / np.sqrt(2) for _ in range(4)]
    out = []
    for econ in ('1', '0'):
        monkeypatch.setenv('LTE_CHT_ECON', econ)
        cs = lte_phy.ChannelSimulator(channel_type='rayleigh_mp', snr_db=18.0, fs=30.72e6,
                                      itu_profile='Pedestrian_A', frequency_ghz=2.0, velocity_kmh=3.0,
                                      verbose=False, precision='f64')
        np.random.seed(99)
        ys, _ = cs.transmit_spatial_multiplexing(list(xs), num_rx=4)
        out.append(ys)
    for a, b in zip(*out):
        assert np.linalg.norm(a - b) / np.linalg.norm(b) < 1e-14
