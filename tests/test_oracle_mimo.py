"""CPU: the multi-antenna oracle (oracle/mimo_oracle.py) against vectors from
running the reference (tests/golden/make_golden_mimo.py): SFBC Alamouti (a33),
MIMO CRS estimation (a34), transmit_mimo (a12), spatial-multiplexing channel
(a13), layer mapping (a35), MMSE (a36) and the config-4 / config-5 drivers
(a37, simulate_mimo / simulate_miso with the documented Q19 estimator fix).
Exact equality unless stated."""
import numpy as np
import pytest

from conftest import unpack


def _num(O, bw, mod):
    return O.Numerology(bandwidth=bw, modulation=mod)


def test_sfbc_kat_and_encode(golden_mimo, mimo_oracle):
    t0, t1 = mimo_oracle.sfbc_encode(np.array([1.0 + 1.0j, -1.0 + 1.0j]))
    assert np.array_equal(t0, golden_mimo['sfbc_kat_tx0']) and np.array_equal(t1, golden_mimo['sfbc_kat_tx1'])
    rx = np.array([t0[0] + 1j * t1[0], t0[1] + 1j * t1[1]])
    dec = mimo_oracle.sfbc_decode(rx, np.array([1, 1], dtype=complex), np.array([1j, 1j]))
    assert np.array_equal(dec, golden_mimo['sfbc_kat_dec'])
    assert np.max(np.abs(dec - [1 + 1j, -1 + 1j])) < 1e-10          # the reference test's own bar
    t0, t1 = mimo_oracle.sfbc_encode(golden_mimo['sfbc_sym'])
    assert np.array_equal(t0, golden_mimo['sfbc_tx0']) and np.array_equal(t1, golden_mimo['sfbc_tx1'])
    with pytest.raises(ValueError):
        mimo_oracle.sfbc_encode(np.ones(3))


@pytest.mark.parametrize('i', [0, 1])
def test_sfbc_decode(golden_mimo, mimo_oracle, i):
    g = golden_mimo
    out = mimo_oracle.sfbc_decode(g[f'sfbc_dec{i}_rx'], g[f'sfbc_dec{i}_H0'], g[f'sfbc_dec{i}_H1'])
    assert np.array_equal(out, g[f'sfbc_dec{i}_out'])


def test_sfbc_grid_mapping(golden_mimo, oracle, mimo_oracle):
    num = _num(oracle, 20.0, '64-QAM')
    assert np.array_equal(mimo_oracle.sfbc_data_idx(num), golden_mimo['sfbcmap_data_idx'])
    np.random.seed(99)
    g0, g1 = mimo_oracle.sfbc_map_grid(num, golden_mimo['sfbc_tx0'], golden_mimo['sfbc_tx1'])
    assert np.array_equal(g0, golden_mimo['sfbcmap_grid0']) and np.array_equal(g1, golden_mimo['sfbcmap_grid1'])
    assert np.array_equal(np.array(np.random.get_state()[1][:8], dtype=np.uint32), golden_mimo['sfbcmap_state'])


@pytest.mark.parametrize('ntx,nrx', [(2, 1), (2, 2), (4, 4)])
def test_mimo_estimate(golden_mimo, oracle, mimo_oracle, ntx, nrx):
    num = _num(oracle, 20.0, '64-QAM')
    k = f'mce_{ntx}x{nrx}'
    pidx = mimo_oracle.mimo_pilot_indices(num, ntx)
    for t in range(ntx):
        assert np.array_equal(pidx[t], golden_mimo[f'{k}_pilots_tx{t}'])
    H = mimo_oracle.mimo_estimate(num, golden_mimo[f'{k}_grid'], ntx)
    assert np.array_equal(H, golden_mimo[f'{k}_H'])


@pytest.mark.parametrize('chan', ['awgn', 'rayleigh_mp'])
def test_transmit_mimo(golden_mimo, oracle, mimo_oracle, chan):
    num = _num(oracle, 20.0, '64-QAM')
    np.random.seed(123)
    ys, H = mimo_oracle.transmit_mimo(num, [golden_mimo['txmimo_x0'], golden_mimo['txmimo_x1']], 2, chan, 12.0)
    assert np.array_equal(np.array(ys), golden_mimo[f'txmimo_{chan}_y'])
    assert np.array_equal(H, golden_mimo[f'txmimo_{chan}_H'])
    assert np.array_equal(np.array(np.random.get_state()[1][:8], dtype=np.uint32), golden_mimo[f'txmimo_{chan}_state'])


@pytest.mark.parametrize('chan', ['awgn', 'rayleigh_mp'])
def test_transmit_spatial(golden_mimo, oracle, mimo_oracle, chan):
    num = _num(oracle, 20.0, '64-QAM')
    np.random.seed(321)
    ys, H = mimo_oracle.transmit_sm(num, list(golden_mimo['txsm_x']), 4, chan, 18.0)
    assert np.array_equal(np.array(ys), golden_mimo[f'txsm_{chan}_y'])
    assert np.array_equal(H, golden_mimo[f'txsm_{chan}_H'])
    assert np.array_equal(np.array(np.random.get_state()[1][:8], dtype=np.uint32), golden_mimo[f'txsm_{chan}_state'])


def test_layer_mapping(golden_mimo, mimo_oracle):
    lay = mimo_oracle.layer_map(golden_mimo['layer_in'], 4)
    assert np.array_equal(lay, golden_mimo['layer_map'])
    assert np.array_equal(mimo_oracle.layer_demap(lay, 999), golden_mimo['layer_demap'])


@pytest.mark.parametrize('i', [0, 1])
def test_mmse(golden_mimo, mimo_oracle, i):
    g = golden_mimo
    out = mimo_oracle.mmse_detect(g[f'mmse{i}_y'], g[f'mmse{i}_H'], float(g[f'mmse{i}_s2'][0]), np.eye(4, dtype=complex))
    assert np.array_equal(out, g[f'mmse{i}_out'])


@pytest.mark.parametrize('name,bw,mod,chan,snrs,nrx', [
    ('sfbc_c1', 1.25, 'QPSK', 'awgn', [4], 2),
    ('sfbc_c1miso', 1.25, 'QPSK', 'rayleigh_mp', [10], 1),
    ('sfbc_c4', 20.0, '64-QAM', 'rayleigh_mp', [10, 20, 30], 2)])
def test_simulate_sfbc(golden_mimo, oracle, mimo_oracle, name, bw, mod, chan, snrs, nrx):
    num = _num(oracle, bw, mod)
    nb = int(golden_mimo[name + '_nbits'][0])
    bits = unpack(golden_mimo[name + '_bits'], nb).astype(np.int64)
    for snr in snrs:
        k = f'{name}_snr{snr}'
        r = mimo_oracle.simulate_sfbc(num, bits, snr, num_rx=nrx, channel=chan)
        assert r['bit_errors'] == int(golden_mimo[k + '_errors'][0]), k
        assert np.array_equal(r['bits_received_array'], unpack(golden_mimo[k + '_rx'], nb)), k
        assert np.array_equal(r['channel_matrix'], golden_mimo[k + '_H'])
        assert np.allclose([r['papr_db_tx0'], r['papr_db_tx1'], r['papr_db']], golden_mimo[k + '_papr'], rtol=0, atol=1e-12)
        assert np.array_equal(np.array(np.random.get_state()[1][:8], dtype=np.uint32), golden_mimo[k + '_state'])


@pytest.mark.parametrize('name,bw,mod,chan,snrs', [
    ('sm_c1', 1.25, 'QPSK', 'awgn', [15]),
    ('sm_c5awgn', 20.0, '64-QAM', 'awgn', [25]),
    ('sm_c5ray', 20.0, '64-QAM', 'rayleigh_mp', [25, 35])])
def test_simulate_spatial(golden_mimo, oracle, mimo_oracle, name, bw, mod, chan, snrs):
    num = _num(oracle, bw, mod)
    nb = int(golden_mimo[name + '_nbits'][0])
    bits = unpack(golden_mimo[name + '_bits'], nb).astype(np.int64)
    for snr in snrs:
        k = f'{name}_snr{snr}'
        r = mimo_oracle.simulate_spatial(num, bits, snr, channel=chan)
        assert r['bit_errors'] == int(golden_mimo[k + '_errors'][0]), k
        assert np.array_equal(r['bits_received_array'], unpack(golden_mimo[k + '_rx'], nb)), k
        assert np.array_equal(r['channel_matrix'], golden_mimo[k + '_H'])
        assert np.array_equal(r['precoder_matrix'], golden_mimo[k + '_W'])
        assert np.array_equal(np.array(np.random.get_state()[1][:8], dtype=np.uint32), golden_mimo[k + '_state'])


def test_sfbc_coded_fixture_frames(oracle, mimo_oracle, fixture_curve_c4):
    """The config-4 composition (simulate_sfbc_coded) regenerates the committed
    fixture's verdicts for one frame past the cliff and one clean frame (the
    fixture's draws are RandomState-seeded, tests/golden/make_fixture_ber_curve.py)."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        'mkfx', os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'make_fixture_ber_curve.py'))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    for s, f in [(8, 3), (12, 0)]:
        _, _, err, crc = mk.one_c4((s, f))
        assert err == int(fixture_curve_c4['bit_errors'][s, f]) and crc == int(fixture_curve_c4['crc_ok'][s, f])


def test_transmit_mimo_combined_link_noise(golden_mimo, oracle, mimo_oracle):
    """The device's Philox mode for transmit_mimo (draws[r]['combined_link_noise']):
    the RX stream takes the faded links' sum plus ONE draw of standard deviation
    sqrt(sum_t s_rt^2) on link (r, 0)'s numbers, while the reported channel
    matrix keeps each link's own draw -- against the per-link form on the same
    draws: Hm identical, the noise-free parts equal, and the difference of the
    streams exactly the two noise terms (before the RX noise, which the
    measured power then scales)."""
    num = _num(oracle, 20.0, '64-QAM')
    xs = [golden_mimo['txmimo_x0'], golden_mimo['txmimo_x1']]
    L = len(xs[0])
    np.random.seed(5)
    draws = mimo_oracle.transmit_mimo_draws(2, 2, 'rayleigh_mp', L)
    comb = [dict(d, combined_link_noise=True) for d in draws]
    # RX noise off (huge SNR) so the streams show the link noise alone
    ys_a, H_a = mimo_oracle.transmit_mimo(num, xs, 2, 'rayleigh_mp', 400.0, draws=draws)
    ys_b, H_b = mimo_oracle.transmit_mimo(num, xs, 2, 'rayleigh_mp', 400.0, draws=comb)
    assert np.array_equal(H_a, H_b)
    dl, g = mimo_oracle.itu_paths(num, 'Pedestrian_A')
    for r in range(2):
        s2, y0 = 0.0, np.zeros(L, dtype=complex)
        per_link = np.zeros(L, dtype=complex)
        for t in range(2):
            d = draws[r]['links'][t]
            y = mimo_oracle.multipath(xs[t], dl, g, d['phases'], 0.0, num.fs)
            s = np.sqrt((np.mean(np.abs(y) ** 2) / 1e10) / 2)
            s2 = s2 + s * s
            y0 += y
            per_link += s * d['z_re'] + 1j * (s * d['z_im'])
        z0 = draws[r]['links'][0]
        sr = np.sqrt(s2)
        comb_noise = sr * z0['z_re'] + 1j * (sr * z0['z_im'])
        assert np.allclose(ys_a[r], y0 + per_link, rtol=0, atol=1e-12)
        assert np.allclose(ys_b[r], y0 + comb_noise, rtol=0, atol=1e-12)
        # same distribution: both noise terms carry the summed variance
        assert abs(np.var(comb_noise) / np.var(per_link) - 1) < 0.05


def test_transmit_mimo_merged_link_noise(golden_mimo, oracle, mimo_oracle):
    """The device's merged mode (draws[r]['merged_link_noise'], config 4's full
    chain): no link-noise draw; the RX stream is the faded links' sum plus ONE
    draw of standard deviation sqrt((2 s2 + npow) / 2) on the RX noise numbers,
    s2 = ((sum_t mean |y0_t|^2) / 1e10) / 2, npow = ((mean |y0|^2 + 2 s2) /
    num_tx) / SNR -- the link noise's power in expectation (k_npow_sfbc_merged's
    expression and order)."""
    num = _num(oracle, 20.0, '64-QAM')
    xs = [golden_mimo['txmimo_x0'], golden_mimo['txmimo_x1']]
    L = len(xs[0])
    np.random.seed(6)
    draws = mimo_oracle.transmit_mimo_draws(2, 2, 'rayleigh_mp', L)
    merged = [dict(d, combined_link_noise=True, merged_link_noise=True) for d in draws]
    snr = 13.0
    ys, H = mimo_oracle.transmit_mimo(num, xs, 2, 'rayleigh_mp', snr, draws=merged)
    ys_c, H_c = mimo_oracle.transmit_mimo(num, xs, 2, 'rayleigh_mp', snr,
                                          draws=[dict(d, combined_link_noise=True) for d in draws])
    assert np.array_equal(H, H_c)   # each link's own draw still forms its Hm entry
    dl, g = mimo_oracle.itu_paths(num, 'Pedestrian_A')
    for r in range(2):
        pl, y0 = 0.0, np.zeros(L, dtype=complex)
        for t in range(2):
            y = mimo_oracle.multipath(xs[t], dl, g, draws[r]['links'][t]['phases'], 0.0, num.fs)
            pl = pl + np.mean(np.abs(y) ** 2)
            y0 += y
        s2 = (pl / 1e10) / 2
        npow = 2.0 * s2 + ((np.mean(np.abs(y0) ** 2) + 2.0 * s2) / 2) / 10 ** (snr / 10)
        st = np.sqrt(npow / 2)
        assert np.array_equal(ys[r], y0 + (st * draws[r]['z_re'] + 1j * (st * draws[r]['z_im'])))
        # the same noise power as the separate draws up to the link noise's cross terms
        ref = ys_c[r] - y0
        assert abs(np.mean(np.abs(ys[r] - y0) ** 2) / np.mean(np.abs(ref) ** 2) - 1) < 0.05
