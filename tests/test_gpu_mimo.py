"""GPU parity of the multi-antenna chains (SURVEY §8 a12, a13, a33-a37;
configs 4 and 5) against the reference's own outputs (tests/golden/
golden_mimo.npz, frozen global RNG) and the oracle (oracle/mimo_oracle.py).

Bars, float64 (the default, the reference's complex128): identical bit
errors and received bits, identical global-RNG side effects, channel matrices
to 1e-12 relative, received streams to 1e-12 relative; coded SFBC: in-chain
LLRs vs the oracle's max-log demapper to 1e-12 and decoding bit-exact vs the
float64 reference decoder.  float32 fast mode: |dBER| < 1e-3 absolute (the
north_star tolerance), matrices / streams to float32 precision, decoding
bit-exact vs the decoder's float32 model."""
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


def _sim(bw, mod, chan, precision='f64'):
    import lte_phy
    return lte_phy.OFDMSimulator(lte_phy.LTEConfig(bandwidth=bw, modulation=mod), channel_type=chan,
                                 precision=precision)


SFBC_CASES = [('sfbc_c1', 1.25, 'QPSK', 'awgn', [4], 2),
              ('sfbc_c1miso', 1.25, 'QPSK', 'rayleigh_mp', [10], 1),
              ('sfbc_c4', 20.0, '64-QAM', 'rayleigh_mp', [10, 20, 30], 2)]


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('name,bw,mod,chan,snrs,nrx', SFBC_CASES)
def test_sfbc_ref_compat(C, golden_mimo, name, bw, mod, chan, snrs, nrx, prec):
    """simulate_miso / simulate_mimo (with the Q19 estimator fix) == the fixed
    reference: bit errors, received bits, global RNG state, channel matrix,
    per-TX PAPR.  f64: identical decisions; f32: within the north_star 1e-3."""
    sim = _sim(bw, mod, chan, prec)
    nb = int(golden_mimo[name + '_nbits'][0])
    bits = unpack(golden_mimo[name + '_bits'], nb).astype(np.int64)
    for snr in snrs:
        k = f'{name}_snr{snr}'
        r = sim.simulate_miso(bits, snr) if nrx == 1 else sim.simulate_mimo(bits, snr, num_rx=nrx)
        ref_err = int(golden_mimo[k + '_errors'][0])
        ref_rx = unpack(golden_mimo[k + '_rx'], nb)
        H = golden_mimo[k + '_H']
        p = golden_mimo[k + '_papr']
        assert np.array_equal(_state(), golden_mimo[k + '_state'])
        if prec == 'f64':
            assert r['bit_errors'] == ref_err, (k, r['bit_errors'], ref_err)
            assert np.array_equal(r['bits_received_array'], ref_rx), k
            assert np.max(np.abs(r['channel_matrix'] - H)) < 1e-12 * (1 + np.max(np.abs(H))), k
            assert np.allclose([r['papr_db_tx0'], r['papr_db_tx1'], r['papr_db']], p, rtol=0, atol=1e-9), k
        else:
            assert abs(r['bit_errors'] - ref_err) / nb < 1e-3, (k, r['bit_errors'], ref_err)
            assert np.mean(r['bits_received_array'] != ref_rx) < 1e-3
            assert np.max(np.abs(r['channel_matrix'] - H)) < 1e-4 * (1 + np.max(np.abs(H))), k
            assert np.allclose([r['papr_db_tx0'], r['papr_db_tx1'], r['papr_db']], p, atol=1e-3), k


SM_CASES = [('sm_c1', 1.25, 'QPSK', 'awgn', [15]),
            ('sm_c5awgn', 20.0, '64-QAM', 'awgn', [25]),
            ('sm_c5ray', 20.0, '64-QAM', 'rayleigh_mp', [25, 35])]


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('name,bw,mod,chan,snrs', SM_CASES)
def test_spatial_ref_compat(C, golden_mimo, name, bw, mod, chan, snrs, prec):
    """simulate_spatial_multiplexing 4x4 rank 4 MMSE == the reference (f64:
    identical bit errors and received bits; f32: within 1e-3)."""
    import lte_phy
    nb = int(golden_mimo[name + '_nbits'][0])
    bits = unpack(golden_mimo[name + '_bits'], nb).astype(np.int64)
    for snr in snrs:
        k = f'{name}_snr{snr}'
        c = lte_phy.LTEConfig(bandwidth=bw, modulation=mod)
        r = lte_phy.simulate_spatial_multiplexing(bits, num_tx=4, num_rx=4, rank=4, detector_type='MMSE',
                                                  modulation=mod, snr_db=snr, config=c, channel_type=chan,
                                                  itu_profile='Pedestrian_A', velocity_kmh=3,
                                                  enable_csi_feedback=False, precision=prec)
        ref_err = int(golden_mimo[k + '_errors'][0])
        ref_rx = unpack(golden_mimo[k + '_rx'], nb)
        if prec == 'f64':
            assert r['bit_errors'] == ref_err, (k, r['bit_errors'], ref_err)
            assert np.array_equal(r['bits_received_array'], ref_rx), k
        else:
            assert abs(r['bit_errors'] - ref_err) / nb < 1e-3, (k, r['bit_errors'], ref_err)
            assert np.mean(r['bits_received_array'] != ref_rx) < 1e-3
        assert np.array_equal(_state(), golden_mimo[k + '_state'])
        assert np.array_equal(r['channel_matrix'], golden_mimo[k + '_H'])
        assert np.array_equal(r['precoder_matrix'], golden_mimo[k + '_W'])


def test_spatial_vs_oracle_awgn_high_snr(C, oracle, mimo_oracle):
    """Config 5 at 40 dB, flat channel, float64: GPU and oracle decode the same
    bits (identical received bits and bit errors)."""
    import lte_phy
    num = oracle.Numerology(bandwidth=5.0, modulation='16-QAM')
    bits = np.random.RandomState(4).randint(0, 2, 14 * num.Nd * 4)
    np.random.seed(17)
    o = mimo_oracle.simulate_spatial(num, bits, 40.0, channel='awgn')
    np.random.seed(17)
    r = lte_phy.simulate_spatial_multiplexing(bits, num_tx=4, num_rx=4, rank=4, modulation='16-QAM', snr_db=40,
                                              config=lte_phy.LTEConfig(bandwidth=5.0, modulation='16-QAM'),
                                              channel_type='awgn', enable_csi_feedback=False)
    assert r['bit_errors'] == o['bit_errors']
    assert np.array_equal(r['bits_received_array'], o['bits_received_array'])
    assert np.array_equal(r['channel_matrix'], o['channel_matrix'])


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('chan', ['awgn', 'rayleigh_mp'])
def test_sfbc_coded_llrs_and_decoding(C, oracle, chan, prec):
    """Config 4 chain on Philox frames: the LLRs k_det_sfbc writes equal the
    oracle's max-log LLRs of the same combined symbols with the documented
    noise-variance rule (f64 1e-12, f32 1e-4), and the GPU decoder's output
    equals the float64 reference decoder (f64) / the float32 decoder model
    (f32) run on those LLRs (T/F de-interleave with cols = Nd & ~1, rate
    dematch, turbo, CRC)."""
    sim = _sim(20.0, '64-QAM', chan, prec)
    plan = sim._sfbc_plan(0, 27760, 2, coded=True, max_frames=4)
    snrs = np.array([8.0, 14.0, 20.0, 30.0])
    r = plan.run(snrs, seed=9, capture=('llr', 'data_syms', 'H', 'bits_rx'))
    num = oracle.Numerology(bandwidth=20.0, modulation='64-QAM')
    res, bps = plan.res, 6
    d = num.data_idx[:res]
    tb = np.zeros(27760, dtype=np.uint8)
    _, seg_plan = oracle.segment(oracle.attach_crc24a(tb))
    rm = [3 * p[0] + 12 for p in seg_plan]
    coded = plan.coded_bits
    ncs = coded // bps
    rows = -(-ncs // res)
    q = np.arange(ncs)
    src = (q % res) * rows + q // res
    for b, snr in enumerate(snrs):
        z = r['data_syms'][b].astype(np.complex128)
        H = r['H'][b].astype(np.complex128)
        s2 = 1.0 / 10 ** (snr / 10)
        nv = np.zeros(len(z))
        for l in range(plan.n_sym):
            e = l // 14
            inv_g = np.zeros(res // 2)
            for a in range(2):
                h0, h1 = H[a, e, 0], H[a, e, 1]
                a0, a1 = (h0[0::2] + h0[1::2]) / 2, (h1[0::2] + h1[1::2]) / 2
                nrm = (np.hypot(a0.real, a0.imag) ** 2 + np.hypot(a1.real, a1.imag) ** 2) + 1e-10
                inv_g += 1.0 / np.clip(nrm, 1e-6, 1e6)
            v = np.maximum(s2 / 4.0 * inv_g, s2 / 4.0)   # s2 / R^2 * sum 1/norm, R = 2
            nv[l * res:(l + 1) * res] = np.repeat(v, 2)
        ref = oracle.llrs(z, nv, '64-QAM')
        got = r['llr'][b].astype(np.float64)[:len(ref)]
        tol = 1e-12 if prec == 'f64' else 1e-4
        assert np.max(np.abs(got - ref) / (1 + np.abs(ref))) < tol, (chan, snr)
        L = got.reshape(-1, bps)[src].reshape(-1)[:coded]
        dec, ok = oracle.coded_rx_decode(L, seg_plan, rm, 8, f32_model=prec == 'f32')
        assert np.array_equal(dec, r['bits_rx'][b]) and bool(ok) == bool(r['crc_ok'][b]), (chan, snr)
    if chan == 'awgn':
        assert r['crc_ok'][-1] == 1 and r['frame_errors'][-1] == 0


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('mode', ['spatial', 'sfbc'])
def test_flat_channel_fused_tx(C, prec, mode, monkeypatch):
    """Flat (AWGN) links: TX and channel in one pass per (frame, symbol, RX),
    y_r = IFFT(sum_t h_rt G_t) (k_ofdm_txch_flat, default) against the TX
    streams through HBM and the channel pass (LTE_MIMO_FLAT_FUSE=0): received
    streams equal to float64 rounding (the sums are taken in the frequency
    domain), identical per-frame bit errors."""
    from lte_phy.ofdm_core import _spatial_plan
    cfg_sim = _sim(20.0, '64-QAM', 'awgn', prec)
    if mode == 'spatial':
        plan = _spatial_plan(cfg_sim.config, 'awgn', 'Pedestrian_A', 3.0, 2.0, 14, 14 * 999 * 6, 6, precision=prec)[0]
    else:
        plan = cfg_sim._sfbc_plan(14, 14 * 998 * 6, 2, max_frames=6)
    snrs = np.array([5.0, 10.0, 15.0, 20.0, 25.0, 30.0])
    outs = []
    for fuse in ('1', '0'):
        monkeypatch.setenv('LTE_MIMO_FLAT_FUSE', fuse)
        outs.append(plan.run(snrs, seed=33, capture=('signal_rx', 'data_syms')))
    a, b = outs
    y0, y1 = a['signal_rx'].astype(np.complex128), b['signal_rx'].astype(np.complex128)
    assert np.linalg.norm(y0 - y1) / np.linalg.norm(y1) < (1e-14 if prec == 'f64' else 2e-6)
    z0, z1 = a['data_syms'].astype(np.complex128), b['data_syms'].astype(np.complex128)
    assert np.linalg.norm(z0 - z1) / np.linalg.norm(z1) < (1e-13 if prec == 'f64' else 1e-5)
    assert np.array_equal(a['frame_errors'], b['frame_errors'])


@pytest.mark.parametrize('prec', ['f64', 'f32'])
def test_link_power_in_tx_matches_separate_pass(C, prec, monkeypatch):
    """Config 4 (SFBC 2x2, Rayleigh links, transmit_mimo's 100 dB link noise):
    the link powers formed on the TX symbols in LDS (k_ofdm_tx_mimo +
    k_link_power_fix, default) against the separate k_link_power pass over x
    (LTE_MIMO_LP_FUSE=0): received streams equal to 1e-15 relative (the power
    sums differ only in their order, which moves the 1e-5 link noise by ulps),
    identical per-frame errors and CRC."""
    sim = _sim(20.0, '64-QAM', 'rayleigh_mp', prec)
    plan = sim._sfbc_plan(0, 27760, 2, coded=True, max_frames=6)
    snrs = np.array([6.0, 12.0, 16.0, 18.0, 22.0, 30.0])
    outs = []
    monkeypatch.setenv('LTE_SFBC_TXCH_FUSE', '0')   # the separate TX / channel kernels this test compares
    for fuse in ('1', '0'):
        monkeypatch.setenv('LTE_MIMO_LP_FUSE', fuse)
        outs.append(plan.run(snrs, seed=21, capture=('signal_rx',)))
    a, b = outs
    y0, y1 = a['signal_rx'].astype(np.complex128), b['signal_rx'].astype(np.complex128)
    assert np.linalg.norm(y0 - y1) / np.linalg.norm(y1) < (1e-15 if prec == 'f64' else 1e-6)
    assert np.array_equal(a['frame_errors'], b['frame_errors']) and np.array_equal(a['crc_ok'], b['crc_ok'])


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('coded,nrx', [(True, 2), (False, 2), (False, 1)])
def test_sfbc_txch_fused_matches_separate_kernels(C, prec, coded, nrx, monkeypatch):
    """Config 4's TX + static-tap Rayleigh links in one pass per frame
    (k_ofdm_txch_sfbc + k_link_noise_pairs, default on the Philox path) against
    the TX streams through HBM and the channel pass (LTE_SFBC_TXCH_FUSE=0):
    received streams (signal_rx: the faded links, the combined 100 dB link
    noise, the RX noise) equal to float64 rounding -- the link paths are summed
    per link here and straight into the RX sum there, and the power sums in
    another order move the 1e-5 link noise by ulps -- and identical per-frame
    errors and CRC verdicts, over the delayed samples that cross every symbol
    boundary (the kept tails), 1 and 2 RX, coded and uncoded (float32: the
    north_star 1e-3 on the blocks past the cliff, identical CRC verdicts)."""
    sim = _sim(20.0, '64-QAM', 'rayleigh_mp', prec)
    plan = (sim._sfbc_plan(0, 27760, nrx, coded=True, max_frames=6) if coded else
            sim._sfbc_plan(14, 14 * 998 * 6, nrx, max_frames=6))
    snrs = np.array([6.0, 12.0, 16.0, 18.0, 22.0, 30.0])
    outs = []
    for fuse in ('1', '0'):
        monkeypatch.setenv('LTE_SFBC_TXCH_FUSE', fuse)
        outs.append(plan.run(snrs, seed=27, frame_id0=1000, capture=('signal_rx',)))
    a, b = outs
    y0, y1 = a['signal_rx'].astype(np.complex128), b['signal_rx'].astype(np.complex128)
    assert y0.shape == (6, nrx, plan.L)
    assert np.linalg.norm(y0 - y1) / np.linalg.norm(y1) < (1e-14 if prec == 'f64' else 1e-6)
    # the first samples of every symbol after the first (their taps reach into the previous symbol)
    S = 2192
    for l in range(1, 14):
        seg0, seg1 = y0[..., l * S:l * S + 16], y1[..., l * S:l * S + 16]
        assert np.max(np.abs(seg0 - seg1)) <= (1e-13 if prec == 'f64' else 1e-5) * np.max(np.abs(seg1))
    if coded:
        assert np.array_equal(a['crc_ok'], b['crc_ok'])
    if prec == 'f64':
        assert np.array_equal(a['frame_errors'], b['frame_errors'])
    else:   # float32: rounding-level LLR changes move a few decisions of the blocks that fail anyway
        nb = 27760 if coded else 14 * 998 * 6
        assert np.max(np.abs(a['frame_errors'].astype(np.int64) - b['frame_errors'])) / nb < 1e-3
        assert np.array_equal(a['frame_errors'] == 0, b['frame_errors'] == 0)


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('coded,nrx,chan', [(True, 2, 'rayleigh_mp'), (False, 2, 'rayleigh_mp'),
                                            (False, 1, 'rayleigh_mp'), (True, 2, 'awgn'), (False, 2, 'awgn')])
def test_sfbc_rx_fused_matches_separate_kernels(C, prec, coded, nrx, chan, monkeypatch):
    """Config 4's receiver and SFBC detector in one pass per frame (k_rx_sfbc,
    default when nothing captures Y / H / the symbols) against k_rx_fft_mimo +
    k_det_sfbc through HBM (LTE_SFBC_RX_FUSE=0): the same operations per
    subcarrier pair (mimo_interp, sfbc_combine, the RX sum in RX order), so
    identical per-frame bit errors and CRC verdicts, coded (the demapper's
    inputs) and uncoded, 1 and 2 RX, Rayleigh and flat links (float32: the
    north_star 1e-3 and identical CRC verdicts)."""
    sim = _sim(20.0, '64-QAM', chan, prec)
    plan = (sim._sfbc_plan(0, 27760, nrx, coded=True, max_frames=7) if coded else
            sim._sfbc_plan(14, 14 * 998 * 6, nrx, max_frames=7))
    snrs = np.array([6.0, 10.0, 14.0, 16.0, 18.0, 22.0, 30.0])
    outs = []
    cap = ('bits_rx',) if coded else ()   # coded: the decoder's bits (k_crc_count), fused path kept
    monkeypatch.setenv('LTE_SFBC_LINK_MERGE', '0')   # the same link-noise draws on both sides
    for fuse in ('1', '0'):
        monkeypatch.setenv('LTE_SFBC_RX_FUSE', fuse)
        outs.append(plan.run(snrs, seed=31, frame_id0=4242, capture=cap))
    a, b = outs
    if coded:
        assert np.array_equal(a['crc_ok'], b['crc_ok'])
        if prec == 'f64':
            assert np.array_equal(a['bits_rx'], b['bits_rx'])
    assert 0 < int(a['counts'][:, 0].sum())
    if prec == 'f64':
        assert np.array_equal(a['frame_errors'], b['frame_errors'])
        assert np.array_equal(a['counts'], b['counts'])
    else:   # float32: the compiler contracts other products into FMAs in the fused kernel
        nb = 27760 if coded else 14 * 998 * 6
        assert np.max(np.abs(a['frame_errors'].astype(np.int64) - b['frame_errors'])) / nb < 1e-3
        assert np.array_equal(a['frame_errors'] == 0, b['frame_errors'] == 0)


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('chan,det', [('rayleigh_mp', 'DET_MMSE'), ('awgn', 'DET_MMSE'), ('rayleigh_mp', 'DET_ZF'),
                                      ('rayleigh_mp', 'DET_SIC')])
def test_spatial_pilot_handoff_matches_interpolated_h(C, prec, chan, det, monkeypatch):
    """Config 5's receiver hands the detector each symbol's LS pilot estimates
    and k_det_spatial interpolates them per RE (default without an H capture)
    against the interpolated H through HBM (LTE_SPATIAL_HP=0): the same
    mimo_interp per (RX, TX, RE), so identical per-frame bit errors in float64
    (float32: the north_star 1e-3)."""
    from lte_phy.ofdm_core import _spatial_plan
    sim = _sim(20.0, '64-QAM', chan, prec)
    nb = 14 * 999 * 6
    plan = _spatial_plan(sim.config, chan, 'Pedestrian_A', 3.0, 2.0, 14, nb, 7, detector=getattr(C, det),
                         precision=prec)[0]
    snrs = np.array([6.0, 10.0, 14.0, 18.0, 22.0, 26.0, 30.0])
    outs = []
    monkeypatch.setenv('LTE_MIMO_RX_WAVE', '0')   # the block receiver on both sides: only the handoff changes
    for hp in ('1', '0'):
        monkeypatch.setenv('LTE_SPATIAL_HP', hp)
        outs.append(plan.run(snrs, seed=17, frame_id0=777))
    a, b = outs
    assert 0 < int(a['counts'][:, 0].sum())
    if prec == 'f64':
        assert np.array_equal(a['frame_errors'], b['frame_errors'])
        assert np.array_equal(a['counts'], b['counts'])
    else:
        assert np.max(np.abs(a['frame_errors'].astype(np.int64) - b['frame_errors'])) / nb < 1e-3


@pytest.mark.parametrize('chan,det,inject', [('rayleigh_mp', 'DET_MMSE', False), ('awgn', 'DET_SIC', False),
                                             ('rayleigh_mp', 'DET_MMSE', True)])
def test_wave_mimo_receiver_matches_block_receiver(C, chan, det, inject, monkeypatch):
    """Config 5's receiver as one wave per (frame, RX antenna)
    (k_rx_fft_mimo_w: wave_symbol_noisy + wfft's 2048-point FFT, the pilot
    estimates through the wave's LDS half a symbol at a time) vs the block
    kernel k_rx_fft_mimo<.., HPO> on the same frames (Philox or injected
    noise): the two FFTs differ in round-off only (each within a few 1e-14 of
    the exact DFT), so per-frame bit errors and counts are identical.  7
    frames x 4 RX = 28 waves: a partial last block."""
    from lte_phy.ofdm_core import _spatial_plan
    sim = _sim(20.0, '64-QAM', chan, 'f64')
    nb = 14 * 999 * 6
    plan = _spatial_plan(sim.config, chan, 'Pedestrian_A', 3.0, 2.0, 14, nb, 7, detector=getattr(C, det),
                         precision='f64')[0]
    snrs = np.array([6.0, 10.0, 14.0, 18.0, 22.0, 26.0, 30.0])
    kw = {}
    if inject:
        kw = dict(noise=np.random.default_rng(3).standard_normal((7, 4, 2, plan.L)))
    outs = []
    for wave in ('1', '0'):
        monkeypatch.setenv('LTE_MIMO_RX_WAVE', wave)
        outs.append(plan.run(snrs, seed=17, frame_id0=777, **kw))
    a, b = outs
    assert 0 < int(a['counts'][:, 0].sum())
    assert np.array_equal(a['frame_errors'], b['frame_errors'])
    assert np.array_equal(a['counts'], b['counts'])


@pytest.mark.parametrize('det,inject,rank', [('DET_MMSE', False, 4), ('DET_SIC', True, 4), ('DET_ZF', False, 2)])
def test_wave_mimo_tx_matches_block_tx(C, det, inject, rank, monkeypatch):
    """Config 5's TX + flat links as one wave per (frame, RX antenna)
    (k_ofdm_txch_flat_w: the bins of Y_r = sum_t h_rt G_t formed through the
    wave's LDS, wfft's 2048-point inverse FFT, the CP and the power partial by
    one wave reduction) vs the block kernel k_ofdm_txch_flat on the same frames:
    the transforms and power sums differ in round-off only, so per-frame bit
    errors and counts are identical.  7 frames x 4 RX = 28 waves: a partial
    last block; rank 2 too."""
    from lte_phy.ofdm_core import _spatial_plan
    sim = _sim(20.0, '64-QAM', 'awgn', 'f64')
    nb = 14 * 999 * 6
    plan = _spatial_plan(sim.config, 'awgn', 'Pedestrian_A', 3.0, 2.0, 14, nb, 7, detector=getattr(C, det),
                         precision='f64', rank=rank)[0]
    snrs = np.array([6.0, 10.0, 14.0, 18.0, 22.0, 26.0, 30.0])
    kw = {}
    if inject:
        kw = dict(noise=np.random.default_rng(4).standard_normal((7, 4, 2, plan.L)))
    outs = []
    for wave in ('1', '0'):
        monkeypatch.setenv('LTE_MIMO_TX_WAVE', wave)
        outs.append(plan.run(snrs, seed=19, frame_id0=555, **kw))
    a, b = outs
    assert 0 < int(a['counts'][:, 0].sum())
    assert np.array_equal(a['frame_errors'], b['frame_errors'])
    assert np.array_equal(a['counts'], b['counts'])


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('mimo,coded,chan', [('sfbc', True, 'rayleigh_mp'), ('spatial', False, 'rayleigh_mp'),
                                            ('spatial', False, 'awgn')])
def test_run_grid_mimo_sharding_invariant(C, mimo, coded, chan, prec):
    sim = _sim(20.0, '64-QAM', chan, prec)
    kw = dict(mimo=mimo, coded=coded, num_rx=2 if mimo == 'sfbc' else 4)
    a = sim.run_grid([10.0, 25.0], 24, seed=5, **kw)
    b0 = sim.run_grid([10.0, 25.0], 24, seed=5, rank=0, world_size=2, **kw)
    b1 = sim.run_grid([10.0, 25.0], 24, seed=5, rank=1, world_size=2, **kw)
    assert np.array_equal(a['counts'], b0['counts'] + b1['counts'])
    assert a['ber'][1] <= a['ber'][0] + 1e-12


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('chan', ['awgn', 'rayleigh_mp'])
def test_transmit_mimo_stage(C, golden_mimo, chan, prec):
    """OFDMChannel.transmit_mimo (a12) == the reference on the same seed:
    received streams (f64 1e-12, f32 1e-5 relative), channel matrix, RNG state."""
    import lte_phy
    x = [golden_mimo['txmimo_x0'], golden_mimo['txmimo_x1']]
    ch = lte_phy.OFDMChannel(channel_type=chan, snr_db=12.0, fs=30.72e6, itu_profile='Pedestrian_A', precision=prec)
    np.random.seed(123)
    ys, Hm = ch.transmit_mimo(x, num_rx=2)
    ref = golden_mimo[f'txmimo_{chan}_y']
    tol = 1e-12 if prec == 'f64' else 1e-5
    assert np.max(np.abs(np.array(ys) - ref)) < tol * (1 + np.max(np.abs(ref)))
    assert np.allclose(Hm, golden_mimo[f'txmimo_{chan}_H'], rtol=tol, atol=tol * 0.1)
    assert np.array_equal(_state(), golden_mimo[f'txmimo_{chan}_state'])


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('chan', ['awgn', 'rayleigh_mp'])
def test_transmit_spatial_multiplexing_stage(C, golden_mimo, chan, prec):
    """ChannelSimulator.transmit_spatial_multiplexing (a13), 4x4, PedA 3 km/h
    (time-varying Jakes: f64 degree-5 Taylor sets per OFDM symbol) == the reference on the
    same seed (streams f64 1e-12, f32 1e-5 relative)."""
    import lte_phy
    cs = lte_phy.ChannelSimulator(channel_type=chan, snr_db=18.0, fs=30.72e6, itu_profile='Pedestrian_A',
                                  frequency_ghz=2.0, velocity_kmh=3, verbose=False, precision=prec)
    np.random.seed(321)
    ys, Hm = cs.transmit_spatial_multiplexing(list(golden_mimo['txsm_x']), num_rx=4)
    ref = golden_mimo[f'txsm_{chan}_y']
    tol = 1e-12 if prec == 'f64' else 1e-5
    assert np.max(np.abs(np.array(ys) - ref)) < tol * (1 + np.max(np.abs(ref)))
    assert np.allclose(Hm, golden_mimo[f'txsm_{chan}_H'], rtol=1e-9, atol=1e-12)
    assert np.array_equal(_state(), golden_mimo[f'txsm_{chan}_state'])


def test_mimo_argument_errors(C):
    import lte_phy
    sim = _sim(1.25, 'QPSK', 'awgn')
    with pytest.raises(ValueError):
        sim.simulate_mimo(np.array([], dtype=int), 10.0)
    with pytest.raises(NotImplementedError):      # 8 TX: outside the GPU path (num_tx 2 / 4)
        lte_phy.simulate_spatial_multiplexing(np.ones(100, dtype=int), num_tx=8, num_rx=2, rank=2,
                                              enable_csi_feedback=False)
    with pytest.raises(ValueError):
        lte_phy.OFDMChannel().transmit_mimo([])
    with pytest.raises(ValueError):
        lte_phy.OFDMChannel().transmit_mimo([np.ones(10), np.ones(11)])


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('mod', ['16-QAM', '64-QAM'])
def test_sfbc_demap_in_dematch_matches_llr_path(C, monkeypatch, mod, prec):
    """Coded SFBC: k_det_sfbc handing the combined symbols and each RE pair's
    sigma^2_eff to k_dematch_zn (which runs the same max-log demapper while it
    builds the decoder rows) decodes exactly like the LLR round trip
    (k_det_sfbc LLRs -> k_dematch): identical per-frame bit errors, CRC flags
    and counts on the same Philox frames, over more than one decoder group
    (both through k_det_sfbc: LTE_SFBC_RX_FUSE=0; the fused receiver has its
    own test)."""
    monkeypatch.setenv('LTE_SFBC_RX_FUSE', '0')
    sim = _sim(20.0, mod, 'rayleigh_mp', prec)
    B = 64 + 7
    plan = sim._sfbc_plan(0, 27760 if mod == '64-QAM' else 18000, 2, coded=True, max_frames=B)
    snr = np.tile(np.arange(0.0, 31.0, 2.0), B)[:B]
    monkeypatch.setenv('LTE_DEMAP_IN_DEMATCH', '0')
    a = plan.run(snr, seed=0x5EED, frame_id0=5)
    monkeypatch.setenv('LTE_DEMAP_IN_DEMATCH', '1')
    b = plan.run(snr, seed=0x5EED, frame_id0=5)
    assert np.array_equal(a['crc_ok'], b['crc_ok']) and np.array_equal(a['counts'], b['counts'])
    assert np.array_equal(a['frame_errors'], b['frame_errors'])
