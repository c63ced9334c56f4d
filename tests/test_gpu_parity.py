"""GPU parity: the HIP path (through the C ABI) against the oracle / golden
vectors.  The chains run in float64 by default (the reference's arithmetic);
float32 is the opt-in fast mode.  Tolerances:
  * FFT: relative L2 error <= 1e-14 (f64) / 2e-6 (f32) vs np.fft
  * integer/bit work (turbo encoder, CRC, packing): bit-exact
  * turbo decoder: f64 bit-exact with the reference; f32 bit-exact with its
    float32 model (oracle turbo_decode_f32_model)
  * end-to-end vs the reference's own outputs on its own random numbers: f64
    bit errors and CRC verdicts equal; f32 |BER_gpu - BER_ref| < 1e-3 (the
    north_star tolerance) where the reference decodes
"""
import numpy as np
import pytest

from conftest import unpack

pytestmark = pytest.mark.gpu
MODS = ['QPSK', '16-QAM', '64-QAM']


@pytest.fixture(scope='module')
def C():
    from lte_phy import _capi
    _capi.device_init()
    return _capi


TOL_FFT = {'f64': 1e-14, 'f32': 2e-6}


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('N', [128, 256, 512, 1024, 2048])
def test_fft_matches_numpy(C, N, prec):
    rs = np.random.RandomState(N)
    x = rs.randn(37, N) + 1j * rs.randn(37, N)
    if prec == 'f32':
        x = x.astype(np.complex64).astype(np.complex128)
    f = C.fft(x, inverse=False, precision=prec)
    ref = np.fft.fft(x, axis=1) / np.sqrt(N)
    assert np.linalg.norm(f - ref) / np.linalg.norm(ref) < TOL_FFT[prec]
    i = C.fft(x, inverse=True, precision=prec)
    ref = np.fft.ifft(x, axis=1) * np.sqrt(N)
    assert np.linalg.norm(i - ref) / np.linalg.norm(ref) < TOL_FFT[prec]


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('mod', MODS)
def test_hard_decision(C, golden, oracle, mod, prec):
    pts = golden[f'qam_{mod}_pts']
    bps = oracle.BPS[mod]
    out = np.zeros(len(pts) * bps, dtype=np.uint8)
    if prec == 'f64':
        x = np.ascontiguousarray(pts, dtype=np.complex128)
        C.check(C.load().lte_hard_host64(bps, len(x), C.ptr(x.view(np.float64), C.F64), C.ptr(out, C.U8)))
    else:
        x = pts.astype(np.complex64)
        C.check(C.load().lte_hard_host(bps, len(x), C.ptr(x.view(np.float32), C.F32), C.ptr(out, C.U8)))
    ref = golden[f'qam_{mod}_hard']
    # exact away from decision boundaries (the golden set deliberately puts a
    # third of its points ON boundaries, where the reference's argmin of
    # hypot distances and a per-axis slicer may round a tie differently)
    nl = {2: 2, 4: 4, 6: 8}[bps]
    sc = {2: np.sqrt(2), 4: np.sqrt(10), 6: np.sqrt(42)}[bps]
    bnd = np.array([0.0]) if bps == 2 else (np.arange(1, nl) * 2 - nl) / sc
    far = np.ones(len(pts), bool)
    for v in (pts.real, pts.imag):
        far &= np.min(np.abs(v[:, None] - bnd[None, :]), axis=1) > (1e-12 if prec == 'f64' else 1e-5)
    far_bits = np.repeat(far, bps)
    assert far.sum() > len(pts) // 2
    assert np.array_equal(out[far_bits], ref[far_bits])


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('mod', MODS)
def test_llr(C, golden, oracle, mod, prec):
    pts, nv = golden['llr_pts'], golden['llr_nv']
    bps = oracle.BPS[mod]
    ref = golden[f'llr_{mod}']
    if prec == 'f64':
        # float64 max-log LLRs; the reference takes min |y - c|^2 over the 2-D
        # constellation (np.abs = hypot), the kernel the separable per-axis
        # minimum (the other axis' term cancels): equal up to f64 round-off
        x = np.ascontiguousarray(pts, dtype=np.complex128)
        n64 = np.ascontiguousarray(nv, dtype=np.float64)
        out = np.zeros(len(x) * bps)
        C.check(C.load().lte_llr_host64(bps, len(x), C.ptr(x.view(np.float64), C.F64), C.ptr(n64, C.F64),
                                        C.ptr(out, C.F64)))
        assert np.max(np.abs(out - ref) / (1 + np.abs(ref))) < 1e-12
    else:
        x = pts.astype(np.complex64)
        n32 = nv.astype(np.float32)
        out = np.zeros(len(x) * bps, dtype=np.float32)
        C.check(C.load().lte_llr_host(bps, len(x), C.ptr(x.view(np.float32), C.F32), C.ptr(n32, C.F32),
                                      C.ptr(out, C.F32)))
        assert np.max(np.abs(out - ref) / (1 + np.abs(ref))) < 1e-4


@pytest.mark.parametrize('K', [40, 1024, 5568, 5632, 6144])
def test_turbo_encode_bit_exact(C, golden, K):
    from lte_phy import channel_coding as cc
    cb = unpack(golden[f'enc_{K}_in'], K)
    assert np.array_equal(cc.turbo_encode(cb), unpack(golden[f'enc_{K}_out'], 3 * K + 12))


def test_turbo_encode_batch(C, oracle):
    K, n = 5632, 200
    bits = np.random.RandomState(1).randint(0, 2, (n, K)).astype(np.uint8)
    out = np.zeros((n, 3 * K + 12), dtype=np.uint8)
    C.check(C.load().lte_turbo_encode_host(K, n, C.ptr(bits, C.U8), C.ptr(out, C.U8)))
    for i in range(0, n, 37):
        assert np.array_equal(out[i], oracle.turbo_encode(bits[i]))


@pytest.mark.parametrize('vec', ['zeros40', 'ones40', 'alt40', 'rand27760'])
def test_crc24a(C, golden, vec):
    from lte_phy import channel_coding as cc
    assert np.array_equal(cc.calculate_crc24a(golden[f'crc_{vec}_in']), golden[f'crc_{vec}_24a'])


def test_bcjr_app(C, golden):
    """f32 fast mode: K + 3 steps through the decoder rows, within f32 round-off."""
    ls, lp, la = golden['bcjr_ls'], golden['bcjr_lp'], golden['bcjr_la']
    K = len(ls) - 3
    app = np.zeros(K, dtype=np.float32)
    f = [np.ascontiguousarray(v, dtype=np.float32) for v in (ls, lp, la)]
    C.check(C.load().lte_bcjr_host(K, 1, *[C.ptr(v, C.F32) for v in f], C.ptr(app, C.F32)))
    ref = golden['bcjr_app'][:K]
    assert np.max(np.abs(app - ref)) < 2e-3 * (1 + np.max(np.abs(ref)))
    assert np.array_equal(app < 0, ref < 0)


def test_bcjr_app_f64_exact(C, golden, oracle):
    """float64 LogMAPDecoder.decode (return_extrinsic=False) over all K + 3
    steps: bit-identical to the reference's output and to the C oracle."""
    ls, lp, la = (np.ascontiguousarray(golden[k], dtype=np.float64) for k in ('bcjr_ls', 'bcjr_lp', 'bcjr_la'))
    n = len(ls)
    app = np.zeros(n)
    C.check(C.load().lte_bcjr_host64(n, 1, *[C.ptr(v, C.F64) for v in (ls, lp, la)], C.ptr(app, C.F64)))
    assert np.array_equal(app, golden['bcjr_app'])
    assert np.array_equal(app, oracle.bcjr_app(ls, lp, la))


@pytest.mark.parametrize('K,its', [(40, 8), (1024, 1), (1024, 8), (5568, 2)])
def test_turbo_decode_golden(C, golden, oracle, K, its):
    """Default (float64) decoder == the reference's own decoded bits on its own
    decoder inputs, for every case (north_star: BER match; here exact)."""
    from lte_phy import channel_coding as cc
    key = f'td_{K}_{its}'
    llr = golden[key + '_llr'].astype(np.float64)
    dec = cc.turbo_decode(llr, K, its)
    ref = unpack(golden[key + '_dec'], K)
    assert np.array_equal(dec, ref)
    assert np.array_equal(dec, oracle.turbo_decode(llr, K, its))


@pytest.mark.parametrize('K,its', [(40, 8), (1024, 1), (1024, 8), (5568, 2)])
def test_turbo_decode_golden_f32(C, golden, oracle, K, its):
    """f32 fast mode == its float32 algorithm bit-for-bit (how that algorithm
    relates to the float64 reference is pinned on the CPU:
    tests/test_turbo_model.py)."""
    from lte_phy import channel_coding as cc
    key = f'td_{K}_{its}'
    llr = golden[key + '_llr'].astype(np.float32)
    dec = cc.turbo_decode(llr, K, its, precision='f32')
    assert np.array_equal(dec, oracle.turbo_decode_f32_model(llr, K, its))
    ref = unpack(golden[key + '_dec'], K)
    if its <= 2 or K == 40:    # converging cases: equal to the reference itself
        assert np.array_equal(dec, ref)


@pytest.mark.parametrize('K,n,snr', [(5568, 130, 1.5), (5632, 70, 3.0), (6144, 64, 5.0), (40, 200, 2.0),
                                     (48, 64, 2.0), (56, 64, 2.0), (1056, 64, 2.5)])
def test_turbo_decode_batch_vs_oracle(C, oracle, K, n, snr):
    """Several decoder waves of one K (partial last wave included), below and
    above the turbo cliff: the float64 decoder is bit-exact vs the float64
    oracle (= the reference) on every code block; the f32 fast mode is
    bit-exact vs its float32 model."""
    from lte_phy import channel_coding as cc
    rs = np.random.RandomState(K)
    cbs = rs.randint(0, 2, (n, K)).astype(np.uint8)
    llr = np.zeros((n, 3 * K + 12))
    s2 = 10 ** (-snr / 10)
    for i in range(n):
        s = 1 - 2.0 * oracle.turbo_encode(cbs[i])
        llr[i] = 2 * (s + np.sqrt(s2) * rs.randn(len(s))) / s2
    dec = cc.turbo_decode_batch(llr, K, 8)
    for i in range(n):
        assert np.array_equal(dec[i], oracle.turbo_decode(llr[i], K, 8)), i
    l32 = llr.astype(np.float32)
    dec = cc.turbo_decode_batch(l32, K, 8, precision='f32')
    for i in range(n):
        assert np.array_equal(dec[i], oracle.turbo_decode_f32_model(l32[i], K, 8)), i


def _sim(bw, mod, chan, prec=None, **kw):
    import lte_phy
    return lte_phy.OFDMSimulator(lte_phy.LTEConfig(bandwidth=bw, modulation=mod), channel_type=chan,
                                 precision=prec, **kw)


def _state_head():
    return np.array(np.random.get_state()[1][:8], dtype=np.uint32)


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('name,bw,mod,chan,snrs', [
    ('e2e_c1', 1.25, 'QPSK', 'awgn', [0, 5, 10]),
    ('e2e_c1odd', 1.25, 'QPSK', 'awgn', [3]),
    ('e2e_c2', 20.0, '64-QAM', 'rayleigh_mp', [0, 10, 20, 30]),
    ('e2e_c2awgn', 20.0, '16-QAM', 'awgn', [12])])
def test_simulate_siso_ref_compat(C, golden, name, bw, mod, chan, snrs, prec):
    """Drop-in OFDMSimulator.simulate_siso == the reference's own output (frozen
    RNG).  f64: identical received bits; f32: within the north-star 1e-3."""
    sim = _sim(bw, mod, chan, prec)
    nb = int(golden[name + '_nbits'][0])
    bits = unpack(golden[name + '_bits'], nb).astype(np.int64)
    for snr in snrs:
        k = f'{name}_snr{snr}'
        r = sim.simulate_siso(bits, snr)
        ref_err = int(golden[k + '_errors'][0])
        diff = np.mean(r['bits_received_array'] != unpack(golden[k + '_rx'], nb))
        if prec == 'f64':
            assert r['bit_errors'] == ref_err and diff == 0, (k, r['bit_errors'], ref_err, diff)
        else:
            assert abs(r['bit_errors'] - ref_err) / nb < 1e-3, (k, r['bit_errors'], ref_err)
            assert diff < 1e-3, (k, diff)
        assert abs(r['papr_db'] - golden[k + '_papr'][0]) < (1e-9 if prec == 'f64' else 1e-3)
        assert np.array_equal(_state_head(), golden[k + '_state']), 'global RNG side effects differ'


@pytest.mark.parametrize('prec,tol', [('f64', 1e-13), ('f32', 1e-5)])
def test_simulate_siso_signals_vs_oracle(C, oracle, golden, prec, tol):
    """Sample-level parity of the captured TX / RX streams (config 2)."""
    sim = _sim(20.0, '64-QAM', 'rayleigh_mp', prec)
    nb = int(golden['e2e_c2_nbits'][0])
    bits = unpack(golden['e2e_c2_bits'], nb).astype(np.int64)
    r = sim.simulate_siso(bits, 20)
    num = oracle.Numerology(bandwidth=20.0, modulation='64-QAM')
    o = oracle.simulate_siso(num, bits, 20, 'rayleigh_mp')
    for key in ['signal_tx', 'signal_rx']:
        a, b = r[key], o[key]
        assert np.linalg.norm(a - b) / np.linalg.norm(b) < tol, key
    a, b = r['symbols_rx'], o['symbols_rx']
    assert np.median(np.abs(a - b)) < (1e-12 if prec == 'f64' else 1e-4)


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('name,bw,mod,chan,snrs,nrx', [
    ('e2e_c3', 10.0, '16-QAM', 'rayleigh_mp', [5, 15], 4),
    ('e2e_c1simo', 1.25, 'QPSK', 'awgn', [2], 2)])
def test_simulate_simo_ref_compat(C, golden, name, bw, mod, chan, snrs, nrx, prec):
    sim = _sim(bw, mod, chan, prec)
    nb = int(golden[name + '_nbits'][0])
    bits = unpack(golden[name + '_bits'], nb).astype(np.int64)
    for snr in snrs:
        k = f'{name}_snr{snr}'
        r = sim.simulate_simo(bits, snr, num_rx=nrx, parallel=False)
        ref_err = int(golden[k + '_errors'][0])
        if prec == 'f64':
            assert r['bit_errors'] == ref_err, (k, r['bit_errors'], ref_err)
        else:
            assert abs(r['bit_errors'] - ref_err) / nb < 1e-3, (k, r['bit_errors'], ref_err)
        assert np.array_equal(_state_head(), golden[k + '_state'])


@pytest.mark.parametrize('name,bw,mod,chan,snrs', [
    ('e2e_cod_small', 1.25, 'QPSK', 'awgn', [0, 6]),
    ('e2e_cod_c2s', 20.0, '64-QAM', 'rayleigh_mp', [8, 20]),
    ('e2e_cod_c2', 20.0, '64-QAM', 'rayleigh_mp', [20])])
def test_simulate_siso_coded_ref_compat(C, golden, name, bw, mod, chan, snrs):
    """Headline chain (TX coding -> Rayleigh -> RX + turbo) in float64 vs the
    reference's own output on its own random numbers: identical bit errors,
    CRC verdict, measured SNR and noise variance, and global-RNG state --
    including the frames the reference fails to decode (past the turbo cliff)."""
    sim = _sim(bw, mod, chan, 'f64')
    if name + '_nbits' not in golden:
        pytest.skip('slow golden vector absent')
    nb = int(golden[name + '_nbits'][0])
    bits = unpack(golden[name + '_bits'], nb).astype(np.int64)
    for snr in snrs:
        k = f'{name}_snr{snr}'
        r = sim.simulate_siso_coded(bits, snr)
        ref_err = int(golden[k + '_errors'][0])
        assert r['bit_errors'] == ref_err, (k, r['bit_errors'], ref_err)
        assert bool(r['crc_pass']) == bool(int(golden[k + '_crc'][0])), k
        assert abs(r['channel_snr_db'] - golden[k + '_chsnr'][0]) < 1e-9
        assert abs(r['noise_var_mean'] / golden[k + '_nvmean'][0] - 1) < 1e-12
        assert np.array_equal(_state_head(), golden[k + '_state'])


@pytest.mark.parametrize('name,bw,mod,chan,snrs', [
    ('e2e_cod_small', 1.25, 'QPSK', 'awgn', [0, 6]),
    ('e2e_cod_c2s', 20.0, '64-QAM', 'rayleigh_mp', [8, 20])])
def test_simulate_siso_coded_ref_compat_f32(C, golden, name, bw, mod, chan, snrs):
    """f32 fast mode on the same vectors: frames the reference decodes decode
    cleanly with identical CRC; past the turbo cliff f32 round-off changes which
    wrong bits come out, so only the CRC verdict is compared there."""
    sim = _sim(bw, mod, chan, 'f32')
    nb = int(golden[name + '_nbits'][0])
    bits = unpack(golden[name + '_bits'], nb).astype(np.int64)
    for snr in snrs:
        k = f'{name}_snr{snr}'
        r = sim.simulate_siso_coded(bits, snr)
        ref_err = int(golden[k + '_errors'][0])
        if ref_err == 0:
            assert r['bit_errors'] == 0 and r['crc_pass'] and int(golden[k + '_crc'][0]) == 1, k
        else:
            assert not r['crc_pass'] and int(golden[k + '_crc'][0]) == 0, k
        assert np.array_equal(_state_head(), golden[k + '_state'])


@pytest.mark.parametrize('prec', ['f64', 'f32'])
def test_run_grid_sharding_invariant(C, prec):
    """Philox keyed by global frame id: 2-way sharded counts sum to the unsharded counts."""
    sim = _sim(20.0, '64-QAM', 'rayleigh_mp', prec)
    a = sim.run_grid([5.0, 15.0], 40, seed=7)
    b0 = sim.run_grid([5.0, 15.0], 40, seed=7, rank=0, world_size=2)
    b1 = sim.run_grid([5.0, 15.0], 40, seed=7, rank=1, world_size=2)
    assert np.array_equal(a['counts'], b0['counts'] + b1['counts'])


def test_run_grid_statistics_vs_oracle(C, oracle):
    """Philox Monte-Carlo BER vs the oracle's own Monte-Carlo (independent
    draws, same model): agree within a binomial-confidence tolerance."""
    sim = _sim(20.0, '64-QAM', 'rayleigh_mp')
    g = sim.run_grid([10.0, 20.0], 64, seed=3)
    num = oracle.Numerology(bandwidth=20.0, modulation='64-QAM')
    rs = np.random.RandomState(11)
    for i, snr in enumerate([10.0, 20.0]):
        errs = bits = 0
        for t in range(24):
            b = rs.randint(0, 2, 14 * num.Nd * 6)
            L = 14 * (num.N + num.cp)
            np.random.seed(1000 + t)
            d = [{'phases': [2 * np.pi * np.random.rand(16) for _ in range(4)],
                  'z_re': np.random.randn(L), 'z_im': np.random.randn(L)}]
            r = oracle.simulate_siso(num, b, snr, 'rayleigh_mp', draws=d)
            errs += r['bit_errors']
            bits += len(b)
        p_ref = errs / bits
        p_gpu = g['ber'][i]
        # the per-frame fading realisation dominates the variance: allow 35 % relative
        assert abs(p_gpu - p_ref) <= 0.35 * p_ref + 2e-3, (snr, p_gpu, p_ref)


@pytest.mark.parametrize('prec', ['f64', 'f32'])
def test_coded_rx_decode_vs_oracle_on_philox_frames(C, oracle, prec):
    """RX decode path (T/F de-interleave + rate dematch + turbo + desegment +
    CRC) on realistic Philox frames: feed the GPU's own LLRs (captured) to the
    oracle's RX decode chain.  f64: the reference's float64 decoder gives the
    GPU's decoded TB bits and CRC verdicts on every frame; f32: its float32
    decoder model does."""
    sim = _sim(20.0, '64-QAM', 'rayleigh_mp', prec)
    plan = sim._plan(C.CHAIN_CODED, 0, 27760, max_frames=8)
    snrs = np.array([6, 9, 12, 15, 18, 21, 24, 30], dtype=np.float64)
    r = plan.run(snrs, seed=11, capture=('llr', 'bits_rx'))
    assert r['llr'].dtype == (np.float64 if prec == 'f64' else np.float32)
    num = oracle.Numerology(bandwidth=20.0, modulation='64-QAM')
    bps, Nd = 6, num.Nd
    coded = plan.coded_bits
    ncs = coded // bps
    rows = -(-ncs // Nd)
    tb = np.zeros(27760, dtype=np.uint8)
    _, seg_plan = oracle.segment(oracle.attach_crc24a(tb))
    q = np.arange(ncs)
    src_re = (q % Nd) * rows + q // Nd
    rm = [3 * p[0] + 12 for p in seg_plan]
    n_ok = 0
    for b in range(len(snrs)):
        L_re = r['llr'][b].astype(np.float64).reshape(-1, bps)
        L = L_re[src_re].reshape(-1)[:coded]
        dec, ok = oracle.coded_rx_decode(L, seg_plan, rm, 8, f32_model=(prec == 'f32'))
        assert np.array_equal(dec, r['bits_rx'][b]) and bool(ok) == bool(r['crc_ok'][b]), b
        n_ok += int(ok)
    assert 2 <= n_ok < len(snrs)   # decoded and failed frames both covered


@pytest.mark.parametrize('prec,tol', [('f64', 1e-12), ('f32', 1e-4)])
@pytest.mark.parametrize('bw,mod', [(20.0, '64-QAM'), (5.0, '16-QAM'), (1.25, 'QPSK')])
def test_coded_chain_llrs_vs_oracle(C, oracle, bw, mod, prec, tol):
    """In-chain soft demapper: the LLRs k_rx_data writes == the oracle's max-log
    LLRs (core/ofdm_core.py:791-923) of the same equalised symbols with the
    same per-RE noise variance (ofdm_core.py:1224-1243)."""
    sim = _sim(bw, mod, 'rayleigh_mp', prec)
    plan = sim._plan(C.CHAIN_CODED, 0, 2000, max_frames=3)
    snrs = np.array([3.0, 12.0, 25.0])
    r = plan.run(snrs, seed=5, capture=('llr', 'data_syms', 'H'))
    num = oracle.Numerology(bandwidth=bw, modulation=mod)
    for b, snr in enumerate(snrs):
        sy = r['data_syms'][b].astype(np.complex128)
        Hs = r['H'][b, 0].astype(np.complex128)
        Hd = np.concatenate([Hs[l // 14][num.data_idx] for l in range(plan.n_sym)])
        nv = oracle.noise_var_per_symbol(Hd, snr, 'rayleigh_mp')
        ref = oracle.llrs(sy, nv, mod)
        got = r['llr'][b].astype(np.float64)[:len(ref)]
        assert np.max(np.abs(got - ref) / (1 + np.abs(ref))) < tol, (b, snr)


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('chain', ['coded', 'uncoded'])
def test_fused_tx_channel_matches_separate_kernels(C, monkeypatch, chain, prec):
    """TX with the static-tap channel fused in (k_ofdm_tx<.., CH> + k_chan_fix)
    vs the separate TX and channel kernels, on the same Philox frames: noise
    power (the measured-power SNR, Q5), channel estimates and LLRs agree to
    round-off (the power is summed per symbol instead of per 2048-sample
    block); decisions agree up to that round-off."""
    sim = _sim(20.0, '64-QAM', 'rayleigh_mp', prec)
    B = 3 * 64 + 5
    coded = chain == 'coded'
    plan = sim._plan(C.CHAIN_CODED, 0, 27760, max_frames=B) if coded else \
        sim._plan(C.CHAIN_UNCODED, 14, 14 * sim.Nd * 6, max_frames=B)
    snr = np.tile(np.arange(0.0, 31.0, 2.0), B)[:B]
    cap = ('noise_power', 'H') + (('llr',) if coded else ())
    monkeypatch.setenv('LTE_TXCH_FUSE', '0')
    a = plan.run(snr, seed=0x5EED, frame_id0=77, capture=cap)
    monkeypatch.setenv('LTE_TXCH_FUSE', '1')
    b = plan.run(snr, seed=0x5EED, frame_id0=77, capture=cap)
    f64 = prec == 'f64'
    assert np.max(np.abs(b['noise_power'] / a['noise_power'] - 1)) < (1e-13 if f64 else 2e-6)
    assert np.max(np.abs(b['H'] - a['H'])) < (1e-12 if f64 else 1e-4) * np.max(np.abs(a['H']))
    if coded:
        # LLR = d^2 difference / (2 sigma^2_eff): at 30 dB a 1e-7 change of the
        # received sample moves it by ~1e-4 (measured 2e-4 at most) in f32
        assert np.max(np.abs(b['llr'] - a['llr']) / (1 + np.abs(a['llr']))) < (1e-9 if f64 else 1e-3)
        assert int(np.sum(a['crc_ok'] != b['crc_ok'])) <= (0 if f64 else 1)
    ea, eb = int(a['counts'][:, 0].sum()), int(b['counts'][:, 0].sum())
    assert abs(ea - eb) <= (2 if f64 else 1e-3 * ea + 5), (ea, eb)
    assert np.array_equal(a['counts'][:, 1], b['counts'][:, 1])


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('chain,bw,mod', [('coded', 20.0, '64-QAM'), ('coded', 5.0, '16-QAM'),
                                          ('uncoded', 20.0, '64-QAM'), ('uncoded', 1.25, 'QPSK')])
def test_fused_receiver_matches_separate_kernels(C, monkeypatch, chain, bw, mod, prec):
    """The fused SISO receiver (k_rx_frame: estimation on each group's first
    symbol + data path, per-subcarrier equaliser terms) vs k_rx_chest +
    k_rx_data on the same Philox frames: channel estimates, pilot statistics,
    equalised symbols and LLRs to round-off (same operations; the per-
    subcarrier terms are formed once instead of per RE), identical decisions
    and counts; and without captures (the demap-in-dematch path) identical
    per-frame bit errors and CRC verdicts."""
    sim = _sim(bw, mod, 'rayleigh_mp', prec)
    B = 64 + 7
    coded = chain == 'coded'
    plan = sim._plan(C.CHAIN_CODED, 0, 27760 if bw == 20.0 else 3000, max_frames=B) if coded else \
        sim._plan(C.CHAIN_UNCODED, 14, 14 * sim.Nd * sim.config.bits_per_symbol, max_frames=B)
    snr = np.tile(np.arange(0.0, 31.0, 2.0), B)[:B]
    cap = ('H', 'pilot_stats', 'data_syms') + (('llr',) if coded else ('bits_rx',))
    runs = {}
    for fuse in ('0', '1'):
        monkeypatch.setenv('LTE_RX_FUSE', fuse)
        runs[fuse] = (plan.run(snr, seed=0x5EED, frame_id0=3, capture=cap),
                      plan.run(snr, seed=0x5EED, frame_id0=3))
    (a, a0), (b, b0) = runs['0'], runs['1']
    tol = 1e-13 if prec == 'f64' else 1e-5
    for k in ('H', 'pilot_stats', 'data_syms'):
        assert np.max(np.abs(b[k] - a[k])) <= tol * np.max(np.abs(a[k])), k
    if coded:
        assert np.max(np.abs(b['llr'] - a['llr']) / (1 + np.abs(a['llr']))) < (1e-10 if prec == 'f64' else 1e-3)
        assert np.array_equal(a['crc_ok'], b['crc_ok'])
        assert np.array_equal(a0['frame_errors'], b0['frame_errors']) and np.array_equal(a0['crc_ok'], b0['crc_ok'])
        assert 0 < int(np.sum(b0['crc_ok'])) < B
    else:
        assert int(np.sum(a['bits_rx'] != b['bits_rx'])) <= 2
    assert abs(int(a0['counts'][:, 0].sum()) - int(b0['counts'][:, 0].sum())) <= (0 if coded else 2)
    assert np.array_equal(a0['counts'][:, 1], b0['counts'][:, 1])


@pytest.mark.parametrize('mod,chan,inject', [('64-QAM', 'rayleigh_mp', False), ('16-QAM', 'awgn', False),
                                             ('64-QAM', 'rayleigh_mp', True)])
def test_wave_receiver_matches_block_receiver(C, monkeypatch, mod, chan, inject):
    """The wave-private receiver (k_rx_frame_w: one wave per frame, wfft's
    register / wave-local-LDS 2048-point FFT, pair-shared Philox draws traded
    by DPP) vs the block receiver k_rx_frame (fft_lds) on the same frames,
    Philox or injected noise: channel estimates, pilot statistics and
    equalised symbols agree to the two FFTs' round-off (each within a few
    1e-14 of the exact DFT), and the decoded outcome -- per-frame bit errors,
    CRC verdicts, counts -- is identical.  B = 4 k + 3 leaves a block with
    three of its four waves."""
    sim = _sim(20.0, mod, chan, 'f64')
    B = 4 * 12 + 3
    plan = sim._plan(C.CHAIN_CODED, 0, 27760, max_frames=B)
    snr = np.tile(np.arange(4.0, 31.0, 2.0), B)[:B]
    kw = {}
    if inject:
        z = np.random.default_rng(11).standard_normal((B, 2, plan.L))
        kw = dict(noise=z)
    runs = {}
    for wave in ('0', '1'):
        monkeypatch.setenv('LTE_RX_WAVE', wave)
        runs[wave] = (plan.run(snr, seed=0x5EED, frame_id0=3, capture=('H', 'pilot_stats', 'data_syms'), **kw),
                      plan.run(snr, seed=0x5EED, frame_id0=3, **kw))
    (a, a0), (b, b0) = runs['0'], runs['1']
    for k in ('H', 'pilot_stats', 'data_syms'):
        assert np.max(np.abs(b[k] - a[k])) <= 1e-12 * np.max(np.abs(a[k])), k
    for r, s in ((a, b), (a0, b0)):
        assert np.array_equal(r['frame_errors'], s['frame_errors']) and np.array_equal(r['crc_ok'], s['crc_ok'])
        assert np.array_equal(r['counts'], s['counts'])
    assert 0 < int(np.sum(b0['crc_ok'])) < B


@pytest.mark.parametrize('prec,inject', [('f64', False), ('f64', True), ('f32', False)])
def test_simo_symbol_handoff_matches_rx_streams(C, monkeypatch, prec, inject):
    """Config 3's TX hands the paired receiver its symbols and the receiver
    applies each RX's taps (TxChannelT::x_out, k_rx_frame_simo2<.., XIN>,
    opt-in LTE_SIMO_XHAND=1) vs the TX writing every RX stream (default): the same
    taps in the same order over the cyclic symbol, so combined symbols agree to
    round-off (float64 1e-12) and decisions and counts are identical in
    float64; Philox and injected noise; 4 RX, Vehicular-A (delays to the CP)."""
    import lte_phy
    sim = lte_phy.OFDMSimulator(lte_phy.LTEConfig(bandwidth=10.0, modulation='16-QAM'), channel_type='rayleigh_mp',
                                itu_profile='Vehicular_A', precision=prec)
    B = 32 + 3
    plan = sim._plan(C.CHAIN_SIMO, 14, 14 * sim.Nd * 4, num_rx=4, max_frames=B)
    snr = np.tile(np.arange(0.0, 31.0, 2.0), B)[:B]
    kw = {}
    if inject:
        kw = dict(noise=np.random.default_rng(5).standard_normal((B, 4, 2, plan.L)))
    runs = {}
    monkeypatch.setenv('LTE_SIMO_RX_WAVE', '0')   # both sides on k_rx_frame_simo2 (the wave receiver: its own test)
    monkeypatch.setenv('LTE_SIMO_TX_WAVE', '0')   # and on k_ofdm_tx (the wave TX: its own test)
    for xh in ('0', '1'):
        monkeypatch.setenv('LTE_SIMO_XHAND', xh)
        runs[xh] = (plan.run(snr, seed=0x5EED, frame_id0=11, capture=('data_syms', 'bits_rx', 'noise_power'), **kw),
                    plan.run(snr, seed=0x5EED, frame_id0=11, **kw))
    (a, a0), (b, b0) = runs['0'], runs['1']
    tol = 1e-12 if prec == 'f64' else 1e-5
    assert np.array_equal(a['noise_power'], b['noise_power'])   # the TX forms the powers either way
    assert np.max(np.abs(b['data_syms'] - a['data_syms'])) <= tol * np.max(np.abs(a['data_syms']))
    if prec == 'f64':
        assert np.array_equal(a['bits_rx'], b['bits_rx'])
        assert np.array_equal(a0['counts'], b0['counts']) and np.array_equal(a0['frame_errors'], b0['frame_errors'])
    else:
        assert int(np.sum(a['bits_rx'] != b['bits_rx'])) <= 4
    assert 0 < int(b0['counts'][:, 0].sum())


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('bw,mod,nrx,prof', [(10.0, '16-QAM', 4, 'Vehicular_A'), (20.0, '64-QAM', 2, 'Pedestrian_A'),
                                             (1.25, 'QPSK', 3, 'Pedestrian_A')])
def test_fused_simo_receiver_matches_separate_kernels(C, monkeypatch, bw, mod, nrx, prof, prec):
    """The fused SIMO MRC receiver (k_rx_frame_simo: every RX's estimate on
    each group's first symbol, kept per data subcarrier, MRC over the RX in
    order) vs k_rx_chest + k_rx_data<SIMO> on the same Philox frames: channel
    estimates, pilot statistics and combined symbols to round-off, decisions
    and counts identical."""
    import lte_phy
    sim = lte_phy.OFDMSimulator(lte_phy.LTEConfig(bandwidth=bw, modulation=mod), channel_type='rayleigh_mp',
                                itu_profile=prof, precision=prec)
    B = 64 + 5
    bps = sim.config.bits_per_symbol
    plan = sim._plan(C.CHAIN_SIMO, 14, 14 * sim.Nd * bps, num_rx=nrx, max_frames=B)
    snr = np.tile(np.arange(0.0, 31.0, 2.0), B)[:B]
    cap = ('H', 'pilot_stats', 'data_syms', 'bits_rx')
    runs = {}
    for fuse in ('0', '1'):
        monkeypatch.setenv('LTE_RX_FUSE', fuse)
        runs[fuse] = (plan.run(snr, seed=0x5EED, frame_id0=11, capture=cap),
                      plan.run(snr, seed=0x5EED, frame_id0=11))
    (a, a0), (b, b0) = runs['0'], runs['1']
    tol = 1e-13 if prec == 'f64' else 1e-5
    for k in ('H', 'pilot_stats', 'data_syms'):
        assert np.max(np.abs(b[k] - a[k])) <= tol * np.max(np.abs(a[k])), k
    assert int(np.sum(a['bits_rx'] != b['bits_rx'])) <= 2
    assert abs(int(a0['counts'][:, 0].sum()) - int(b0['counts'][:, 0].sum())) <= 2
    assert np.array_equal(a0['counts'][:, 1], b0['counts'][:, 1])
    assert 0 < int(b0['counts'][:, 0].sum())


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('nrx,mod', [(4, '16-QAM'), (2, '64-QAM'), (4, 'QPSK')])
def test_simo_receiver_rx_pairs_match_sequential(C, monkeypatch, nrx, mod, prec):
    """10 MHz SIMO MRC: k_rx_frame_simo2 (one frame per block, the RX in pairs,
    each half of the block transforming one RX of the pair, the MRC sums in
    RX order) against k_rx_frame_simo (the RX in sequence, LTE_RXS_PAIRS=0):
    the same operations per RE, so identical combined symbols, received bits
    and counts on the same Philox frames (float64; float32 to round-off)."""
    import lte_phy
    sim = lte_phy.OFDMSimulator(lte_phy.LTEConfig(bandwidth=10.0, modulation=mod), channel_type='rayleigh_mp',
                                itu_profile='Vehicular_A', precision=prec)
    B = 64 + 3
    bps = sim.config.bits_per_symbol
    plan = sim._plan(C.CHAIN_SIMO, 14, 14 * sim.Nd * bps - 5, num_rx=nrx, max_frames=B)
    snr = np.tile(np.arange(0.0, 31.0, 2.0), B)[:B]
    cap = ('data_syms', 'bits_rx')
    runs = {}
    monkeypatch.setenv('LTE_SIMO_RX_WAVE', '0')   # k_rx_frame_simo2, not the wave receiver (its own test)
    for pairs in ('0', '1'):
        monkeypatch.setenv('LTE_RXS_PAIRS', pairs)
        runs[pairs] = plan.run(snr, seed=0x5EED, frame_id0=77, capture=cap)
    a, b = runs['0'], runs['1']
    if prec == 'f64':
        assert np.array_equal(a['data_syms'], b['data_syms'])
        assert np.array_equal(a['bits_rx'], b['bits_rx'])
        assert np.array_equal(a['counts'], b['counts'])
    else:
        assert np.max(np.abs(b['data_syms'] - a['data_syms'])) <= 1e-5 * np.max(np.abs(a['data_syms']))
        assert int(np.sum(a['bits_rx'] != b['bits_rx'])) <= 2
    assert 0 < int(b['counts'][:, 0].sum())


@pytest.mark.parametrize('nrx,mod,prof', [(4, '16-QAM', 'Vehicular_A'), (2, '64-QAM', 'Pedestrian_A'),
                                          (3, 'QPSK', 'Vehicular_A')])
def test_wave_simo_tx_matches_block_tx(C, monkeypatch, nrx, mod, prof):
    """10 MHz SIMO TX + static taps, float64: the wave-private TX
    (k_ofdm_tx_simo_w: one wave per (frame, symbol), wfft::fft1024<INV>, the
    symbol staged in LDS for every RX's taps; the default) against k_ofdm_tx
    (LTE_SIMO_TX_WAVE=0) on the same frames: identical transmitted symbols;
    noise powers and combined symbols to 1e-12 (the transform and the power
    sums differ in round-off only); decisions and counts match (at most 2 flips
    allowed).  4, 2 and 3 RX; 6 and 2 paths."""
    import lte_phy
    sim = lte_phy.OFDMSimulator(lte_phy.LTEConfig(bandwidth=10.0, modulation=mod), channel_type='rayleigh_mp',
                                itu_profile=prof, precision='f64')
    B = 64 + 3
    bps = sim.config.bits_per_symbol
    plan = sim._plan(C.CHAIN_SIMO, 14, 14 * sim.Nd * bps - 5, num_rx=nrx, max_frames=B)
    snr = np.tile(np.arange(0.0, 31.0, 2.0), B)[:B]
    cap = ('tx_syms', 'noise_power', 'data_syms', 'bits_rx')
    runs = {}
    for wave in ('0', '1'):
        monkeypatch.setenv('LTE_SIMO_TX_WAVE', wave)
        runs[wave] = (plan.run(snr, seed=0x5EED, frame_id0=91, capture=cap),
                      plan.run(snr, seed=0x5EED, frame_id0=91))
    (a, a0), (b, b0) = runs['0'], runs['1']
    assert np.array_equal(a['tx_syms'], b['tx_syms'])
    assert np.max(np.abs(b['noise_power'] - a['noise_power']) / np.abs(a['noise_power'])) <= 1e-12
    assert np.max(np.abs(b['data_syms'] - a['data_syms'])) <= 1e-12 * np.max(np.abs(a['data_syms']))
    assert int(np.sum(a['bits_rx'] != b['bits_rx'])) <= 2
    assert abs(int(a0['counts'][:, 0].sum()) - int(b0['counts'][:, 0].sum())) <= 2
    assert np.array_equal(a0['counts'][:, 1], b0['counts'][:, 1])
    assert 0 < int(b0['counts'][:, 0].sum())


@pytest.mark.parametrize('nrx,mod,inject', [(4, '16-QAM', False), (4, '16-QAM', True), (2, '64-QAM', False),
                                            (4, 'QPSK', False)])
def test_wave_simo_receiver_matches_block_receiver(C, monkeypatch, nrx, mod, inject):
    """10 MHz SIMO MRC, float64: the wave-private receiver (k_rx_frame_simo_w:
    one wave per RX with wfft::fft1024, the MRC sums in RX order in LDS; the
    default) against k_rx_frame_simo2 (LTE_SIMO_RX_WAVE=0) on the same Philox
    (or injected) noise.  Only the transform's rounding differs (both FFTs
    within a few 1e-14 of the exact DFT), so combined symbols agree to 1e-12 of
    their scale and decisions and counts match (a decision flip needs a symbol
    within ~1e-13 of a boundary: at most 2 allowed)."""
    import lte_phy
    sim = lte_phy.OFDMSimulator(lte_phy.LTEConfig(bandwidth=10.0, modulation=mod), channel_type='rayleigh_mp',
                                itu_profile='Vehicular_A', precision='f64')
    B = 64 + 3
    bps = sim.config.bits_per_symbol
    plan = sim._plan(C.CHAIN_SIMO, 14, 14 * sim.Nd * bps - 5, num_rx=nrx, max_frames=B)
    snr = np.tile(np.arange(0.0, 31.0, 2.0), B)[:B]
    kw = {}
    if inject:
        kw = dict(noise=np.random.default_rng(7).standard_normal((B, nrx, 2, plan.L)))
    runs = {}
    for wave in ('0', '1'):
        monkeypatch.setenv('LTE_SIMO_RX_WAVE', wave)
        runs[wave] = (plan.run(snr, seed=0x5EED, frame_id0=77, capture=('data_syms', 'bits_rx'), **kw),
                      plan.run(snr, seed=0x5EED, frame_id0=77, **kw))
    (a, a0), (b, b0) = runs['0'], runs['1']
    assert np.max(np.abs(b['data_syms'] - a['data_syms'])) <= 1e-12 * np.max(np.abs(a['data_syms']))
    assert int(np.sum(a['bits_rx'] != b['bits_rx'])) <= 2
    assert abs(int(a0['counts'][:, 0].sum()) - int(b0['counts'][:, 0].sum())) <= 2
    assert np.array_equal(a0['counts'][:, 1], b0['counts'][:, 1])
    assert 0 < int(b0['counts'][:, 0].sum())


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('bw,mod', [(20.0, '64-QAM'), (5.0, '16-QAM'), (10.0, 'QPSK')])
def test_frame_tx_matches_symbol_tx(C, monkeypatch, bw, mod, prec):
    """Coded TX + channel with one slot per frame (k_ofdm_txf, coded streams
    staged once per frame) vs one slot per OFDM symbol (k_ofdm_tx<.., CH>):
    the same operations per sample, so noise powers, transmitted symbols and
    LLRs are identical."""
    sim = _sim(bw, mod, 'rayleigh_mp', prec)
    B = 64 + 3
    plan = sim._plan(C.CHAIN_CODED, 0, 27760 if bw == 20.0 else 4000, max_frames=B)
    snr = np.tile(np.arange(0.0, 31.0, 2.0), B)[:B]
    cap = ('noise_power', 'tx_syms', 'llr')
    monkeypatch.setenv('LTE_TX_WAVE', '0')   # the block per-frame kernel (k_ofdm_txf_w: its own test)
    monkeypatch.setenv('LTE_TX_FRAME', '0')
    a = plan.run(snr, seed=0x5EED, frame_id0=21, capture=cap)
    monkeypatch.setenv('LTE_TX_FRAME', '1')
    b = plan.run(snr, seed=0x5EED, frame_id0=21, capture=cap)
    for k in cap:
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(a['crc_ok'], b['crc_ok']) and np.array_equal(a['counts'], b['counts'])


@pytest.mark.parametrize('mod', ['64-QAM', '16-QAM'])
def test_wave_tx_matches_block_tx(C, monkeypatch, mod):
    """The wave-private coded TX + static taps (k_ofdm_txf_w: one wave per
    frame, wfft's inverse 2048-point FFT, the taps' cyclic reach through the
    wave's LDS window) vs the block kernel k_ofdm_txf on the same frames:
    identical transmitted symbols; the received stream and the noise powers
    agree to the two inverse FFTs' round-off; identical decoded outcome.  Both
    values of LTE_TXW_STAGE (coded streams staged in LDS or gathered through
    L1 / L2) are the same kernel otherwise and must agree exactly."""
    sim = _sim(20.0, mod, 'rayleigh_mp', 'f64')
    B = 2 * 20 + 1
    plan = sim._plan(C.CHAIN_CODED, 0, 27760 if mod == '64-QAM' else 18000, max_frames=B)
    snr = np.tile(np.arange(0.0, 31.0, 2.0), B)[:B]
    cap = ('noise_power', 'tx_syms', 'signal_rx')
    runs = {}
    for wave, stage in (('0', '1'), ('1', '1'), ('1', '0')):
        monkeypatch.setenv('LTE_TX_WAVE', wave)
        monkeypatch.setenv('LTE_TXW_STAGE', stage)
        runs[wave + stage] = plan.run(snr, seed=0x5EED, frame_id0=5, capture=cap)
    a, b, c = runs['01'], runs['11'], runs['10']
    assert np.array_equal(a['tx_syms'], b['tx_syms'])
    for k in ('signal_rx', 'noise_power'):
        assert np.max(np.abs(b[k] - a[k])) <= 1e-12 * np.max(np.abs(a[k])), k
    for k in cap + ('crc_ok', 'counts', 'frame_errors'):
        assert np.array_equal(b[k], c[k]), k
    assert np.array_equal(a['crc_ok'], b['crc_ok']) and np.array_equal(a['counts'], b['counts'])
    assert np.array_equal(a['frame_errors'], b['frame_errors'])


@pytest.mark.parametrize('prec', ['f64', 'f32'])
def test_txf_lane_order_matches_re_order(C, monkeypatch, prec):
    """k_ofdm_txf with the plan-time bank-aware lane order (LTE_TXF_LANE_ORDER=1,
    off by default since round 5) and in RE order: the lane order only changes
    which lane forms which RE, so the transmitted symbols, noise powers, LLRs
    and counts are identical; plan creation with the order times its greedy
    search (printed for the record)."""
    import time
    from lte_phy import engine
    sim = _sim(20.0, '64-QAM', 'rayleigh_mp', prec)
    B = 64 + 5
    snr = np.tile(np.arange(0.0, 31.0, 2.0), B)[:B]
    cap = ('noise_power', 'tx_syms', 'llr')
    outs, secs = [], []
    monkeypatch.setenv('LTE_TX_WAVE', '0')   # RE order on the block kernel too
    for lo in ('1', '0'):
        monkeypatch.setenv('LTE_TXF_LANE_ORDER', lo)
        engine.clear_cache()
        t = time.perf_counter()
        plan = sim._plan(C.CHAIN_CODED, 0, 27760, max_frames=B)
        secs.append(time.perf_counter() - t)
        outs.append(plan.run(snr, seed=0x5EED, frame_id0=77, capture=cap))
    engine.clear_cache()
    a, b = outs
    for k in cap:
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(a['crc_ok'], b['crc_ok']) and np.array_equal(a['counts'], b['counts'])
    print(f'plan create: lane order {secs[0] * 1e3:.1f} ms, RE order {secs[1] * 1e3:.1f} ms')


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('mod', ['16-QAM', '64-QAM'])
def test_demap_in_dematch_matches_llr_path(C, monkeypatch, mod, prec):
    """k_rx_data handing (z, sigma^2_eff) per RE to k_dematch_zn, which runs the
    same max-log demapper while it builds the decoder rows, decodes exactly
    like the LLR round trip (k_rx_data LLRs -> k_dematch): identical per-frame
    bit errors and CRC flags on the same Philox frames."""
    monkeypatch.setenv('LTE_RX_WAVE', '0')   # both paths on the block receiver: only the demap moves
    sim = _sim(20.0, mod, 'rayleigh_mp', prec)
    B = 2 * 64 + 9
    plan = sim._plan(C.CHAIN_CODED, 0, 27760 if mod == '64-QAM' else 18000, max_frames=B)
    snr = np.tile(np.arange(0.0, 31.0, 2.0), B)[:B]
    monkeypatch.setenv('LTE_DEMAP_IN_DEMATCH', '0')
    a = plan.run(snr, seed=0x5EED, frame_id0=5)
    monkeypatch.setenv('LTE_DEMAP_IN_DEMATCH', '1')
    b = plan.run(snr, seed=0x5EED, frame_id0=5)
    assert np.array_equal(a['frame_errors'], b['frame_errors'])
    assert np.array_equal(a['crc_ok'], b['crc_ok'])
    assert 0 < int(np.sum(a['crc_ok'])) < B


@pytest.mark.parametrize('prec,tol', [('f64', 1e-13), ('f32', 1e-5)])
@pytest.mark.parametrize('chan,profile', [('awgn', 'Pedestrian_A'), ('rayleigh_mp', 'Pedestrian_A'),
                                          ('rayleigh_mp', 'Vehicular_A')])
def test_ofdm_channel_transmit_vs_oracle(C, oracle, monkeypatch, chan, profile, prec, tol):
    """OFDMChannel.transmit (ChannelSimulator.transmit, core/channel.py:334-345)
    on an arbitrary stream through lte_channel_host64 / lte_channel_host: the
    same global-RNG draws as the reference (phases per path, then the two
    normal(L) vectors), output equal to the oracle to round-off."""
    import lte_phy
    monkeypatch.setenv('LTE_PRECISION', prec)
    num = oracle.Numerology(bandwidth=20.0, modulation='64-QAM')
    rs = np.random.RandomState(4)
    x = (rs.randn(20000) + 1j * rs.randn(20000)) / np.sqrt(2)
    ch = lte_phy.OFDMChannel(chan, 12.0, num.fs, itu_profile=profile)
    np.random.seed(99)
    y = ch.transmit(x)
    st = _state_head()
    np.random.seed(99)
    ref = oracle.channel_transmit(num, x, chan, 12.0, profile)
    assert np.array_equal(st, _state_head())
    assert np.linalg.norm(y - ref) / np.linalg.norm(ref) < tol
