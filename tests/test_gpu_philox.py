"""GPU: the Philox mode -- the random streams bench.py and run_grid draw on the
device -- pinned to the oracle's restatement (oracle/philox.py), so the frames
the bench times are the reference's computation on known inputs:

* the device's Philox4x32-10 outputs equal the oracle's bit for bit (the oracle
  is itself pinned to the published known-answer vectors,
  tests/test_oracle_philox.py);
* the device's float64 Box-Muller (table-driven box_muller64t, lte_common.h)
  against the Box-Muller formula evaluated in x87 extended precision (libm
  long double, ~1e-19), errors in ulp of the radius r = sqrt(-2 ln u), on 2^20
  counters (4 M normals): at most 2.5 ulp (the radius itself carries <= 1.15
  ulp, each of cos / sin <= 2^-53; a CPU restatement of the same operations
  measures 2.18 on these draws -- this test found 81 ulp before ln u got its
  own table on [1/2, 1), where -ln 2 + ln c cancelled); against the oracle's
  own float64 libm formula within 8 ulp (that formula itself carries up to 6.1
  ulp from rounding 2 pi v); moments and tails of the float64 and float32
  normals;
* end to end: config-2 bench frames (seed 0x5EED, SNR = frame id mod 16 on
  0:2:30 dB, frame ids at both ends of 65 536-frame bench steps) through the
  float64 GPU chain and through the oracle on the oracle's Philox draws give
  identical per-frame bit errors and CRC verdicts -- at fD = 0 (the headline)
  and at 3 km/h.  tests/test_gpu_fullsize.py does the same on frames of an
  actual 65 536-frame call.
"""
import numpy as np
import pytest

from oracle import philox as P

pytestmark = pytest.mark.gpu

F = 65536
TB = 27760


@pytest.fixture(scope='module')
def C():
    from lte_phy import _capi
    _capi.device_init()
    return _capi


@pytest.mark.parametrize('seed,stream', [(0x5EED, P.STREAM_BITS), (0x5EED, P.STREAM_NOISE),
                                         (0x0123456789ABCDEF, P.STREAM_FADE + 64 * 3 + 5),
                                         (0xFFFFFFFFFFFFFFFF, P.STREAM_MIMO_LINK + 17)])
def test_device_philox_outputs_exact(C, seed, stream):
    fids = np.array([0, 1, 65535, 19 * F + 7, (1 << 32) + 5, (1 << 63) + 12345], dtype=np.uint64)
    u, _, _ = C.philox(seed, fids, stream, 3000)
    for i, f in enumerate(fids):
        ref = P.rng4(seed, int(f), stream, np.arange(3000))
        assert np.array_equal(u[i], ref.T), (i, int(f))


def _bm_longdouble(a, b):
    ld = np.longdouble
    pi = ld('3.14159265358979323846264338327950288')
    u = (a.astype(ld) + ld(0.5)) * ld(2.0) ** -32
    v = (b.astype(ld) + ld(0.5)) * ld(2.0) ** -32
    r = np.sqrt(-2 * np.log(u))
    t = 2 * pi * v
    return r, r * np.cos(t), r * np.sin(t)


def test_device_box_muller64_vs_libm(C):
    n = 1 << 20
    u, g64, g32 = C.philox(0x5EED, [12345], P.STREAM_NOISE, n)
    u, g64, g32 = u[0], g64[0], g32[0]
    worst_x, worst_o = 0.0, 0.0
    for h in range(2):                            # (x, y) -> normals 0, 1; (z, w) -> 2, 3
        a, b = u[:, 2 * h], u[:, 2 * h + 1]
        r, xr, xi = _bm_longdouble(a, b)
        ulp = np.spacing(r.astype(np.float64))
        dev_re, dev_im = g64[:, 2 * h], g64[:, 2 * h + 1]
        ex = np.maximum(np.abs(dev_re - xr), np.abs(dev_im - xi)) / ulp
        o_re, o_im = P.box_muller(a, b)
        eo = np.maximum(np.abs(dev_re - o_re), np.abs(dev_im - o_im)) / ulp
        worst_x, worst_o = max(worst_x, float(ex.max())), max(worst_o, float(eo.max()))
    assert worst_x <= 2.5, worst_x          # vs the exact formula
    assert worst_o <= 8.0, worst_o          # vs the oracle's float64 libm formula
    for z, tol in ((g64.reshape(-1), 0.004), (g32.reshape(-1).astype(np.float64), 0.004)):
        assert np.all(np.isfinite(z))
        assert abs(z.mean()) < tol and abs(z.var() - 1.0) < 2 * tol
        assert abs(np.mean(z ** 3)) < 3 * tol and abs(np.mean(z ** 4) - 3.0) < 10 * tol
        for k, p in ((2.0, 4.5500e-2), (3.0, 2.6998e-3), (4.0, 6.334e-5)):
            assert abs(np.mean(np.abs(z) > k) - p) < 5 * np.sqrt(p / z.size) + 1e-6, k
    assert np.max(np.abs(g64)) < np.sqrt(-2 * np.log(0.5 * 2.0 ** -32)) + 1e-12
    # float32 normals: the same outputs on a 24-bit uniform grid (u01), so they
    # track the float64 ones away from the smallest uniforms
    close = np.abs(g32.astype(np.float64) - g64) < 1e-3
    assert close.mean() > 0.999


def _bench_ids():
    """Frame ids from both ends of 65 536-frame bench steps (step 0 and step 19,
    rank 0), every SNR of the grid at the low end and the waterfall (16-22 dB)
    at both."""
    lo = np.arange(16)
    hi = F - 16 + np.array([8, 9, 10, 11, 15])
    top = 19 * F + np.array([8, 9, 10, 11]) + 16 * 7
    return np.concatenate([lo, hi, top, 19 * F + F - 16 + np.array([8, 9, 10, 11])]).astype(np.uint64)


@pytest.mark.parametrize('velocity', [0.0, 3.0])
def test_bench_frames_match_oracle(C, velocity):
    import lte_phy
    from oracle import lte_oracle as O
    O.lib()
    sim = lte_phy.OFDMSimulator(lte_phy.LTEConfig(bandwidth=20.0, modulation='64-QAM'),
                                channel_type='rayleigh_mp', itu_profile='Pedestrian_A', velocity_kmh=velocity,
                                precision='f64')
    ids = _bench_ids()
    S = len(P.BENCH_SNRS)
    si = (ids % np.uint64(S)).astype(np.int32)
    plan = sim._plan(C.CHAIN_CODED, 0, TB, max_frames=len(ids))
    out = plan.run(P.BENCH_SNRS[si], snr_index=si, n_snr=S, seed=P.BENCH_SEED, frame_ids=ids)
    fD = O.doppler_hz(2.0, velocity) if velocity else 0.0
    ref = [P.config2_frame(int(f), fD=fD) for f in ids]
    got = list(zip(out['frame_errors'].tolist(), out['crc_ok'].astype(bool).tolist()))
    assert got == ref
    # the sample covers failures, partial decodes and clean frames
    errs = np.array([r[0] for r in ref])
    assert np.any(errs == 0) and np.any(errs > 1000)


def _config_plan(config, n):
    import lte_phy
    from lte_phy import _capi as C
    Cfg, Sim = lte_phy.LTEConfig, lte_phy.OFDMSimulator
    if config == 3:
        s = Sim(Cfg(bandwidth=10.0, modulation='16-QAM'), channel_type='rayleigh_mp', itu_profile='Vehicular_A')
        return s._plan(C.CHAIN_SIMO, 14, 14 * 499 * 4, num_rx=4, max_frames=n)
    if config == 4:
        s = Sim(Cfg(bandwidth=20.0, modulation='64-QAM'), channel_type='rayleigh_mp', itu_profile='Pedestrian_A')
        return s._sfbc_plan(0, TB, 2, coded=True, max_frames=n)
    from lte_phy.ofdm_core import _spatial_plan
    return _spatial_plan(Cfg(bandwidth=20.0, modulation='64-QAM'), 'awgn', 'Pedestrian_A', 3.0, 2.0, 14,
                         14 * 999 * 6, n)[0]


def test_config4_unmerged_link_noise_matches_oracle(C, monkeypatch):
    """Config 4 with the link noise drawn on its own links' streams
    (LTE_SFBC_LINK_MERGE=0: k_link_noise_pairs, the RX power measured after it)
    against the oracle's 'combined_link_noise' composition: identical per-frame
    bit errors and CRC verdicts.  (The default merged form is
    test_other_config_bench_frames_match_oracle[4].)"""
    monkeypatch.setenv('LTE_SFBC_LINK_MERGE', '0')
    from lte_phy import engine
    engine.clear_cache()
    from oracle import lte_oracle as O, mimo_oracle as M
    ids = np.array([0, 1, 2, 5, 7, 9, 11, 13], dtype=np.uint64)
    S = len(P.BENCH_SNRS)
    si = (ids % np.uint64(S)).astype(np.int32)
    plan = _config_plan(4, len(ids))
    out = plan.run(P.BENCH_SNRS[si], snr_index=si, n_snr=S, seed=P.BENCH_SEED, frame_ids=ids)
    num = O.Numerology(bandwidth=20.0, modulation='64-QAM')
    L = 14 * (num.N + num.cp)
    ref = []
    for f in ids:
        r = M.simulate_sfbc_coded(num, P.payload_bits(P.BENCH_SEED, int(f), P.BENCH_TB), P.bench_snr(int(f)), 2,
                                  'rayleigh_mp', draws=P.sfbc_draws(P.BENCH_SEED, int(f), L, 2, 4, merged=False))
        ref.append((int(r['bit_errors']), bool(r['crc_pass'])))
    engine.clear_cache()
    assert out['frame_errors'].tolist() == [r[0] for r in ref]
    assert out['crc_ok'].astype(bool).tolist() == [r[1] for r in ref]


def test_config4_merged_link_noise_same_distribution(C, monkeypatch):
    """The merged link noise (default) and the separate draws
    (LTE_SFBC_LINK_MERGE=0) are different realisations of the same
    distribution: over 2 048 config-4 frames at 8 / 10 / 12 dB (the BER cliff)
    the bit-error totals agree within 4 binomial-frame standard deviations,
    and the noise variance per RX differs only by the link term 2 s2
    (~1e-10 of the signal power)."""
    from lte_phy import engine
    snrs = np.repeat([8.0, 10.0, 12.0], 683)[:2048]
    res = {}
    for merge in ('1', '0'):
        monkeypatch.setenv('LTE_SFBC_LINK_MERGE', merge)
        engine.clear_cache()
        plan = _config_plan(4, len(snrs))
        out = plan.run(snrs, seed=91, frame_id0=10_000)
        res[merge] = out['frame_errors'].astype(np.float64)
    engine.clear_cache()
    for k in range(3):
        sl = slice(683 * k, min(683 * (k + 1), 2048))
        a, b = res['1'][sl], res['0'][sl]
        sd = np.sqrt((a.var() + b.var()) / len(a))
        assert abs(a.mean() - b.mean()) <= 4 * sd + 1e-9, (k, a.mean(), b.mean(), sd)


@pytest.mark.parametrize('config', [3, 4, 5])
def test_other_config_bench_frames_match_oracle(C, config):
    """bench.py --config 3 / 4 / 5 frames (both ends of the first step at the
    configs' default batches) through the float64 GPU chains and the oracle's
    compositions on the oracle's Philox draws (SIMO MRC, SFBC 2x2 + turbo, 4x4
    MMSE on flat CN(0,1) links): identical per-frame bit errors (and CRC)."""
    F_c = {3: 65536, 4: 65536, 5: 32768}[config]
    ids = np.concatenate([np.arange(12), F_c - 16 + np.array([8, 10, 12, 15])]).astype(np.uint64)
    S = len(P.BENCH_SNRS)
    si = (ids % np.uint64(S)).astype(np.int32)
    plan = _config_plan(config, len(ids))
    out = plan.run(P.BENCH_SNRS[si], snr_index=si, n_snr=S, seed=P.BENCH_SEED, frame_ids=ids)
    ref = [P.BENCH_FRAMES[config](int(f)) for f in ids]
    assert out['frame_errors'].tolist() == [r[0] for r in ref]
    if config == 4:
        assert out['crc_ok'].astype(bool).tolist() == [r[1] for r in ref]
    errs = np.array([r[0] for r in ref])
    assert np.any(errs > 100) and np.any(errs < 100)
