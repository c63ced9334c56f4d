"""The bench's per-stage rooflines are reproducible from profiles/: for every
stage of configs 2-5 whose kernels the committed rocprofv3 --pmc summary
lists, the algorithmic bytes bench.py prices (stage_bytes_per_frame, the
kernels the default path launches) are at most the measured HBM bytes of
those kernels (+5 % for the counters' gfx950 corrections), and the rate they
imply at the kernels' measured time is below the 8 TB/s peak.  A gpu test
checks that the dry-run geometry the CPU side prices equals what the real
bench plans report."""
import importlib.util
import os
import types

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location('bench_mod', os.path.join(ROOT, 'bench.py'))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    return b


@pytest.mark.parametrize('config', [2, 3, 4, 5])
def test_stage_bytes_within_pmc_traffic(config):
    b = _bench()
    pmc = b.load_profile(b.PMC_FILES[config])
    assert pmc, b.PMC_FILES[config]
    geom = types.SimpleNamespace(**b.DRY_GEOM[config])
    sb = b.stage_bytes_per_frame(config, geom, 'f64')
    checked = 0
    for stage, (kernels, alg, what) in sb.items():
        tr = b.pmc_stage_bytes(pmc, kernels)
        if tr is None:        # the summary does not list this (tiny) kernel
            continue
        assert alg <= 1.05 * tr, (stage, kernels, alg, tr)
        ms = 0.0
        for k in kernels:
            hits = [v for n, v in pmc['kernels'].items() if n == k or n.startswith(k + '<')]
            ms += max(hits, key=lambda v: v.get('ms', 0))['ms'] if hits else 0.0
        gbs = alg * pmc['frames'] / (ms * 1e-3) / 1e9
        assert gbs <= b.HBM_PEAK_GBS, (stage, gbs)
        checked += 1
    # every stage that moves the signal is covered by the summary (config 4's
    # 'channel' is the merged link noise's noise-power kernels since round 6)
    assert checked >= {2: 5, 3: 4, 4: 4, 5: 3}[config], checked


def test_config5_prices_the_pilot_estimate_handoff():
    """Config 5 (spatial, no H capture): the receiver hands the detector LS
    pilot estimates (4 RX x 14 x 4 TX x 50 pilots), not the interpolated H,
    and reads the RX streams without their CP: 2 238 208 B per frame, the
    PMC-measured bytes of the float64 receiver (the wave-private
    k_rx_fft_mimo_w by default, round 6; k_rx_fft_mimo in round 5) to 0.2 %."""
    b = _bench()
    geom = types.SimpleNamespace(**b.DRY_GEOM[5])
    sb = b.stage_bytes_per_frame(5, geom, 'f64')
    c = 16
    assert sb['rx_chest'][1] == 4 * 14 * 2048 * c + 14 * 4 * 250 * c + 4 * 14 * 4 * 50 * c == 2238208
    assert sb['rx_chest'][0] == ['k_rx_fft_mimo_w']
    pmc = b.load_profile(b.PMC_FILES[5])
    assert abs(sb['rx_chest'][1] / b.pmc_stage_bytes(pmc, ['k_rx_fft_mimo_w']) - 1) < 2e-3
    r5 = b.load_profile('r5_pmc_c5_hp.json')
    assert abs(sb['rx_chest'][1] / b.pmc_stage_bytes(r5, ['k_rx_fft_mimo']) - 1) < 1e-3
    # flat links: TX + links are one kernel; the channel timer is the noise power only
    assert sb['ofdm_tx'][0] == ['k_ofdm_txch_flat'] and sb['channel'][0] == ['k_npow_mimo']


def test_turbo_roofline_bound_is_the_measured_limiter():
    b = _bench()
    F = 65536
    tim = {'turbo': (5 * 322.6, 5)}
    r = b.turbo_roofline('f64', tim, F)
    assert r['bound'] == r['measured_limiter'] == 'hbm'
    assert r['unit'] == 'GB/s' and r['peak'] == 8000.0
    assert abs(r['frac'] - r['hbm_row_stream']['frac_row_stream']) < 1e-9
    assert 0.6 < r['frac'] < 0.7 and 0.7 < r['hbm_frac'] < 0.75 and 0.2 < r['valu_frac'] < 0.3
    assert r['valu']['frac'] == r['valu_frac'] and r['valu']['unit'] == 'Top/s'
    share = r['hbm_row_stream']['store_cost']['store_share_of_bytes']
    assert share == round(b.shape_store_share(), 4) and 0.15 < share < 0.2


@pytest.mark.gpu
@pytest.mark.parametrize('config', [2, 3, 4, 5])
def test_dry_geometry_matches_bench_plans(config):
    b = _bench()
    args = types.SimpleNamespace(frames=64, precision='f64', velocity=0.0, iters=8, channel=None)
    plan = b.make_plan(config, args)
    for k, v in b.DRY_GEOM[config].items():
        assert getattr(plan, k) == v, (config, k, getattr(plan, k), v)
