"""GPU parity of TM4 spatial multiplexing beyond 4x4 / rank 4 / PMI 0 (SURVEY
§8(f) rank 1) against the reference's own outputs (tests/golden/
golden_tm4.npz, frozen global RNG).

Bars: MMSE / IRC / ZF / MRC detector outputs (float64 on the device, Cholesky
vs the reference's LAPACK inverse / pinv) within 1e-9 relative; SIC outputs
(constellation points) identical; end to end: rank, PMI, W, channel matrix and
global-RNG state identical, received bits within the north_star 1e-3 BER bar."""
import numpy as np
import pytest

from conftest import unpack

pytestmark = pytest.mark.gpu

MODS = {2: 'QPSK', 4: '16-QAM', 6: '64-QAM'}


@pytest.fixture(scope='module')
def C():
    from lte_phy import _capi
    _capi.device_init(0)
    return _capi


def _name(a):
    return bytes(np.asarray(a, dtype=np.uint8)).decode().strip()


def test_detectors_vs_reference(C, golden_tm4, oracle):
    from lte_phy.tm4 import MIMODetector
    g = golden_tm4
    for i in range(int(g['det_n'][0])):
        ntx, nrx, rank, bps, pmi = (int(v) for v in g[f'det{i}_cfg'])
        det = _name(g[f'det{i}_name'])
        const = oracle.constellation(MODS[bps]) if bps else None
        out = MIMODetector(nrx, rank, detector_type=det, constellation=const).detect(
            g[f'det{i}_y'], g[f'det{i}_H'], g[f'det{i}_s2'][0], W_precoder=g[f'det{i}_W'])
        ref = g[f'det{i}_out']
        assert out.shape == ref.shape
        if det == 'SIC' and bps:
            assert np.array_equal(out, ref), (i, int(np.sum(out != ref)))
        else:
            err = np.max(np.abs(out - ref)) / np.max(np.abs(ref))
            assert err < 1e-9, (i, det, err)


def test_single_point_detect(C, golden_tm4):
    """detect() on one subcarrier (y 1-D) takes the _detect_single path."""
    from lte_phy.tm4 import MIMODetector
    g = golden_tm4
    y, H, W, s2 = g['det0_y'][:, 5], g['det0_H'][:, :, 5], g['det0_W'], g['det0_s2'][0]
    out = MIMODetector(4, 4, 'MMSE').detect(y, H, s2, W_precoder=W)
    assert out.shape == (4,)
    assert np.max(np.abs(out - g['det0_out'][:, 5])) < 1e-9 * np.max(np.abs(g['det0_out'][:, 5]))


E2E = ['e_zf22', 'e_mmse42ad', 'e_sic44r2', 'e_mrc22r1', 'e_sic44ad', 'e_mmse43r3', 'e_mmse41ad', 'e_zf22low',
       'e_mmse24nocsi', 'e_sic44c5', 'e_zf22c20']


@pytest.mark.parametrize('name', E2E)
def test_simulate_spatial_ref_compat(C, golden_tm4, name):
    import lte_phy
    g = golden_tm4
    bw, bps, ray, snr, ntx, nrx, rank, csi = g[f'{name}_cfg']
    mod = MODS[int(bps)]
    n = int(g[f'{name}_nbits'][0])
    bits = unpack(g[f'{name}_bits'], n).astype(np.int64)
    np.random.seed(int(g[f'{name}_seed'][0]))
    r = lte_phy.simulate_spatial_multiplexing(
        bits, num_tx=int(ntx), num_rx=int(nrx), rank='adaptive' if rank < 0 else int(rank),
        detector_type=_name(g[f'{name}_det']), modulation=mod, snr_db=float(snr),
        config=lte_phy.LTEConfig(bandwidth=float(bw), modulation=mod),
        channel_type='rayleigh_mp' if ray else 'awgn', itu_profile='Pedestrian_A', velocity_kmh=3,
        enable_csi_feedback=bool(csi))
    assert [r['rank'], r['pmi_used']] == list(g[f'{name}_rank_pmi'])
    assert np.array_equal(r['precoder_matrix'], g[f'{name}_W'])
    assert np.array_equal(r['channel_matrix'], g[f'{name}_H'])
    assert np.array_equal(np.array(np.random.get_state()[1][:8], dtype=np.uint32), g[f'{name}_state'])
    ref_rx = unpack(g[f'{name}_rx'], n)
    mism = int(np.sum(r['bits_received_array'] != ref_rx))
    ref_err = int(g[f'{name}_errors'][0])
    assert abs(r['bit_errors'] - ref_err) / n < 1e-3 or mism <= 1, (name, r['bit_errors'], ref_err, mism)
    assert mism / n < 1e-3 or mism <= 1, (name, mism)


@pytest.mark.parametrize('sp', [dict(num_tx=2, num_rx=2, rank=2, detector='ZF', pmi=1),
                                dict(num_tx=4, num_rx=4, rank=2, detector='SIC', pmi=5),
                                dict(num_tx=4, num_rx=2, rank=1, detector='MRC', pmi=3)])
def test_run_grid_spatial_variants_sharding_invariant(C, sp):
    """Philox grid over TM4 variants: per-shard counts sum to the unsharded
    counts; BER falls with SNR."""
    import lte_phy
    sim = lte_phy.OFDMSimulator(lte_phy.LTEConfig(bandwidth=5.0, modulation='16-QAM'), channel_type='awgn')
    snrs = [0.0, 10.0, 30.0]
    full = sim.run_grid(snrs, 6, seed=3, mimo='spatial', spatial=sp, frames_per_call=8)
    parts = [sim.run_grid(snrs, 6, seed=3, mimo='spatial', spatial=sp, frames_per_call=8, rank=r, world_size=2)
             for r in range(2)]
    assert np.array_equal(full['counts'], parts[0]['counts'] + parts[1]['counts'])
    ber = full['ber']
    assert ber[0] > ber[1] >= ber[2] and ber[0] > 0.01


def test_spatial_argument_errors(C):
    import lte_phy
    bits = np.ones(100, dtype=int)
    with pytest.raises(ValueError):     # MRC needs rank 1
        lte_phy.simulate_spatial_multiplexing(bits, num_tx=2, num_rx=2, rank=2, detector_type='MRC',
                                              enable_csi_feedback=False)
    with pytest.raises(ValueError):     # num_rx < rank
        lte_phy.simulate_spatial_multiplexing(bits, num_tx=4, num_rx=2, rank=3, enable_csi_feedback=False)
    with pytest.raises(ValueError):
        lte_phy.simulate_spatial_multiplexing(bits, num_tx=2, num_rx=2, rank=2, detector_type='ML')
