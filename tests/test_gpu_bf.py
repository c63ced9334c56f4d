"""GPU parity of beamforming (simulate_beamforming,
LTE_CHAIN_BEAMFORMING) against the reference's own outputs
(tests/golden/golden_bf.npz, seeded global RNG).

Bars, float64 (the default, the reference's complex128): PMI history, channel
matrix and global-RNG state identical; received bits and bit errors identical
to the reference's; equalised symbols vs the oracle (same random numbers)
within 1e-12 relative; gain within 1e-9 dB.  float32 fast mode: the same
PMI / channel / RNG state, gain within 1e-4 dB (float64 setup from the float32
channel), received bits within the north_star 1e-3 BER bar, symbols within 1e-5."""
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


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('name', ['bf_21a', 'bf_42s', 'bf_81a', 'bf_24s', 'bf_44a'])
def test_simulate_beamforming_ref_compat(C, golden_bf, oracle, bf_oracle, name, prec):
    import lte_phy
    g = golden_bf
    bw, bps, snr, ntx, nrx, tm4, adaptive, v, seed = g[f'{name}_cfg']
    mod = MODS[int(bps)]
    n = int(g[f'{name}_nbits'][0])
    bits = unpack(g[f'{name}_bits'], n).astype(np.int64)
    sim = lte_phy.OFDMSimulator(lte_phy.LTEConfig(bandwidth=float(bw), modulation=mod), precision=prec)
    np.random.seed(int(seed))
    r = sim.simulate_beamforming(bits, snr_db=float(snr), num_tx=int(ntx), num_rx=int(nrx),
                                 codebook_type='TM4' if tm4 else 'TM6', velocity_kmh=float(v),
                                 update_mode='adaptive' if adaptive else 'static')
    assert np.array_equal(np.array(np.random.get_state()[1][:8], dtype=np.uint32), g[f'{name}_state'])
    assert np.array_equal(r['channel_matrix'], g[f'{name}_H'])
    assert np.array_equal(np.array(r['pmi_history']), g[f'{name}_pmi'])
    f64 = prec == 'f64'
    assert abs(r['beamforming_gain_db'] - g[f'{name}_gain'][0]) < (1e-9 if f64 else 1e-4)
    ref = unpack(g[f'{name}_rx'], n)
    if f64:
        assert np.array_equal(r['bits_received_array'], ref)
        assert r['bit_errors'] == int(g[f'{name}_errors'][0])
    else:
        assert np.mean(r['bits_received_array'] != ref) < 1e-3
        assert abs(r['bit_errors'] - int(g[f'{name}_errors'][0])) / n < 1e-3
    # symbols vs the oracle on the same random numbers
    np.random.seed(int(seed))
    o = bf_oracle.simulate_beamforming(oracle.Numerology(bandwidth=float(bw), modulation=mod), bits, float(snr),
                                       int(ntx), int(nrx), 'TM4' if tm4 else 'TM6',
                                       'adaptive' if adaptive else 'static')
    a, b = r['symbols_rx'], o['symbols_rx']
    assert np.linalg.norm(a - b) / np.linalg.norm(b) < (1e-12 if f64 else 1e-5)


@pytest.mark.parametrize('prec', ['f64', 'f32'])
@pytest.mark.parametrize('bfo', [dict(num_tx=4, num_rx=1, update_mode='adaptive'),
                                 dict(num_tx=8, num_rx=2, update_mode='static'),
                                 dict(num_tx=2, num_rx=4, update_mode='adaptive')])
def test_run_grid_beamforming_sharding_invariant(C, bfo, prec):
    import lte_phy
    sim = lte_phy.OFDMSimulator(lte_phy.LTEConfig(bandwidth=5.0, modulation='16-QAM'), precision=prec)
    snrs = [0.0, 10.0, 25.0]
    full = sim.run_grid(snrs, 6, seed=2, mimo='beamforming', beamforming=bfo, frames_per_call=8)
    parts = [sim.run_grid(snrs, 6, seed=2, mimo='beamforming', beamforming=bfo, frames_per_call=8, rank=r,
                          world_size=2) for r in range(2)]
    assert np.array_equal(full['counts'], parts[0]['counts'] + parts[1]['counts'])
    assert full['ber'][0] > full['ber'][1] >= full['ber'][2]


def test_beamforming_argument_errors(C):
    import lte_phy
    sim = lte_phy.OFDMSimulator(lte_phy.LTEConfig(bandwidth=1.25, modulation='QPSK'))
    with pytest.raises(ValueError):
        sim.simulate_beamforming(np.array([], dtype=int))
    with pytest.raises(ValueError):
        sim.simulate_beamforming(np.ones(100, dtype=int), num_tx=3)
    with pytest.raises(ValueError):
        sim.simulate_beamforming(np.ones(100, dtype=int), codebook_type='TM9')
