"""CPU: the product's beamforming host classes (lte_phy/beamforming.py:
BeamformingPrecoder, AdaptiveBeamforming, CSIFeedback) against the
reference's own outputs (tests/golden/golden_bf.npz).  Control logic on one
small matrix per call: exact equality."""
import numpy as np


def test_precoders_and_feedback_match_reference(golden_bf):
    from lte_phy.beamforming import BeamformingPrecoder, CSIFeedback
    g = golden_bf
    for i in range(int(g['p_n'][0])):
        ntx, nrx, tm4 = (int(v) for v in g[f'p{i}_cfg'])
        H = g[f'p{i}_H']
        bp = BeamformingPrecoder(ntx)
        wm = bp.update_precoder(H, method='MRT').copy()
        gm = bp.calculate_beamforming_gain(H)
        we = bp.update_precoder(H, method='eigen').copy()
        ge = bp.calculate_beamforming_gain(H)
        assert np.array_equal(wm, g[f'p{i}_wmrt']) and np.array_equal(we, g[f'p{i}_weig'])
        assert [gm, ge] == list(g[f'p{i}_gain'])
        assert np.array_equal(bp.apply_precoding(g[f'p{i}_s'], wm), g[f'p{i}_x'])
        fb = CSIFeedback(ntx, nrx, codebook_type='TM4' if tm4 else 'TM6').generate_feedback(H, noise_variance=0.3)
        assert [fb['pmi'], fb['cqi'], fb['ri'], fb['sinr_db']] == list(g[f'p{i}_fb']), i
        assert np.array_equal(fb['precoder'], g[f'p{i}_fbW'])


def test_adaptive_update_period(golden_bf):
    from lte_phy.beamforming import AdaptiveBeamforming
    per = [AdaptiveBeamforming(4, v, 2.0).update_period for v in (0.0, 3.0, 30.0, 120.0, 500.0)]
    assert per == list(golden_bf['update_period'])
    ab = AdaptiveBeamforming(2, 3.0, 2.0)
    H = golden_bf['p3_H'][:, :2] if golden_bf['p3_H'].shape[1] >= 2 else golden_bf['p0_H']
    x = ab.process_symbol(np.ones(4, dtype=complex), H)
    assert x.shape == (2, 4) and ab.symbols_since_update == 1
