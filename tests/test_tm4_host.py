"""CPU: the product's TM4 host classes (lte_phy/tm4.py: LTECodebook,
RankAdaptation, LayerMapper, MIMODetector argument checks) against vectors from
running the reference (tests/golden/golden_tm4.npz).  These are control logic
on one small matrix per call; they must reproduce the reference's decisions
exactly (the detectors themselves run on the GPU: tests/test_gpu_tm4.py)."""
import numpy as np
import pytest


def test_codebooks_match_reference(golden_tm4):
    from lte_phy.tm4 import LTECodebook
    g = golden_tm4
    for ntx in (2, 4, 8):
        assert np.array_equal(np.array(LTECodebook(ntx, 'TM6', 1).get_codebook()), g[f'cb_tm6_{ntx}'])
        for rank in range(1, min(ntx, 4) + 1):
            if ntx == 2 and rank > 2:
                with pytest.raises(ValueError):
                    LTECodebook(ntx, 'TM4', rank)
                continue
            cb = LTECodebook(ntx, transmission_mode='TM4', rank=rank)
            assert np.array_equal(np.array(cb.get_codebook()), g[f'cb_tm4_{ntx}_r{rank}']), (ntx, rank)
            pmi, v = cb.select_best_pmi(g[f'cb_tm4_{ntx}_r{rank}_selH'])
            assert [pmi, v] == list(g[f'cb_tm4_{ntx}_r{rank}_sel'])
            with pytest.raises(ValueError):
                cb.get_precoder(cb.codebook_size)
    with pytest.raises(ValueError):
        LTECodebook(4, 'TM6', 2)


def test_rank_adaptation_matches_reference(golden_tm4):
    from lte_phy.tm4 import RankAdaptation
    g = golden_tm4
    for i in range(int(g['ra_n'][0])):
        ntx, nrx, snr = g[f'ra{i}_cfg']
        ra = RankAdaptation(int(ntx), int(nrx), snr_db=snr)
        fb = ra.get_feedback(g[f'ra{i}_H'])
        ri_cap = ra.calculate_optimal_rank(g[f'ra{i}_H'], method='capacity')
        pmi_f, _ = ra.select_precoder_for_rank(g[f'ra{i}_H'], fb['ri'], metric='frobenius')
        assert [fb['ri'], fb['pmi'], ri_cap, pmi_f] == list(g[f'ra{i}_out']), i
        assert np.array_equal(fb['W'], g[f'ra{i}_W'])
        assert np.array_equal(fb['eigenvalues'], g[f'ra{i}_eig'])
        assert fb['condition_number'] == g[f'ra{i}_cond'][0]


@pytest.mark.parametrize('rank', [1, 2, 3])
def test_layer_mapper_matches_reference(golden_tm4, rank):
    from lte_phy.tm4 import LayerMapper
    g = golden_tm4
    lm = LayerMapper(rank)
    lay = lm.map_to_layers(g[f'lm{rank}_in'])
    assert np.array_equal(lay, g[f'lm{rank}_map'])
    assert np.array_equal(lm.demap_from_layers(lay, original_length=62), g[f'lm{rank}_demap'])
    assert lm.get_padded_length(62) == lay.size
    with pytest.raises(ValueError):
        LayerMapper(9)


def test_detector_argument_errors():
    from lte_phy.tm4 import MIMODetector
    with pytest.raises(ValueError):
        MIMODetector(1, 2)                         # num_rx < num_layers (core/mimo_detector.py:34-35)
    import lte_phy
    with pytest.raises(ValueError):
        lte_phy.simulate_spatial_multiplexing(np.array([], dtype=int))
