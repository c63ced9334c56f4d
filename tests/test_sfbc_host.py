"""CPU: the SFBCAlamouti / SFBCResourceMapper drop-in (core/sfbc_alamouti.py)
without device compute: constructor and argument errors with the
reference's messages, the disabled pass-through, statistics, and the SFBC
grid mapping (index bookkeeping + native pilots + the global-RNG reseed)
against the reference's own output (golden_mimo 'sfbcmap_*')."""
import numpy as np
import pytest


def test_sfbc_class_surface():
    from lte_phy import SFBCAlamouti
    with pytest.raises(ValueError, match='exactly 2 TX antennas'):
        SFBCAlamouti(num_tx=4)
    al = SFBCAlamouti(num_tx=2, enabled=False)
    s = np.array([1 + 1j, 2, 3j])
    t0, t1 = al.encode(s)
    assert np.array_equal(t0, s) and np.array_equal(t1, s) and t0 is not s
    assert np.array_equal(al.decode(s, s, s), s)
    st = SFBCAlamouti().get_statistics()
    assert st == {'enabled': True, 'num_tx': 2, 'coding_scheme': 'Alamouti SFBC', 'rate': 1.0,
                  'diversity_order': 2}
    al = SFBCAlamouti()
    with pytest.raises(ValueError, match='must be even, got 3'):
        al.decode(np.ones(3, complex), np.ones(3, complex), np.ones(3, complex))
    with pytest.raises(ValueError, match='must have length 4'):
        al.decode(np.ones(4, complex), np.ones(3, complex), np.ones(4, complex))


def test_sfbc_resource_mapper_matches_reference(golden_mimo):
    import lte_phy
    from lte_phy.sfbc_alamouti import SFBCResourceMapper
    sm = SFBCResourceMapper(lte_phy.LTEConfig(bandwidth=20.0, modulation='64-QAM'))
    assert np.array_equal(sm.data_indices, golden_mimo['sfbcmap_data_idx'])
    assert sm.num_data == 998
    np.random.seed(99)
    g0, g1 = sm.map_sfbc_to_grid(golden_mimo['sfbc_tx0'], golden_mimo['sfbc_tx1'])
    assert np.array_equal(g0, golden_mimo['sfbcmap_grid0'])
    assert np.array_equal(g1, golden_mimo['sfbcmap_grid1'])
    assert np.array_equal(np.array(np.random.get_state()[1][:8], dtype=np.uint32), golden_mimo['sfbcmap_state'])
    assert np.array_equal(sm.extract_data_from_grid(g0), golden_mimo['sfbc_tx0'])
    assert len(sm.prepare_data_for_sfbc(np.ones(10))) == 998
    W = np.array([[1], [1j]]) / np.sqrt(2)
    tx = sm.apply_generic_precoding(golden_mimo['sfbc_sym'], W)
    assert len(tx) == 2 and np.array_equal(tx[1], np.zeros(998, complex) + W[1, 0] * golden_mimo['sfbc_sym'])
