"""CPU: the TM4 oracle (oracle/tm4_oracle.py) against
vectors from running the reference (tests/golden/make_golden_tm4.py):
LTE codebooks, PMI selection, rank adaptation, the MMSE / IRC / ZF / SIC /
MRC detectors, layer mapping for ranks 1-3 and simulate_spatial_multiplexing
end to end for 2 / 4 TX, 1-4 RX, fixed and adaptive rank.  Exact equality
unless stated."""
import numpy as np
import pytest

from conftest import unpack

MODS = {2: 'QPSK', 4: '16-QAM', 6: '64-QAM'}


def _name(a):
    return bytes(np.asarray(a, dtype=np.uint8)).decode().strip()


def test_codebooks(golden_tm4, tm4_oracle):
    g = golden_tm4
    for ntx in (2, 4, 8):
        assert np.array_equal(np.array(tm4_oracle.codebook(ntx, 'TM6', 1)), g[f'cb_tm6_{ntx}'])
        for rank in range(1, min(ntx, 4) + 1):
            if ntx == 2 and rank > 2:
                with pytest.raises(ValueError):
                    tm4_oracle.codebook(ntx, 'TM4', rank)
                continue
            cb = tm4_oracle.codebook(ntx, 'TM4', rank)
            assert np.array_equal(np.array(cb), g[f'cb_tm4_{ntx}_r{rank}']), (ntx, rank)
            pmi, v = tm4_oracle.select_best_pmi(cb, g[f'cb_tm4_{ntx}_r{rank}_selH'])
            assert [pmi, v] == list(g[f'cb_tm4_{ntx}_r{rank}_sel'])
    with pytest.raises(ValueError):
        tm4_oracle.codebook(2, 'TM6', 2)


def test_rank_adaptation(golden_tm4, tm4_oracle):
    g = golden_tm4
    for i in range(int(g['ra_n'][0])):
        ntx, nrx, snr = g[f'ra{i}_cfg']
        ntx, nrx = int(ntx), int(nrx)
        H = g[f'ra{i}_H']
        fb = tm4_oracle.feedback(H, ntx, nrx, snr)
        ri_cap = tm4_oracle.optimal_rank(H, ntx, nrx, snr, 'capacity')
        pmi_f, _ = tm4_oracle.precoder_for_rank(H, ntx, nrx, snr, fb['ri'], 'frobenius')
        assert [fb['ri'], fb['pmi'], ri_cap, pmi_f] == list(g[f'ra{i}_out']), i
        assert np.array_equal(fb['W'], g[f'ra{i}_W'])
        assert np.array_equal(fb['eigenvalues'], g[f'ra{i}_eig'])
        assert fb['condition_number'] == g[f'ra{i}_cond'][0]


def test_detectors(golden_tm4, tm4_oracle, oracle):
    g = golden_tm4
    for i in range(int(g['det_n'][0])):
        ntx, nrx, rank, bps, pmi = (int(v) for v in g[f'det{i}_cfg'])
        const = oracle.constellation(MODS[bps]) if bps else None
        out = tm4_oracle.detect(_name(g[f'det{i}_name']), g[f'det{i}_y'], g[f'det{i}_H'], g[f'det{i}_s2'][0],
                                g[f'det{i}_W'], rank, const)
        assert np.array_equal(out, g[f'det{i}_out']), (i, np.max(np.abs(out - g[f'det{i}_out'])))
    assert g['det_err_rx_lt_layers'][0] == 1
    with pytest.raises(ValueError):
        tm4_oracle.detect('MMSE', np.zeros((1, 4)), np.zeros((1, 2, 4)), 0.1, np.eye(2), 2)


@pytest.mark.parametrize('rank', [1, 2, 3])
def test_layer_mapping(golden_tm4, mimo_oracle, rank):
    g = golden_tm4
    lay = mimo_oracle.layer_map(g[f'lm{rank}_in'], rank)
    assert np.array_equal(lay, g[f'lm{rank}_map'])
    assert np.array_equal(mimo_oracle.layer_demap(lay, original_length=62), g[f'lm{rank}_demap'])


def _e2e_names(g):
    return bytes(g['e2e_names']).decode().split(',')


@pytest.mark.parametrize('name', ['e_zf22', 'e_mmse42ad', 'e_sic44r2', 'e_mrc22r1', 'e_sic44ad', 'e_mmse43r3',
                                  'e_mmse41ad', 'e_zf22low', 'e_mmse24nocsi', 'e_sic44c5', 'e_zf22c20'])
def test_simulate_spatial_e2e(golden_tm4, oracle, tm4_oracle, name):
    g = golden_tm4
    assert name in _e2e_names(g)
    bw, bps, ray, snr, ntx, nrx, rank, csi = g[f'{name}_cfg']
    num = oracle.Numerology(bandwidth=float(bw), modulation=MODS[int(bps)])
    n = int(g[f'{name}_nbits'][0])
    bits = unpack(g[f'{name}_bits'], n).astype(np.int64)
    np.random.seed(int(g[f'{name}_seed'][0]))
    r = tm4_oracle.simulate_tm4(num, bits, float(snr), int(ntx), int(nrx), 'adaptive' if rank < 0 else int(rank),
                                _name(g[f'{name}_det']), 'rayleigh_mp' if ray else 'awgn', csi=bool(csi))
    assert [r['rank'], r['pmi_used']] == list(g[f'{name}_rank_pmi'])
    assert np.array_equal(r['precoder_matrix'], g[f'{name}_W'])
    assert np.array_equal(r['channel_matrix'], g[f'{name}_H'])
    assert r['bit_errors'] == g[f'{name}_errors'][0]
    assert np.array_equal(r['bits_received_array'], unpack(g[f'{name}_rx'], n))
    assert np.array_equal(np.array(np.random.get_state()[1][:8], dtype=np.uint32), g[f'{name}_state'])
