"""GPU: the device-backed names of the core.channel_coding drop-in against the
reference's own outputs (golden.npz round 1, golden_coding_r2.npz round 2):
CRC-24B, segmentation with CRC-24B, LogMAPDecoder (max-log exact; log-MAP to
libm round-off), exact log-MAP turbo_decode, rate_dematching_turbo with
puncturing and repetition."""
import numpy as np
import pytest

from conftest import unpack

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def cc():
    from lte_phy import _capi, channel_coding
    _capi.device_init()
    return channel_coding


@pytest.mark.parametrize('vec', ['zeros40', 'ones40', 'alt40', 'rand27760'])
def test_crc24b(cc, golden, vec):
    v = golden[f'crc_{vec}_in']
    crc = cc.calculate_crc24b(v)
    assert np.array_equal(crc, golden[f'crc_{vec}_24b'])
    w = cc.attach_crc24b(v)
    assert cc.check_crc24b(w) and cc.check_crc24a(cc.attach_crc24a(v))
    w[0] ^= 1
    assert not cc.check_crc24b(w)
    assert not cc.check_crc24b(np.zeros(10, dtype=np.uint8))


@pytest.mark.parametrize('B', [6145, 9232, 27784])
def test_segmentation_with_crc24b(cc, golden_coding, B):
    g, meta = golden_coding
    blocks, md = cc.segment_code_blocks(g[f'seg{B}_tb'])
    assert md == meta[f'seg{B}']
    assert np.array_equal(np.concatenate(blocks), g[f'seg{B}_blocks'])
    assert all(cc.check_crc24b(b) for b in blocks)
    assert np.array_equal(cc.desegment_code_blocks(blocks, md), g[f'seg{B}_back'])


def test_log_map_decoder_max_log_exact(cc, golden_coding):
    """LogMAPDecoder.decode (max-log, the default): bit-identical extrinsic and
    a-posteriori LLRs and decisions."""
    g, _ = golden_coding
    d = cc.LogMAPDecoder()
    b, ext = d.decode(g['lmd_ls'], g['lmd_lp'], g['lmd_la'], return_extrinsic=True)
    _, app = d.decode(g['lmd_ls'], g['lmd_lp'], g['lmd_la'], return_extrinsic=False)
    assert np.array_equal(b, g['lmd_maxlog_bits'])
    assert np.array_equal(ext, g['lmd_maxlog_ext'])
    assert np.array_equal(app, g['lmd_maxlog_app'])
    assert d.next_state.tolist() == [[0, 4], [4, 0], [5, 1], [1, 5], [2, 6], [6, 2], [7, 3], [3, 7]]


def test_exact_log_map_mode(cc, golden_coding, golden):
    """set_decoder_mode(False): exact log-MAP max* (log_sum_exp) on the GPU in
    float64.  LLRs agree with the reference to libm round-off (the GPU's and
    NumPy's exp / log1p differ in the last ulp), decisions exactly -- for the
    LogMAPDecoder pass and for full turbo decodes."""
    g, _ = golden_coding
    try:
        cc.set_decoder_mode(False)
        d = cc.LogMAPDecoder()
        b, ext = d.decode(g['lmd_ls'], g['lmd_lp'], g['lmd_la'], return_extrinsic=True)
        _, app = d.decode(g['lmd_ls'], g['lmd_lp'], g['lmd_la'], return_extrinsic=False)
        assert np.array_equal(b, g['lmd_logmap_bits'])
        assert np.max(np.abs(app - g['lmd_logmap_app'])) < 1e-9 * (1 + np.max(np.abs(g['lmd_logmap_app'])))
        assert np.max(np.abs(ext - g['lmd_logmap_ext'])) < 1e-9 * (1 + np.max(np.abs(g['lmd_logmap_ext'])))
        assert not np.array_equal(app, g['lmd_maxlog_app'])      # the mode really changed the arithmetic
        for key, its in [('td_40_8', 8), ('td_1024_1', 1)]:
            K = int(key.split('_')[1])
            dec = cc.turbo_decode(golden[key + '_llr'], K, its)
            assert np.array_equal(dec, g[key + '_logmap_dec']), key
        with pytest.raises(NotImplementedError):                  # the f32 decoder is max-log only
            cc.turbo_decode(golden['td_40_8_llr'], 40, 8, precision='f32')
    finally:
        cc.set_decoder_mode(True)
    dec = cc.turbo_decode(golden['td_1024_8_llr'], 1024, 8)
    assert np.array_equal(dec, unpack(golden['td_1024_8_dec'], 1024))


@pytest.mark.parametrize('K', [40, 1024, 5568, 5632, 6144])
def test_rate_dematching_punct_and_repeat(cc, golden, K):
    """rate_dematching_turbo: E = 3K+12 (rv 0), E = K+17 (puncturing, rv 2) and
    E = 4K > N_cb (repetition: repeats summed, rv 2), bit-exact."""
    assert np.array_equal(cc.rate_dematching_turbo(golden[f'dm_{K}_in'], K, 0), golden[f'dm_{K}_out'])
    for E2 in [K + 17, 4 * K]:
        out = cc.rate_dematching_turbo(golden[f'dm_{K}_E{E2}_in'], K, 2)
        assert np.array_equal(out, golden[f'dm_{K}_E{E2}_out']), E2


@pytest.mark.parametrize('K', [40, 1024])
def test_rate_dematching_triple_repetition(cc, golden_coding, K):
    g, _ = golden_coding
    assert np.array_equal(cc.rate_dematching_turbo(g[f'dmrep{K}_in'], K, 1), g[f'dmrep{K}_out'])


@pytest.mark.parametrize('bw,mod,n_bits', [(20.0, '64-QAM', 6230), (5.0, '16-QAM', 1000)])
def test_exact_log_map_coded_chain(cc, bw, mod, n_bits):
    """set_decoder_mode(False) on a whole coded float64 plan (k_turbo64_logmap
    in the chain): 96 frames = two 64-frame decoder groups; a 6230-bit TB (two
    code blocks of different sizes, K = 3136 and 3200, in one launch) and a
    1000-bit TB (one code block).  The chain's decoded TB bits and CRC verdicts
    equal the host entry points in the same mode (rate_dematching_turbo +
    turbo_decode, both pinned to the reference's log-MAP goldens above) on the
    chain's own captured LLRs.  One turbo iteration: the exact log-MAP kernel
    (exp / log1p per max*) is far slower than the max-log hot path."""
    import lte_phy
    from lte_phy import _capi as C
    from oracle import lte_oracle as O
    sim = lte_phy.OFDMSimulator(lte_phy.LTEConfig(bandwidth=bw, modulation=mod), channel_type='rayleigh_mp',
                                precision='f64')
    its = 1
    try:
        cc.set_decoder_mode(False)
        plan = sim._plan(C.CHAIN_CODED, 0, n_bits, max_frames=96, iters=its)
        snrs = np.linspace(0.0, 30.0, 96)
        r = plan.run(snrs, seed=19, capture=('llr', 'bits_rx'))
        num = O.Numerology(bandwidth=bw, modulation=mod)
        bps, Nd = num.bps, num.Nd
        coded = plan.coded_bits
        ncs = coded // bps
        rows = -(-ncs // Nd)
        _, seg_plan = O.segment(O.attach_crc24a(np.zeros(n_bits, dtype=np.uint8)))
        assert len({p[0] for p in seg_plan}) == (2 if n_bits > 6120 else 1)
        q = np.arange(ncs)
        src_re = (q % Nd) * rows + q // Nd
        L = np.stack([r['llr'][b].reshape(-1, bps)[src_re].reshape(-1)[:coded] for b in range(len(snrs))])
        off, blocks = 0, []
        for (K, F, info, o, crc) in seg_plan:   # every frame's code block r in one batched host decode
            E = 3 * K + 12
            dm = np.stack([cc.rate_dematching_turbo(L[b, off:off + E], K, 0) for b in range(len(snrs))])
            off += E
            blocks.append(cc.turbo_decode_batch(dm, K, its))
        n_ok = 0
        for b in range(len(snrs)):
            tbc = O.desegment([blk[b] for blk in blocks], seg_plan)
            ok = O.check_crc24a(tbc)
            assert np.array_equal(tbc[:-24], r['bits_rx'][b]) and bool(ok) == bool(r['crc_ok'][b]), b
            n_ok += int(ok)
        assert 4 <= n_ok < len(snrs)   # decoded and failed frames both covered
    finally:
        cc.set_decoder_mode(True)
