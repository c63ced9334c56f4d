"""CPU: the index-bookkeeping names of the core.channel_coding drop-in against
the reference's own outputs (tests/golden/make_golden_coding_r2.py): sub-block
(de)interleaver, QPP (de)interleave, single-block segmentation metadata,
get_segmentation_info and the drop-in's name list.  Their permutations come
from liblte_hip.so's native tables (host functions: no GPU needed)."""
import numpy as np
import pytest


def test_drop_in_exports_every_reference_name():
    from lte_phy import channel_coding as cc
    names = ['calculate_crc24a', 'calculate_crc24b', 'attach_crc24a', 'attach_crc24b', 'check_crc24a',
             'check_crc24b', 'segment_code_blocks', 'desegment_code_blocks', 'get_segmentation_info',
             'turbo_encode', 'turbo_decode', 'LogMAPDecoder', 'qpp_interleave', 'qpp_deinterleave',
             'rate_match_turbo', 'rate_dematching_turbo', 'sub_block_interleaver', 'sub_block_deinterleaver']
    assert sorted(cc.__all__) == sorted(names)   # core/channel_coding/__init__.py:22-40
    for n in names:
        assert callable(getattr(cc, n)), n


@pytest.mark.parametrize('n', [1, 31, 32, 33, 1030, 5574])
def test_sub_block_interleaver(golden_coding, n):
    from lte_phy import channel_coding as cc
    g, _ = golden_coding
    v = cc.sub_block_interleaver(g[f'sbi{n}_in'])
    assert v.dtype == np.uint8 and np.array_equal(v, g[f'sbi{n}_out'])
    assert np.array_equal(cc.sub_block_deinterleaver(v, n), g[f'sbi{n}_back'])


@pytest.mark.parametrize('K', [40, 1024, 6144])
def test_qpp(golden_coding, K):
    from lte_phy import channel_coding as cc
    g, _ = golden_coding
    assert np.array_equal(cc.qpp_interleave(g[f'qpp{K}_in'], K), g[f'qpp{K}_il'])
    assert np.array_equal(cc.qpp_deinterleave(g[f'qpp{K}_in'], K), g[f'qpp{K}_dil'])
    with pytest.raises(ValueError, match='Invalid interleaver size K=41'):
        cc.qpp_interleave(np.zeros(41), 41)


@pytest.mark.parametrize('B', [40, 6144, 6145, 9232, 27784])
def test_segmentation_info(golden_coding, B):
    from lte_phy import channel_coding as cc
    _, meta = golden_coding
    assert cc.get_segmentation_info(B) == meta[f'info{B}']


@pytest.mark.parametrize('B', [40, 6144])
def test_single_block_segmentation(golden_coding, B):
    """B <= Z: fillers first, no CRC-24B (no device call)."""
    from lte_phy import channel_coding as cc
    g, meta = golden_coding
    blocks, md = cc.segment_code_blocks(g[f'seg{B}_tb'])
    assert md == meta[f'seg{B}']
    assert np.array_equal(np.concatenate(blocks), g[f'seg{B}_blocks'])
    assert np.array_equal(cc.desegment_code_blocks(blocks, md), g[f'seg{B}_back'])


@pytest.mark.parametrize('K', [40, 1024, 5568])
def test_empty_inputs_like_the_reference(K):
    """rate_dematching_turbo on E = 0 LLRs returns zeros(3K + 12) (every
    position punctured, rate_matching.py:422-489 with an empty loop) and
    LogMAPDecoder.decode on K = 0 returns empty decisions / LLRs
    (turbo_decoder.py:181-278 with zero recursion steps), in the drop-in and in
    the C-ABI (neither touches the device)."""
    import ctypes
    from lte_phy import _capi as C
    from lte_phy import channel_coding as cc
    out = cc.rate_dematching_turbo(np.zeros(0), K, 0)
    assert out.dtype == np.float64 and out.shape == (3 * K + 12,) and not out.any()
    b, llr = cc.LogMAPDecoder().decode(np.zeros(0), np.zeros(0), return_extrinsic=True)
    assert b.shape == (0,) and b.dtype == np.uint8 and llr.shape == (0,)
    buf = np.full(2 * (3 * K + 12), 7.0)
    assert C.load().lte_rate_dematch_host64(K, 0, 0, 2, None, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_double))) == 0
    assert not buf.any()
    assert C.load().lte_bcjr_host64(0, 3, None, None, None, None) == 0
