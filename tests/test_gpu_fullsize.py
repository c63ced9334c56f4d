"""GPU: the bench workload at its full size (BASELINE.json config 2, F = 65 536
coded subframes per call, bench.py's plan), checked through size-independent
properties -- the oracle cannot run 65 536 frames, but every frame must come
out exactly as it does in a small batch:

* batch invariance: per-frame counts (bit errors, bits, block error) of frames
  at both ends of the 65 536-frame call equal those of the same frame ids run
  in a 64-frame plan -- the last frames sit past 2^31 bytes in every per-frame
  buffer (the received streams alone are 32 GB), so 32-bit offset arithmetic
  anywhere on the path shows up here;
* the SNR curve: BER falls over 0:2:30 dB and the top of the curve decodes;
* f64: those 64 frames (bench step 7's first and last 32) re-run by the oracle
  on its restatement of the device's Philox draws (oracle/philox.py) give the
  same bit errors and block errors frame by frame.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

F = 65536
TB = 27760
SNRS = np.arange(0, 31, 2, dtype=np.float64)


@pytest.fixture(scope='module')
def C():
    from lte_phy import _capi
    _capi.device_init()
    return _capi


@pytest.mark.parametrize('prec', ['f64', 'f32'])
def test_bench_size_batch_invariance(C, prec):
    import lte_phy
    from lte_phy import engine
    sim = lte_phy.OFDMSimulator(lte_phy.LTEConfig(bandwidth=20.0, modulation='64-QAM'), channel_type='rayleigh_mp',
                                itu_profile='Pedestrian_A', precision=prec)
    ids = np.arange(F, dtype=np.uint64) + np.uint64(7 * F)
    snr = SNRS[(ids % np.uint64(len(SNRS))).astype(np.int64)]
    big = sim._plan(C.CHAIN_CODED, 0, TB, max_frames=F)
    per_frame = big.run(snr, snr_index=np.arange(F, dtype=np.int32), n_snr=F, seed=0x5EED,
                        frame_ids=ids)['counts']
    del big
    engine.clear_cache()
    assert per_frame.shape == (F, 4)
    assert np.all(per_frame[:, 1] == TB) and np.all(per_frame[:, 3] == 1)
    # the curve over the whole batch: BER falls with SNR, the top decodes
    by_snr = np.zeros((len(SNRS), 4), dtype=np.uint64)
    np.add.at(by_snr, (ids % np.uint64(len(SNRS))).astype(np.int64), per_frame)
    ber = by_snr[:, 0] / by_snr[:, 1]
    assert ber[0] > 0.05 and ber[-1] < 1e-3
    assert np.all(np.diff(ber[::3]) < 0), ber
    # both ends of the big call against a 64-frame plan on the same frame ids
    sel = np.r_[0:32, F - 32:F]
    small = sim._plan(C.CHAIN_CODED, 0, TB, max_frames=64)
    ref = small.run(snr[sel], snr_index=np.arange(64, dtype=np.int32), n_snr=64, seed=0x5EED,
                    frame_ids=ids[sel])['counts']
    assert np.array_equal(per_frame[sel], ref)
    if prec == 'f64':
        # the same frames through the float64 oracle on its Philox restatement
        # (oracle/philox.py): identical bit errors and block verdicts
        from oracle import philox as P
        orc = np.array([P.config2_frame(int(f)) for f in ids[sel]])
        assert np.array_equal(per_frame[sel, 0], orc[:, 0])
        assert np.array_equal(per_frame[sel, 2], 1 - orc[:, 1])


@pytest.mark.parametrize('prec', ['f64', 'f32'])
def test_decoder_partial_chunk_batch_invariance(C, prec):
    """The decoder's block arrays are chunked over 32 frame groups (TURBO_CH,
    lte_internal.h turbo_elem): a batch of 34 groups (one full chunk + a partial
    one, 2 129 frames: the last group partial too) must give every frame the
    per-frame counts it gets in 64-frame plans (one partial chunk each), around
    the waterfall (14-22 dB) where the counts vary frame to frame."""
    import lte_phy
    from lte_phy import engine
    sim = lte_phy.OFDMSimulator(lte_phy.LTEConfig(bandwidth=20.0, modulation='64-QAM'), channel_type='rayleigh_mp',
                                itu_profile='Pedestrian_A', precision=prec)
    n = 33 * 64 + 17
    ids = np.arange(n, dtype=np.uint64) + np.uint64(12345)
    snr = (14.0 + 2.0 * (ids % np.uint64(5))).astype(np.float64)
    big = sim._plan(C.CHAIN_CODED, 0, TB, max_frames=n)
    per_frame = big.run(snr, snr_index=np.arange(n, dtype=np.int32), n_snr=n, seed=0x5EED, frame_ids=ids)['counts']
    del big
    engine.clear_cache()
    small = sim._plan(C.CHAIN_CODED, 0, TB, max_frames=64)
    ref = np.concatenate([small.run(snr[i:i + 64], snr_index=np.arange(min(64, n - i), dtype=np.int32),
                                    n_snr=min(64, n - i), seed=0x5EED, frame_ids=ids[i:i + 64])['counts']
                          for i in range(0, n, 64)])
    assert per_frame[:, 0].sum() > 0 and np.any(per_frame[:, 2] == 0)   # errors and decoded blocks both present
    assert np.array_equal(per_frame, ref)
