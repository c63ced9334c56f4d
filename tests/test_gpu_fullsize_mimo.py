"""GPU: the multi-antenna bench workloads at their full bench sizes, checked
through size-independent properties (as tests/test_gpu_fullsize.py does for
config 2):

* config 4 (SFBC 2x2 + turbo, 20 MHz 64-QAM PedA, core/ofdm_core.py:2049-2258
  with the coding chain): 65 536 frames per call, bench.py's default;
* config 5 (4x4 rank-4 MMSE, core/ofdm_core.py:2489-2815): 32 768 frames per
  call on flat CN(0,1) links and on PedA links at 3 km/h (about 64 GB of
  received streams -- every per-frame buffer of the multi-antenna workspaces
  runs past 2^31 bytes, and the largest past 2^35).

Per-frame counts (bit errors, bits, block error) of the first and last 32
frames of the big call equal those of the same frame ids in a 64-frame plan;
the BER curve over the whole batch falls with SNR; and 4 frames at each end
re-run by the float64 oracle on its Philox restatement (oracle/philox.py)
give the same bit errors (and CRC verdicts).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TB = 27760
SNRS = np.arange(0, 31, 2, dtype=np.float64)
SEED = 0x5EED


@pytest.fixture(scope='module')
def C():
    from lte_phy import _capi, engine
    _capi.device_init()
    engine.clear_cache()
    return _capi


def _plan(config, n, channel='awgn'):
    import lte_phy
    Cfg, Sim = lte_phy.LTEConfig, lte_phy.OFDMSimulator
    if config == 4:
        s = Sim(Cfg(bandwidth=20.0, modulation='64-QAM'), channel_type='rayleigh_mp', itu_profile='Pedestrian_A')
        return s._sfbc_plan(0, TB, 2, coded=True, max_frames=n)
    from lte_phy.ofdm_core import _spatial_plan
    return _spatial_plan(Cfg(bandwidth=20.0, modulation='64-QAM'), channel, 'Pedestrian_A', 3.0, 2.0, 14,
                         14 * 999 * 6, n)[0]


@pytest.mark.parametrize('config,F,channel', [(4, 65536, 'rayleigh_mp'), (5, 32768, 'awgn'),
                                              (5, 32768, 'rayleigh_mp')])
def test_mimo_bench_size_batch_invariance(C, config, F, channel):
    from lte_phy import engine
    from oracle import philox as P
    nb = TB if config == 4 else 14 * 999 * 6
    ids = np.arange(F, dtype=np.uint64) + np.uint64(3 * F)
    si = (ids % np.uint64(len(SNRS))).astype(np.int64)
    big = _plan(config, F, channel)
    per_frame = big.run(SNRS[si], snr_index=np.arange(F, dtype=np.int32), n_snr=F, seed=SEED,
                        frame_ids=ids)['counts']
    del big
    engine.clear_cache()
    assert per_frame.shape == (F, 4)
    assert np.all(per_frame[:, 1] == nb) and np.all(per_frame[:, 3] == 1)
    by_snr = np.zeros((len(SNRS), 4), dtype=np.uint64)
    np.add.at(by_snr, si, per_frame)
    ber = by_snr[:, 0] / by_snr[:, 1]
    assert ber[0] > 0.05 and np.all(np.diff(ber[::3]) <= 0) and ber[-1] < ber[0], ber
    if config == 4:
        assert ber[-1] < 1e-3
    sel = np.r_[0:32, F - 32:F]
    small = _plan(config, 64, channel)
    ref = small.run(SNRS[si[sel]], snr_index=np.arange(64, dtype=np.int32), n_snr=64, seed=SEED,
                    frame_ids=ids[sel])['counts']
    del small
    engine.clear_cache()
    assert np.array_equal(per_frame[sel], ref)
    # 4 frames at each end through the float64 oracle on its Philox draws
    ends = np.r_[0:4, F - 4:F]
    kw = {'channel': channel} if config == 5 else {}
    orc = np.array([P.BENCH_FRAMES[config](int(f), **kw) for f in ids[ends]])
    assert np.array_equal(per_frame[ends, 0], orc[:, 0])
    if config == 4:
        assert np.array_equal(per_frame[ends, 2], 1 - orc[:, 1])
