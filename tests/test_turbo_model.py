"""CPU: pins the GPU decoder's float32 model (oracle or_turbo_decode_f32,
the algorithm k_turbo implements bit-for-bit -- see test_gpu_parity.py)
against the reference decoder (turbo_decoder.py:338-450).

  * converging cases: identical decisions to the reference's golden output and
    to the float64 oracle;
  * past the decoder's failure point (the reference's decoder stops
    converging below about 3.5 dB SNR on these BPSK LLRs), float round-off decides
    which wrong bits come out; there the f32 model's error rate vs the sent
    code block must agree with the reference's within 0.05.
"""
import numpy as np
import pytest

from conftest import unpack


@pytest.mark.parametrize('K,its', [(40, 8), (1024, 1), (1024, 8), (5568, 2)])
def test_f32_model_vs_reference_golden(golden, oracle, K, its):
    key = f'td_{K}_{its}'
    llr = golden[key + '_llr']
    ref = unpack(golden[key + '_dec'], K)
    cb = unpack(golden[key + '_cb'], K)
    m = oracle.turbo_decode_f32_model(llr.astype(np.float32), K, its)
    ref_ber = np.mean(ref != cb)
    if ref_ber == 0 or its <= 2:
        assert np.array_equal(m, ref)
    else:
        assert abs(np.mean(m != cb) - ref_ber) < 0.05, (np.mean(m != cb), ref_ber)


@pytest.mark.parametrize('K', [40, 528, 2048, 6144])
def test_f32_model_equals_f64_when_converging(oracle, K):
    rs = np.random.RandomState(K)
    for snr in (4.0, 6.0, 10.0):
        cb = rs.randint(0, 2, K).astype(np.uint8)
        s = 1 - 2.0 * oracle.turbo_encode(cb)
        s2 = 10 ** (-snr / 10)
        llr = (2 * (s + np.sqrt(s2) * rs.randn(len(s))) / s2).astype(np.float32)
        a = oracle.turbo_decode(llr.astype(np.float64), K, 8)
        b = oracle.turbo_decode_f32_model(llr, K, 8)
        assert np.array_equal(a, b), (K, snr)
        assert np.array_equal(a, cb), (K, snr)


def test_f32_model_failure_regime_statistics(oracle):
    """Below the cliff both decoders fail; their BERs agree statistically."""
    K, n, snr = 1024, 12, 1.0
    rs = np.random.RandomState(5)
    e64 = e32 = 0
    for _ in range(n):
        cb = rs.randint(0, 2, K).astype(np.uint8)
        s = 1 - 2.0 * oracle.turbo_encode(cb)
        s2 = 10 ** (-snr / 10)
        llr = (2 * (s + np.sqrt(s2) * rs.randn(len(s))) / s2).astype(np.float32)
        e64 += int(np.sum(oracle.turbo_decode(llr.astype(np.float64), K, 8) != cb))
        e32 += int(np.sum(oracle.turbo_decode_f32_model(llr, K, 8) != cb))
    assert abs(e64 - e32) / (n * K) < 0.02, (e64, e32)
