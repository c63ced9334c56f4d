"""CPU: the oracle's restatement of the Philox mode (oracle/philox.py) against
the published Philox4x32-10 known-answer vectors (Random123 kat_vectors:
Salmon et al., SC'11), plus the draw mapping's structure -- the parity anchor
for every GPU test that re-runs a bench frame on the oracle
(tests/test_gpu_philox.py)."""
import numpy as np
import pytest

from oracle import philox as P

KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff), (0xffffffff, 0xffffffff),
     (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


@pytest.mark.parametrize('ctr,key,out', KAT)
def test_philox_known_answers(ctr, key, out):
    got = P.philox4x32_10(*ctr, *key)
    assert tuple(int(x) for x in got) == out


def test_rng4_counter_layout():
    # rng4(seed, frame, stream, idx) = Philox((idx, stream, frame lo, frame hi), (seed lo, seed hi))
    seed, frame = 0x0123456789ABCDEF, 0xFEDCBA9876543210
    r = P.rng4(seed, frame, 0x10003, [5, 6])
    ref = P.philox4x32_10([5, 6], 0x10003, frame & 0xFFFFFFFF, frame >> 32, seed & 0xFFFFFFFF, seed >> 32)
    assert r.shape == (4, 2)
    assert all(np.array_equal(r[i], ref[i]) for i in range(4))


def test_payload_bits_msb_first():
    w = P.payload_words(0x5EED, 77, 27760)
    b = P.payload_bits(0x5EED, 77, 27760)
    assert len(w) == 868 and len(b) == 27760 and b.dtype == np.uint8
    assert int(''.join(map(str, b[:32])), 2) == int(w[0])
    assert int(''.join(map(str, b[32 * 867:])), 2) == int(w[867]) >> (32 - 27760 % 32)
    r = P.rng4(0x5EED, 77, P.STREAM_BITS, [1])
    assert np.array_equal(w[4:8], r[:, 0])   # word 4 q + c = output c of counter q


def test_phases_and_normals_mapping():
    ph = P.fade_phases(0x5EED, 3, 1, 4)
    u = P.rng4(0x5EED, 3, P.STREAM_FADE + 64 + 2, [0, 1, 2, 3])
    assert np.array_equal(ph[2], P.uniform_phase(u.T.reshape(-1)))
    assert np.all((ph > 0) & (ph < 2 * np.pi))
    zr7, _ = P.normals(0x5EED, 3, P.STREAM_NOISE, 7)
    zr, zi = P.normals(0x5EED, 3, P.STREAM_NOISE, 8)
    assert zr7.shape == (7,) and np.array_equal(zr7, zr[:7])
    r = P.rng4(0x5EED, 3, P.STREAM_NOISE, [3])
    e_re, e_im = P.box_muller(r[0], r[1])   # sample 6: (x, y) of counter 3
    o_re, o_im = P.box_muller(r[2], r[3])   # sample 7: (z, w) of counter 3
    assert (zr[6], zi[6], zr[7], zi[7]) == (e_re[0], e_im[0], o_re[0], o_im[0])


def test_normals_moments():
    zr, zi = P.normals(0x5EED, 11, P.STREAM_NOISE, 1 << 18)
    z = np.concatenate([zr, zi])
    assert abs(z.mean()) < 0.01 and abs(z.var() - 1.0) < 0.01
    assert abs(np.mean(np.abs(z) > 3.0) - 2.6998e-3) < 6e-4
    assert np.max(np.abs(z)) < np.sqrt(-2 * np.log(0.5 * 2.0 ** -32)) + 1e-12


def test_bench_frame_snr_and_determinism():
    assert [P.bench_snr(f) for f in (0, 8, 11, 15, 16, 65535)] == [0.0, 16.0, 22.0, 30.0, 0.0, 30.0]
    e1 = P.config2_frame(10)
    assert e1 == P.config2_frame(10)
    assert e1 == (0, True)                          # 20 dB: decodes
    e0 = P.config2_frame(0)
    assert e0[0] > 10000 and not e0[1]              # 0 dB: fails
