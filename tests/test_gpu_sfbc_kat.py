"""GPU: the reference's only assertion-bearing test, test/test_alamouti_unit.py
(:13-126), run against the HIP SFBC path through the drop-in SFBCAlamouti
(lte_phy.sfbc_alamouti -> lte_sfbc_encode_host64 / lte_sfbc_decode_host64,
the pair rule and combiner of the chain kernels), plus the reference's own
SFBC outputs in golden_mimo (tests/golden/make_golden_mimo.py).

Bars: encode exact; the KAT decode within 1e-10 of (s0, s1) as the reference
asserts, and equal to the reference's decode; the seed-42 QPSK 10 dB variant
SER < 0.10 as the reference asserts, decoded symbols equal to the oracle's
restatement to 1e-14; the 998-SC random decodes to 1e-14 relative."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def al():
    from lte_phy import _capi
    from lte_phy.sfbc_alamouti import SFBCAlamouti
    _capi.device_init(0)
    return SFBCAlamouti(num_tx=2, enabled=True)


def test_alamouti_perfect_channel(al, golden_mimo):
    s0, s1 = 1.0 + 1.0j, -1.0 + 1.0j
    tx0, tx1 = al.encode(np.array([s0, s1]))
    assert tx0[0] == s0 and tx0[1] == -np.conj(s1)
    assert tx1[0] == s1 and tx1[1] == np.conj(s0)
    assert np.array_equal(tx0, golden_mimo['sfbc_kat_tx0']) and np.array_equal(tx1, golden_mimo['sfbc_kat_tx1'])
    h0, h1 = 1.0 + 0j, 0.0 + 1.0j
    rx = np.array([h0 * tx0[0] + h1 * tx1[0], h0 * tx0[1] + h1 * tx1[1]])
    dec = al.decode(rx, np.array([h0, h0]), np.array([h1, h1]), regularization=1e-10)
    assert abs(dec[0] - s0) < 1e-10 and abs(dec[1] - s1) < 1e-10
    assert np.array_equal(dec, golden_mimo['sfbc_kat_dec'])


def test_alamouti_with_noise(al, mimo_oracle):
    np.random.seed(42)
    N = 100
    sym = (np.random.choice([-1, 1], N) + 1j * np.random.choice([-1, 1], N)) / np.sqrt(2)
    tx0, tx1 = al.encode(sym)
    h0, h1 = 1.0 + 0j, 0.0 + 1.0j
    rx = h0 * tx0 + h1 * tx1
    snr_linear = 10 ** (10.0 / 10)
    noise_power = np.mean(np.abs(rx) ** 2) / snr_linear
    rx = rx + (np.random.randn(N) + 1j * np.random.randn(N)) * np.sqrt(noise_power / 2)
    H0, H1 = np.full(N, h0), np.full(N, h1)
    dec = al.decode(rx, H0, H1)
    errors = np.sum(~np.isclose(dec.real, sym.real, atol=0.5) | ~np.isclose(dec.imag, sym.imag, atol=0.5))
    assert errors / N < 0.10
    ref = mimo_oracle.sfbc_decode(rx, H0, H1)
    assert np.max(np.abs(dec - ref)) <= 1e-14 * np.max(np.abs(ref))


def test_random_encode_decode_vs_reference(al, golden_mimo):
    t0, t1 = al.encode(golden_mimo['sfbc_sym'])
    assert np.array_equal(t0, golden_mimo['sfbc_tx0']) and np.array_equal(t1, golden_mimo['sfbc_tx1'])
    for i in range(2):
        g = golden_mimo[f'sfbc_dec{i}_out']
        out = al.decode(golden_mimo[f'sfbc_dec{i}_rx'], golden_mimo[f'sfbc_dec{i}_H0'], golden_mimo[f'sfbc_dec{i}_H1'])
        assert np.max(np.abs(out - g) / np.maximum(np.abs(g), 1e-300)) < 1e-14, i


def test_stage_errors(al):
    with pytest.raises(ValueError, match='must be even for Alamouti coding, got 3'):
        al.encode(np.ones(3, complex))
    t0, t1 = al.encode(np.zeros(0, complex))
    assert t0.shape == (0,) and t1.shape == (0,)


def test_reference_callers_through_compat_paths():
    """The reference's own import lines with only PYTHONPATH changed
    (ofdm-lte_amd/compat): test/test_alamouti_unit.py:11's `from
    core.sfbc_alamouti import SFBCAlamouti` runs its KAT on the HIP path, and
    examples/example_basic.py:17's `from module import OFDMModule, LTEConfig`
    transmits through the GPU chain (a child process, one GPU call each)."""
    import os
    import subprocess
    import sys
    from conftest import ROOT
    code = r'''
import numpy as np
from core.sfbc_alamouti import SFBCAlamouti
from module import OFDMModule, LTEConfig
al = SFBCAlamouti(num_tx=2, enabled=True)
s0, s1 = 1.0 + 1.0j, -1.0 + 1.0j
tx0, tx1 = al.encode(np.array([s0, s1]))
rx = np.array([tx0[0] + 1j * tx1[0], tx0[1] + 1j * tx1[1]])
dec = al.decode(rx, np.array([1.0 + 0j, 1.0 + 0j]), np.array([1j, 1j]), regularization=1e-10)
assert abs(dec[0] - s0) < 1e-10 and abs(dec[1] - s1) < 1e-10
m = OFDMModule()
r = m.transmit(np.random.RandomState(0).randint(0, 2, 10000), snr_db=20)
assert r['ber'] < 1e-2, r['ber']
print('ok', m.config.bandwidth, r['ber'])
'''
    env = dict(os.environ)
    env['PYTHONPATH'] = os.path.join(ROOT, 'ofdm-lte_amd', 'compat')
    r = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, text=True, timeout=240, cwd='/tmp')
    assert r.returncode == 0 and 'ok' in r.stdout, (r.stdout[-1000:], r.stderr[-3000:])
