"""Drop-in mirror of core/rayleighchannel.py: RayleighChannel.

The Jakes fading and the multipath filter run on the GPU (lte_channel_host64,
the chains' channel kernel, with the noise set to zero); the random phases are
drawn on the host from the global NumPy RNG exactly as the reference draws
them (np.random.rand(16) per path and call, core/rayleighchannel.py:31), so
the RNG state after a call is the reference's."""
from __future__ import annotations

import numpy as np

from . import _capi as C

N_S = 16   # the kernels' sinusoid count (the reference's default N_s)


def _run_channel(x, delays_samples, gains, fD, fs, phases):
    """y = sum_p gains[p] * jakes_p * x delayed by delays_samples[p] (zero
    prefix), on the GPU; phases [P][16] in radians."""
    x = np.ascontiguousarray(x, dtype=np.complex128)
    L = len(x)
    P = len(delays_samples)
    y = np.zeros(L, dtype=np.complex128)
    if L == 0 or P == 0:
        return y
    dl = np.ascontiguousarray(delays_samples, dtype=np.int32)
    g = np.ascontiguousarray(gains, dtype=np.float64)
    ph = np.ascontiguousarray(np.asarray(phases, dtype=np.float64).reshape(1, P, N_S))
    z = np.zeros((1, 2, L), dtype=np.float64)   # no noise: the filter alone
    npow = np.zeros(1, dtype=np.float64)
    C.device_init()
    C.check(C.load().lte_channel_host64(L, 1, C.CH_RAYLEIGH, P, C.ptr(dl, C.I32), C.ptr(g, C.F64), float(fD),
                                        float(fs), 0.0, 0, C.ptr(x.view(np.float64), C.F64), C.ptr(ph, C.F64),
                                        C.ptr(z, C.F64), C.ptr(y.view(np.float64), C.F64), C.ptr(npow, C.F64)))
    return y


class RayleighChannel:
    """RayleighChannel (core/rayleighchannel.py:5-109).  gains in dB (turned
    into amplitudes here, as the reference does)."""

    def __init__(self, Fs, fD, delays, gains):
        self.Fs = Fs
        self.fD = fD
        self.delays = np.array(delays)
        self.gains = 10 ** (np.array(gains) / 20)
        assert len(self.delays) == len(self.gains), "delays y gains deben tener la misma longitud"
        self.num_paths = len(delays)

    @staticmethod
    def _phases(N_s):
        if N_s != N_S:
            raise NotImplementedError(f"the GPU Jakes sum has N_s = {N_S} sinusoids")
        return 2 * np.pi * np.random.rand(N_s)

    def jakes_fading(self, N, N_s=16):
        """sqrt(2 / N_s) sum_n exp(j (2 pi fD cos(2 pi n / N_s) t + phi_n)),
        t = k / Fs (:20-42): the channel kernel on an all-ones input."""
        phi = self._phases(N_s)
        return _run_channel(np.ones(int(N), dtype=np.complex128), [0], [1.0], self.fD, self.Fs, phi[None])

    def filter(self, x):
        """sum over paths of gain * fading * x delayed by round(tau Fs) with a
        zero prefix (:44-58); a fresh set of 16 phases per path, in path order."""
        N = len(x)
        phases = np.stack([self._phases(N_S) for _ in range(self.num_paths)]) if self.num_paths else np.zeros((0, N_S))
        d = [int(np.round(t * self.Fs)) for t in self.delays]
        return _run_channel(x, d, self.gains, self.fD, self.Fs, phases) if N else np.zeros(0, dtype=complex)

    def large_scale_fading(self, d, fc, PL0=30, n=3.5, sigma=4, d0=100):
        """Log-distance path loss + log-normal shadowing (:60-74): a scalar."""
        PL_dB = PL0 + 10 * n * np.log10(d / d0)
        shadowing = np.random.normal(0, sigma)
        return 10 ** (-(PL_dB + shadowing) / 20)

    def channel_response(self, freqs, h_taps, N_freq=None):
        """sum_i h_taps[i] exp(-j 2 pi f tau_i) over freqs (:76-92): a host
        evaluation of the tap set's frequency response (not a link stage)."""
        Hf = np.zeros_like(freqs, dtype=complex)
        for i in range(self.num_paths):
            Hf += h_taps[i] * np.exp(-1j * 2 * np.pi * freqs * self.delays[i])
        return Hf

    def impulse_response(self, N=1):
        """(delays, taps): each path's gain times the first sample of a fresh
        Jakes process of N samples (:95-109)."""
        taps, delays_out = [], []
        for i in range(self.num_paths):
            taps.append(self.gains[i] * self.jakes_fading(N)[0])
            delays_out.append(self.delays[i])
        return np.array(delays_out), np.array(taps)
