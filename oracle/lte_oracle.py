"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement (NumPy float64 + the C loops in ``coding_oracle.c``) of the
reference's hot path, Darioxavierl/OFDM-LTE @ 2026-02-13.  It is the checker
for the HIP path and the timed CPU baseline ("port") in ``bench.py``.  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import it; the product package (``ofdm-lte_amd/lte_phy``) never does.

Parity pinning: every function below is checked bit-for-bit against golden
vectors produced by running the reference itself in the survey container
(``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``; test:
``tests/test_oracle_golden.py``).  The restatement uses the same NumPy
operations in the same order as the reference, so results are identical, not
merely close.

Every function cites the reference file:line it restates.
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass, field

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))

# --------------------------------------------------------------------------
# config.py:11-60
LTE_PROFILES = {
    1.25: {'Nc': 76, 'N': 128},
    2.5: {'Nc': 150, 'N': 256},
    5.0: {'Nc': 300, 'N': 512},
    10.0: {'Nc': 600, 'N': 1024},
    15.0: {'Nc': 900, 'N': 2048},
    20.0: {'Nc': 1200, 'N': 2048},
}
CP_VALUES = {'normal': 4.7, 'extended_15khz': 16.6, 'extended_7.5khz': 33.0}
ITU_CHANNEL_MODELS = {
    'Pedestrian_A': {'delays_us': [0.0, 0.11, 0.19, 0.41],
                     'power_db': [0.0, -9.7, -19.2, -22.8]},
    'Pedestrian_B': {'delays_us': [0.0, 0.2, 0.8, 1.2, 2.3, 3.7],
                     'power_db': [0.0, -0.9, -4.9, -8.0, -7.8, -23.9]},
    'Vehicular_A': {'delays_us': [0.0, 0.31, 0.71, 1.09, 1.73, 2.51],
                    'power_db': [0.0, -1.0, -9.0, -10.0, -15.0, -20.0]},
    'Vehicular_B': {'delays_us': [0.0, 0.3, 0.7, 1.09, 1.73, 2.51, 3.7, 4.53],
                    'power_db': [0.0, -1.0, -9.0, -10.0, -13.0, -16.0, -21.6, -24.0]},
    'Bad_Urban': {'delays_us': [0.0, 0.1, 0.3, 0.5, 0.9, 1.3, 1.9, 2.6],
                  'power_db': [0.0, -3.0, -5.0, -7.0, -9.0, -11.0, -13.0, -15.0]},
}
BPS = {'QPSK': 2, '16-QAM': 4, '64-QAM': 6}


@dataclass
class Numerology:
    """LTEConfig._calculate_parameters (config.py:101-130) + LTEResourceGrid
    (core/resource_mapper.py:33-93)."""
    bandwidth: float = 5.0
    delta_f: float = 15.0
    modulation: str = 'QPSK'
    cp_type: str = 'normal'
    N: int = 0
    Nc: int = 0
    fs: float = 0.0
    cp: int = 0
    bps: int = 0
    data_idx: np.ndarray = field(default=None, repr=False)
    pilot_idx: np.ndarray = field(default=None, repr=False)
    guard_idx: np.ndarray = field(default=None, repr=False)
    dc: int = 0

    def __post_init__(self):
        if self.bandwidth in LTE_PROFILES:
            p = LTE_PROFILES[self.bandwidth]
            self.Nc, self.N = p['Nc'], p['N']
        else:
            self.Nc = int((self.bandwidth * 1e3) / self.delta_f)
            self.N = int(2 ** np.ceil(np.log2(self.Nc)))
        self.fs = self.N * self.delta_f * 1e3
        if self.cp_type == 'extended':
            cpd = CP_VALUES['extended_15khz'] if self.delta_f == 15.0 else CP_VALUES['extended_7.5khz']
        else:
            cpd = CP_VALUES['normal']
        self.cp = int(cpd * 1e-6 * self.fs)
        self.bps = BPS[self.modulation]
        gl = (self.N - self.Nc) // 2
        gr = self.N - self.Nc - gl
        self.dc = self.N // 2
        k = np.arange(self.N)
        guard = (k < gl) | (k >= self.N - gr)
        dc = (k == self.dc) & ~guard
        pilot = ~guard & ~dc & (((k - gl) % 6) == 3)
        data = ~guard & ~dc & ~pilot
        self.data_idx = k[data]
        self.pilot_idx = k[pilot]
        self.guard_idx = k[guard]

    @property
    def Nd(self):
        return len(self.data_idx)

    @property
    def Np(self):
        return len(self.pilot_idx)


def pilots(cell_id: int, n: int) -> np.ndarray:
    """PilotPattern.generate_pilots (core/resource_mapper.py:137-152).
    Reseeds the GLOBAL NumPy RNG exactly like the reference (quirk Q1)."""
    np.random.seed(cell_id)
    phases = np.random.choice([1, -1], size=n)
    return ((1 + 1j) / np.sqrt(2)) * phases


def constellation(mod: str) -> np.ndarray:
    """QAMModulator._generate_constellation (core/modulator.py:28-59)."""
    if mod == 'QPSK':
        return np.array([1 + 1j, 1 - 1j, -1 + 1j, -1 - 1j]) / np.sqrt(2)
    if mod == '16-QAM':
        v = [-3, -1, 1, 3]
        return np.array([r + 1j * i for r in v for i in v]) / np.sqrt(10)
    if mod == '64-QAM':
        v = [-7, -5, -3, -1, 1, 3, 5, 7]
        return np.array([r + 1j * i for r in v for i in v]) / np.sqrt(42)
    raise ValueError(mod)


def bits_to_indices(bits: np.ndarray, bps: int) -> np.ndarray:
    """QAMModulator.bits_to_symbols index part (core/modulator.py:71-86):
    zero-pad to a multiple of bps, MSB-first natural binary."""
    bits = np.asarray(bits).astype(np.int64)
    if len(bits) % bps:
        bits = np.pad(bits, (0, bps - len(bits) % bps), 'constant')
    b = bits.reshape(-1, bps)
    w = (1 << np.arange(bps - 1, -1, -1)).astype(np.int64)
    return (b * w).sum(axis=1)


def bits_to_symbols(bits, mod):
    c = constellation(mod)
    return c[bits_to_indices(bits, BPS[mod]) % len(c)]


def nearest_indices(symbols: np.ndarray, mod: str) -> np.ndarray:
    """symbols_to_bits / _detect_symbols argmin (core/modulator.py:100-110;
    core/lte_receiver.py:508-521): Euclidean argmin, first index on ties."""
    c = constellation(mod)
    out = np.empty(len(symbols), dtype=np.int64)
    step = 8192
    for s in range(0, len(symbols), step):
        y = symbols[s:s + step]
        out[s:s + step] = np.argmin(np.abs(c[None, :] - y[:, None]), axis=1)
    return out


def indices_to_bits(idx: np.ndarray, bps: int) -> np.ndarray:
    """format(idx, '0{bps}b') (core/modulator.py:108-110)."""
    sh = np.arange(bps - 1, -1, -1)
    return ((idx[:, None] >> sh[None, :]) & 1).reshape(-1).astype(np.int64)


def symbols_to_bits(symbols, mod):
    return indices_to_bits(nearest_indices(np.asarray(symbols), mod), BPS[mod])


# --------------------------------------------------------------------------
# TX: OFDMModulator.modulate_stream / _modulate_lte (core/modulator.py:214-302)
def ofdm_symbols_tx(num: Numerology, data_syms: np.ndarray, pil: np.ndarray) -> np.ndarray:
    """ResourceMapper.map_symbols (core/resource_mapper.py:181-223) + IFFT*sqrt(N)
    + CP (core/modulator.py:242-248) for a stack [n_sym, Nd] of data symbols."""
    n_sym = data_syms.shape[0]
    grid = np.zeros((n_sym, num.N), dtype=complex)
    grid[:, num.data_idx] = data_syms
    grid[:, num.pilot_idx] = pil
    td = np.fft.ifft(grid, axis=1) * np.sqrt(num.N)
    return np.concatenate([td[:, num.N - num.cp:], td], axis=1).reshape(-1)


def dft_matrix(M: int, inverse: bool = False) -> np.ndarray:
    """DFTPrecodifier._compute_dft_matrix / IDFTDecodifier._compute_idft_matrix
    (core/dft_precoding.py:43-54, 156-175): exp(-+j 2 pi k n / M) / sqrt(M)."""
    k = np.arange(M).reshape(-1, 1)
    n = np.arange(M).reshape(1, -1)
    sgn = 1j if inverse else -1j
    return np.exp(sgn * 2 * np.pi * k * n / M) / np.sqrt(M)


def modulate_stream(num: Numerology, bits: np.ndarray, sc_fdm: bool = False):
    """OFDMModulator.modulate_stream (core/modulator.py:252-302), 'lte' mode;
    sc_fdm: each OFDM symbol's Nd QAM symbols are multiplied by the M = Nd DFT
    matrix before mapping (_modulate_lte :232-236, one matrix-vector product per
    symbol as the reference).  Returns (signal, list-of-per-symbol QAM symbols
    (un-precoded, as the reference returns them), n_sym)."""
    bits = np.asarray(bits)
    bpo = num.Nd * num.bps
    n_sym = int(np.ceil(len(bits) / bpo))
    total = n_sym * bpo
    if len(bits) < total:
        bits = np.pad(bits, (0, total - len(bits)), 'constant')
    syms = bits_to_symbols(bits[:total], num.modulation).reshape(n_sym, num.Nd)
    mapped = syms
    if sc_fdm:
        D = dft_matrix(num.Nd)
        mapped = np.stack([D @ syms[i] for i in range(n_sym)])
    pil = pilots(0, num.Np)                    # reseed side effect (Q1)
    sig = ofdm_symbols_tx(num, mapped, pil)
    return sig, [syms[i] for i in range(n_sym)], n_sym


def papr(signal: np.ndarray) -> dict:
    """OFDMTransmitter.calculate_papr (core/ofdm_core.py:114-147)."""
    p = np.abs(signal) ** 2
    pk, av = np.max(p), np.mean(p)
    if av > 0:
        lin = pk / av
        return {'papr_db': 10 * np.log10(lin), 'papr_linear': lin,
                'peak_power': pk, 'avg_power': av}
    return {'papr_db': 0.0, 'papr_linear': 1.0, 'peak_power': pk, 'avg_power': av}


# --------------------------------------------------------------------------
# Channel
def itu_paths(num: Numerology, profile: str, spatial: bool = False):
    """RayleighMultiPathChannel._get_itu_profile_params (core/channel.py:162-186)
    then RayleighChannel.__init__ (core/rayleighchannel.py:13-18): the dB->linear
    conversion is applied twice (quirk Q2); a third time for spatial links
    (core/channel.py:435-444).  Returns (integer delays, gains)."""
    if profile not in ITU_CHANNEL_MODELS:
        raise ValueError(f"Perfil ITU no encontrado: {profile}")
    d = ITU_CHANNEL_MODELS[profile]
    delays_s = np.array(d['delays_us']) * 1e-6
    g = 10 ** (np.array(d['power_db']) / 20)
    g = 10 ** (np.array(g) / 20)
    if spatial:
        g = 10 ** (np.array(g) / 20)
    dl = np.array([int(np.round(delays_s[i] * num.fs)) for i in range(len(delays_s))])
    return dl, g


def doppler_hz(frequency_ghz, velocity_kmh):
    """core/channel.py:113-143 (explicit freq & velocity branch)."""
    return (velocity_kmh / 3.6) * (frequency_ghz * 1e9) / 3e8


def jakes(phi: np.ndarray, fD: float, fs: float, n: int) -> np.ndarray:
    """RayleighChannel.jakes_fading (core/rayleighchannel.py:20-42) with the
    random phases passed in.  For fD == 0 the process is constant (the
    argument is exactly phi for every sample) so a length-1 evaluation is
    broadcast."""
    Ns = len(phi)
    m = n if fD != 0 else 1
    t = np.arange(m) / fs
    alpha = 2 * np.pi * np.arange(1, Ns + 1) / Ns
    h = np.zeros(m, dtype=complex)
    for i in range(Ns):
        h += np.exp(1j * (2 * np.pi * fD * np.cos(alpha[i]) * t + phi[i]))
    h = h * np.sqrt(2 / Ns)
    if m != n:
        h = np.broadcast_to(h, (n,))
    return h


def multipath(x: np.ndarray, delays, gains, phases, fD, fs) -> np.ndarray:
    """RayleighChannel.filter (core/rayleighchannel.py:44-58)."""
    n = len(x)
    y = np.zeros(n, dtype=complex)
    for i in range(len(delays)):
        fading = jakes(phases[i], fD, fs, n)
        xd = np.concatenate([np.zeros(delays[i]), x])[:n]
        y += gains[i] * fading * xd
    return y


def add_noise(y: np.ndarray, snr_db: float, z_re=None, z_im=None):
    """AWGNChannel.transmit / RayleighMultiPathChannel.transmit noise part
    (core/channel.py:44-66, 217-232): SNR referenced to the measured mean power
    of the whole stream (Q5).  z_* = unit normals (None -> draw from the global
    RNG exactly like the reference)."""
    snr_lin = 10 ** (snr_db / 10)
    p = np.mean(np.abs(y) ** 2)
    npow = p / snr_lin
    s = np.sqrt(npow / 2)
    if z_re is None:
        nr = np.random.normal(0, s, len(y))
        ni = np.random.normal(0, s, len(y))
    else:
        nr, ni = s * z_re, s * z_im
    return y + (nr + 1j * ni), npow


def channel_transmit(num, x, channel, snr_db, profile='Pedestrian_A', fD=0.0,
                     draws=None):
    """ChannelSimulator.transmit (core/channel.py:334-345) for 'awgn' and
    'rayleigh_mp'.  Draw order: per path rand(16), then normal(L) x 2."""
    if channel == 'rayleigh_mp':
        dl, g = itu_paths(num, profile)
        if draws is None:
            ph = [2 * np.pi * np.random.rand(16) for _ in range(len(dl))]
        else:
            ph = draws['phases']
        y = multipath(x, dl, g, ph, fD, num.fs)
    elif channel == 'awgn':
        y = x
    else:
        raise ValueError(f"Tipo de canal desconocido: {channel}")
    if draws is None:
        return add_noise(y, snr_db)[0]
    return add_noise(y, snr_db, draws['z_re'], draws['z_im'])[0]


def ref_compat_draws(num: Numerology, channel: str, L: int, n_rx: int = 1,
                     profile='Pedestrian_A'):
    """The random numbers one reference simulate_siso/_coded/_simo call consumes,
    in the reference's order, from the global RNG, leaving the global RNG in the
    same final state: TX pilot reseed (resource_mapper.py:148) -> per RX antenna
    [per path rand(16) (rayleighchannel.py:31), normal(L) re, normal(L) im
    (channel.py:227-228)] -> RX pilot reseed (lte_receiver.py:67)."""
    pilots(0, num.Np)
    out = []
    n_paths = len(ITU_CHANNEL_MODELS[profile]['delays_us']) if channel == 'rayleigh_mp' else 0
    for _ in range(n_rx):
        ph = [2 * np.pi * np.random.rand(16) for _ in range(n_paths)]
        zr = np.random.normal(0, 1.0, L)
        zi = np.random.normal(0, 1.0, L)
        out.append({'phases': ph, 'z_re': zr, 'z_im': zi})
    pilots(0, num.Np)
    return out


# --------------------------------------------------------------------------
# RX
def demod_stream(num: Numerology, y: np.ndarray) -> np.ndarray:
    """LTEReceiver._demodulate_ofdm_stream (core/lte_receiver.py:444-491)."""
    sl = num.N + num.cp
    n_sym = len(y) // sl
    if n_sym == 0:
        n_sym = 1
    if len(y) < n_sym * sl:
        y = np.pad(y, (0, n_sym * sl - len(y)), 'constant')
    blk = y[:n_sym * sl].reshape(n_sym, sl)[:, num.cp:]
    return np.fft.fft(blk, axis=1) / np.sqrt(num.N)


def interp_channel(pilot_idx, hp, N):
    """LTEChannelEstimator._interpolate_channel (core/lte_receiver.py:98-133):
    edge hold + np.linspace between pilots (vectorised, bit-identical)."""
    H = np.zeros(N, dtype=complex)
    H[:pilot_idx[0]] = hp[0]
    H[pilot_idx[-1]:] = hp[-1]
    for i in range(len(pilot_idx) - 1):
        a, b = pilot_idx[i], pilot_idx[i + 1]
        H[a:b + 1] = np.linspace(hp[i], hp[i + 1], b - a + 1)
    return H


def estimate_channel(num: Numerology, Y: np.ndarray, cell_id: int = 0):
    """LTEChannelEstimator.estimate_channel (core/lte_receiver.py:40-96)."""
    kp = pilots(cell_id, num.Np)
    rp = Y[num.pilot_idx]
    hp = rp / kp
    pp = np.mean(np.abs(rp) ** 2)
    en = np.mean(np.abs(rp - kp) ** 2)
    snr = pp / (en + 1e-10)
    return interp_channel(num.pilot_idx, hp, num.N), 10 * np.log10(snr + 1e-10)


def estimate_periodic(num: Numerology, Yf: np.ndarray, slot: int = 14):
    """LTEReceiver._estimate_channel_periodic (core/lte_receiver.py:360-411):
    estimate on symbol 0 of every 14-symbol group, reuse for the group (Q7)."""
    Hs, snrs = [], []
    for s0 in range(0, Yf.shape[0], slot):
        H, sdb = estimate_channel(num, Yf[s0])
        snrs.append(sdb)
        Hs.extend([H] * (min(s0 + slot, Yf.shape[0]) - s0))
    return Hs, (np.mean(snrs) if snrs else 0.0)


def receive(num: Numerology, y: np.ndarray, equalize=True, sc_fdm=False):
    """LTEReceiver.receive_and_decode data path (core/lte_receiver.py:259-333)
    + OFDMDemodulator.demodulate_stream (core/demodulator.py:138-147); sc_fdm:
    the IDFT matrix applied to each symbol's Nd equalised data REs (:318-333).
    Returns (data symbols, bits, channel_snr_db)."""
    Yf = demod_stream(num, y)
    Hs, snr_db = estimate_periodic(num, Yf)
    if equalize:
        eq = np.stack([Yf[i] / (Hs[i] + 1e-6) for i in range(Yf.shape[0])])   # Q8
    else:
        eq = Yf
    data = eq[:, num.data_idx]
    if sc_fdm:
        D = dft_matrix(num.Nd, inverse=True)
        data = np.stack([D @ data[i] for i in range(data.shape[0])])
    data = data.reshape(-1)
    return data, symbols_to_bits(data, num.modulation), snr_db


def simulate_siso(num: Numerology, bits, snr_db, channel='awgn',
                  profile='Pedestrian_A', fD=0.0, draws=None, sc_fdm=False, equalize=True):
    """OFDMSimulator.simulate_siso (core/ofdm_core.py:660-737).  draws=None
    consumes the global RNG like the reference; else uses the given draws.
    sc_fdm: DFT precoding at TX and IDFT after ZF at RX;
    equalize=False: OFDMSimulator(enable_equalization=False), no ZF (:294-299)."""
    bits = np.asarray(bits)
    if bits.size == 0:
        raise ValueError("Bits array cannot be empty")
    n0 = len(bits)
    sig, syms, n_sym = modulate_stream(num, bits, sc_fdm)
    pa = papr(sig)
    d = None if draws is None else draws[0]
    rx = channel_transmit(num, sig, channel, snr_db, profile, fD, d)
    data, brx, _ = receive(num, rx, equalize, sc_fdm)
    if draws is None:
        pass  # reseed already happened inside estimate_channel
    brx = np.pad(brx, (0, n0 - len(brx))) if len(brx) < n0 else brx[:n0]
    err = int(np.sum(bits != brx))
    return {'transmitted_bits': n0, 'received_bits': n0,
            'bits_received_array': brx, 'bit_errors': err, 'errors': err,
            'ber': float(err / n0), 'snr_db': float(snr_db),
            'papr_db': float(pa['papr_db']), 'papr_linear': float(pa['papr_linear']),
            'signal_tx': sig, 'signal_rx': rx, 'symbols_tx': syms,
            'symbols_rx': data}


def simulate_simo(num: Numerology, bits, snr_db, num_rx=2, channel='awgn',
                  profile='Pedestrian_A', fD=0.0, draws=None, sc_fdm=False):
    """OFDMSimulator.simulate_simo (core/ofdm_core.py:1536-1679) with
    transmit_simo (:361-412), _demodulate_with_channel_est (:1340-1403) and
    _combine_symbols_mrc (:1405-1534), hard decision on the MRC output.
    sc_fdm: the transmitter DFT-precodes but this receiver never applies the
    IDFT (the reference's behaviour, BER ~ 0.5)."""
    bits = np.asarray(bits)
    n0 = len(bits)
    sig, syms, n_sym = modulate_stream(num, bits, sc_fdm)
    pa = papr(sig)
    rxs = []
    for r in range(num_rx):
        d = None if draws is None else draws[r]
        rxs.append(channel_transmit(num, sig, channel, snr_db, profile, fD, d))
    num_acc = None
    den_acc = None
    for r in range(num_rx):
        Yf = demod_stream(num, rxs[r])
        Hs, _ = estimate_periodic(num, Yf)
        Y = Yf[:, num.data_idx].reshape(-1)
        H = np.stack(Hs)[:, num.data_idx].reshape(-1)
        if num_acc is None:
            num_acc = np.zeros(len(Y), dtype=complex)
            den_acc = np.zeros(len(Y), dtype=float)
        # The reference accumulates with NumPy *scalar* math per RE
        # (ofdm_core.py:1513-1525); the array loops use SIMD kernels that
        # round differently, so restate the scalar formulas exactly.
        hr, hi, yr, yi = H.real, -H.imag, Y.real, Y.imag
        prod = np.empty(len(Y), dtype=complex)
        prod.real = hr * yr - hi * yi
        prod.imag = hr * yi + hi * yr
        num_acc += prod
        den_acc += np.array([np.abs(h) ** 2 for h in H])
    comb = num_acc / (den_acc + 1e-10)                 # Q17
    brx = symbols_to_bits(comb, num.modulation)
    brx = np.pad(brx, (0, n0 - len(brx))) if len(brx) < n0 else brx[:n0]
    err = int(np.sum(bits != brx))
    return {'transmitted_bits': n0, 'received_bits': n0,
            'bits_received_array': brx, 'bit_errors': err, 'errors': err,
            'ber': float(err / n0), 'snr_db': float(snr_db),
            'papr_db': float(pa['papr_db']), 'papr_linear': float(pa['papr_linear']),
            'signal_tx': sig, 'signal_rx_list': rxs, 'symbols_tx': syms,
            'symbols_rx_combined': comb, 'num_rx': num_rx}


# --------------------------------------------------------------------------
# Soft demapping (core/ofdm_core.py:791-923)
def llrs(symbols: np.ndarray, noise_var: np.ndarray, mod: str) -> np.ndarray:
    if mod == 'QPSK':
        scale = np.sqrt(2)
        out = np.zeros(2 * len(symbols))
        out[0::2] = (2.0 / noise_var) * symbols.real * scale
        out[1::2] = (2.0 / noise_var) * symbols.imag * scale
        return out
    bps = BPS[mod]
    c = constellation(mod)
    M = len(c)
    bitmap = ((np.arange(M)[:, None] >> np.arange(bps - 1, -1, -1)[None, :]) & 1)
    noise_var = np.broadcast_to(noise_var, symbols.shape)
    out = np.zeros((len(symbols), bps))
    step = 4096
    for s in range(0, len(symbols), step):
        y = symbols[s:s + step]
        D = np.abs(y[:, None] - c[None, :]) ** 2
        for b in range(bps):
            m0 = D[:, bitmap[:, b] == 0].min(axis=1)
            m1 = D[:, bitmap[:, b] == 1].min(axis=1)
            out[s:s + step, b] = np.clip((m1 - m0) / (2.0 * noise_var[s:s + step]), -10.0, 10.0)
    return out.reshape(-1)


# --------------------------------------------------------------------------
# Channel coding (core/channel_coding/)
_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, '_build', 'liboracle.so')
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        P = ctypes.POINTER
        L.or_crc.restype = ctypes.c_uint32
        L.or_crc.argtypes = [P(ctypes.c_uint8), ctypes.c_int64, ctypes.c_uint32, ctypes.c_int]
        L.or_rsc_encode.argtypes = [P(ctypes.c_uint8), ctypes.c_int, P(ctypes.c_uint8), P(ctypes.c_uint8)]
        L.or_turbo_decode.argtypes = [P(ctypes.c_double), ctypes.c_int, ctypes.c_int,
                                      P(ctypes.c_int32), P(ctypes.c_uint8), P(ctypes.c_double)]
        L.or_bcjr_maxlog.argtypes = [P(ctypes.c_double)] * 3 + [ctypes.c_int, P(ctypes.c_double), P(ctypes.c_double)]
        L.or_turbo_decode_f32.argtypes = [P(ctypes.c_float), ctypes.c_int, ctypes.c_int, P(ctypes.c_int32),
                                          P(ctypes.c_uint8)]
        L.or_bcjr_scratch_doubles.restype = ctypes.c_size_t
        L.or_bcjr_scratch_doubles.argtypes = [ctypes.c_int]
        _lib = L
    return _lib


def build():
    import subprocess
    subprocess.check_call(['make', '-s', '-C', _HERE])


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


CRC24A_POLY = 0x1864CFB
CRC24B_POLY = 0x1800063
CRC16_POLY = 0x11021


def crc_bits(bits, poly, length):
    """_calculate_crc (core/channel_coding/crc.py:89-134) -> CRC bits MSB-first."""
    b = np.ascontiguousarray(np.asarray(bits).astype(np.uint8))
    v = lib().or_crc(_p(b, ctypes.c_uint8), len(b), poly, length)
    return np.array([(v >> (length - 1 - i)) & 1 for i in range(length)], dtype=np.uint8)


def attach_crc24a(bits):
    """crc.py:212-233"""
    return np.concatenate([np.asarray(bits), crc_bits(bits, CRC24A_POLY, 24)])


def check_crc24a(bits):
    """crc.py:277-307"""
    bits = np.asarray(bits)
    if len(bits) < 24:
        return False
    return bool(np.array_equal(bits[-24:], crc_bits(bits[:-24], CRC24A_POLY, 24)))


TURBO_SIZES = ([40 + 8 * i for i in range(60)] + [528 + 16 * i for i in range(32)] +
               [1056 + 32 * i for i in range(32)] + [2112 + 64 * i for i in range(64)])
# segmentation.py:34-50 (188 sizes)
QPP = {}


def _load_qpp():
    """QPP_INTERLEAVER_PARAMS (turbo_encoder.py:34-73), 3GPP TS 36.212 Table 5.1.3-3."""
    t = [(40, 3, 10), (48, 7, 12), (56, 19, 42), (64, 7, 16), (72, 7, 18), (80, 11, 20),
         (88, 5, 22), (96, 11, 24), (104, 7, 26), (112, 41, 84), (120, 103, 90), (128, 15, 32),
         (136, 9, 34), (144, 17, 108), (152, 9, 38), (160, 21, 120), (168, 101, 84), (176, 21, 44),
         (184, 57, 46), (192, 23, 48), (200, 13, 50), (208, 27, 52), (216, 11, 36), (224, 27, 56),
         (232, 85, 58), (240, 29, 60), (248, 33, 62), (256, 15, 32), (264, 17, 198), (272, 33, 68),
         (280, 103, 210), (288, 19, 36), (296, 19, 74), (304, 37, 76), (312, 19, 78), (320, 21, 120),
         (328, 21, 82), (336, 115, 84), (344, 193, 86), (352, 21, 44), (360, 133, 90), (368, 81, 46),
         (376, 45, 94), (384, 23, 48), (392, 243, 98), (400, 151, 40), (408, 155, 102), (416, 25, 52),
         (424, 51, 106), (432, 47, 72), (440, 91, 110), (448, 29, 168), (456, 29, 114), (464, 247, 58),
         (472, 29, 118), (480, 89, 180), (488, 91, 122), (496, 157, 62), (504, 55, 84), (512, 31, 64),
         (528, 17, 66), (544, 35, 68), (560, 227, 420), (576, 65, 96), (592, 19, 74), (608, 37, 76),
         (624, 41, 234), (640, 39, 80), (656, 185, 82), (672, 43, 252), (688, 21, 86), (704, 155, 44),
         (720, 79, 120), (736, 139, 92), (752, 23, 94), (768, 217, 48), (784, 25, 98), (800, 17, 80),
         (816, 127, 102), (832, 25, 52), (848, 239, 106), (864, 17, 48), (880, 137, 110), (896, 215, 112),
         (912, 29, 114), (928, 15, 58), (944, 147, 118), (960, 29, 60), (976, 59, 122), (992, 65, 124),
         (1008, 55, 84), (1024, 31, 64), (1056, 17, 66), (1088, 171, 204), (1120, 67, 140),
         (1152, 35, 72), (1184, 19, 74), (1216, 39, 76), (1248, 19, 78), (1280, 199, 240),
         (1312, 21, 82), (1344, 211, 252), (1376, 21, 86), (1408, 43, 88), (1440, 149, 60),
         (1472, 45, 92), (1504, 49, 846), (1536, 71, 48), (1568, 13, 28), (1600, 17, 80),
         (1632, 25, 102), (1664, 183, 104), (1696, 55, 954), (1728, 127, 96), (1760, 27, 110),
         (1792, 29, 112), (1824, 29, 114), (1856, 57, 116), (1888, 45, 354), (1920, 31, 120),
         (1952, 59, 610), (1984, 185, 124), (2016, 113, 420), (2048, 31, 64), (2112, 17, 66),
         (2176, 171, 136), (2240, 209, 420), (2304, 253, 216), (2368, 367, 444), (2432, 265, 456),
         (2496, 181, 468), (2560, 39, 80), (2624, 27, 164), (2688, 127, 504), (2752, 143, 172),
         (2816, 43, 88), (2880, 29, 300), (2944, 45, 92), (3008, 157, 188), (3072, 47, 96),
         (3136, 13, 28), (3200, 111, 240), (3264, 443, 204), (3328, 51, 104), (3392, 51, 212),
         (3456, 451, 192), (3520, 257, 220), (3584, 57, 336), (3648, 313, 228), (3712, 271, 232),
         (3776, 179, 236), (3840, 331, 120), (3904, 363, 244), (3968, 375, 248), (4032, 127, 168),
         (4096, 31, 64), (4160, 33, 130), (4224, 43, 264), (4288, 33, 134), (4352, 477, 408),
         (4416, 35, 138), (4480, 233, 280), (4544, 357, 142), (4608, 337, 480), (4672, 37, 146),
         (4736, 71, 444), (4800, 71, 120), (4864, 37, 152), (4928, 39, 462), (4992, 127, 234),
         (5056, 39, 158), (5120, 39, 80), (5184, 31, 96), (5248, 113, 902), (5312, 41, 166),
         (5376, 251, 336), (5440, 43, 170), (5504, 21, 86), (5568, 43, 174), (5632, 45, 176),
         (5696, 45, 178), (5760, 161, 120), (5824, 89, 182), (5888, 323, 184), (5952, 47, 186),
         (6016, 23, 94), (6080, 47, 190), (6144, 263, 480)]
    for K, f1, f2 in t:
        QPP[K] = (f1, f2)


_load_qpp()


def qpp_perm(K):
    """qpp_interleave indices (turbo_encoder.py:76-102): pi(i) = (f1 i + f2 i^2) mod K."""
    if K not in QPP:
        raise ValueError(f"Invalid interleaver size K={K}")
    f1, f2 = QPP[K]
    i = np.arange(K, dtype=np.int64)
    return ((f1 * i + f2 * i * i) % K).astype(np.int32)


def find_interleaver_size(n):
    """segmentation.py:53-71"""
    for s in TURBO_SIZES:
        if s >= n:
            return s
    raise ValueError(f"No valid interleaver size found for min_size={n}")


def segmentation_plan(B):
    """segment_code_blocks metadata (segmentation.py:74-263): returns list of
    (K_r, F_r, info_r, offset_r, has_crc24b)."""
    Z = 6144
    if B <= Z:
        K = find_interleaver_size(B)
        return [(K, K - B, B, 0, False)]
    L = 24
    C = int(np.ceil(B / (Z - L)))
    Bp = B + C * L
    Kp = find_interleaver_size(int(np.ceil(Bp / C)))
    km = TURBO_SIZES.index(Kp) - 1
    Km = TURBO_SIZES[km] if km >= 0 else Kp
    dK = Kp - Km
    Cm = (C * Kp - Bp) // dK if dK > 0 else 0
    plan, rem, off = [], B, 0
    for r in range(C):
        K = Km if r < Cm else Kp
        avail = K - L
        info = rem if r == C - 1 else min(avail, rem // (C - r))
        rem -= info
        plan.append((K, (K - L) - info, info, off, True))
        off += info
    return plan


def segment(tb_with_crc):
    """segment_code_blocks (segmentation.py:74-263): filler at the front of each
    block, CRC-24B appended when segmented (Q12)."""
    tb = np.asarray(tb_with_crc)
    plan = segmentation_plan(len(tb))
    out = []
    for K, F, info, off, crc in plan:
        if not crc:
            cb = np.zeros(K, dtype=np.uint8)
            cb[F:] = tb
        else:
            c = np.zeros(K - 24, dtype=np.uint8)
            c[F:F + info] = tb[off:off + info]
            cb = np.concatenate([c, crc_bits(c, CRC24B_POLY, 24)])
        out.append(cb)
    return out, plan


def desegment(blocks, plan):
    """desegment_code_blocks (segmentation.py:266-359); CRC-24B not checked."""
    parts = []
    for cb, (K, F, info, off, crc) in zip(blocks, plan):
        if not crc:
            parts.append(cb[F:F + info])
        else:
            parts.append(cb[:-24][F:F + info])
    return np.concatenate(parts)


def rsc_encode(bits):
    """rsc_encode (turbo_encoder.py:137-211), via C."""
    b = np.ascontiguousarray(np.asarray(bits).astype(np.uint8))
    K = len(b)
    s = np.zeros(K + 3, dtype=np.uint8)
    p = np.zeros(K + 3, dtype=np.uint8)
    lib().or_rsc_encode(_p(b, ctypes.c_uint8), K, _p(s, ctypes.c_uint8), _p(p, ctypes.c_uint8))
    return s, p


def turbo_encode(cb):
    """turbo_encode (turbo_encoder.py:214-313): output [d0_k d1_k d2_k]*K then
    [sys1(3) par1(3) sys2(3) par2(3)] (Q13)."""
    cb = np.asarray(cb).astype(np.uint8)
    K = len(cb)
    if K not in QPP:
        raise ValueError(f"Invalid code block size K={K}. Must be valid interleaver size.")
    s1, p1 = rsc_encode(cb)
    s2, p2 = rsc_encode(cb[qpp_perm(K)])
    out = np.zeros(3 * K + 12, dtype=np.uint8)
    out[0:3 * K:3] = s1[:K]
    out[1:3 * K:3] = p1[:K]
    out[2:3 * K:3] = p2[:K]
    out[3 * K:3 * K + 3] = s1[K:]
    out[3 * K + 3:3 * K + 6] = p1[K:]
    out[3 * K + 6:3 * K + 9] = s2[K:]
    out[3 * K + 9:3 * K + 12] = p2[K:]
    return out


_SBI_P = np.array([0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30,
                   1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31])


def subblock_perm(n):
    """sub_block_interleaver as an index map (rate_matching.py:25-94): column
    fill R x 32, permute columns by P, row read, NULLs dropped: v[i] = d[perm[i]]."""
    R = int(np.ceil(n / 32))
    rows = np.repeat(np.arange(R), 32)
    cols = np.tile(_SBI_P, R)
    idx = cols * R + rows
    return idx[idx < n]


def rm_params(K, rv_idx=0):
    """Circular buffer geometry (rate_matching.py:249-290)."""
    ml = K + 6
    Ncb = 3 * ml
    start = [0, Ncb // 4, Ncb // 2, 3 * Ncb // 4][rv_idx % 4]
    return ml, Ncb, start


def rate_match(enc, E, K, rv_idx=0):
    """rate_match_turbo (rate_matching.py:193-297)."""
    enc = np.asarray(enc)
    if len(enc) != 3 * K + 12:
        raise ValueError(f"Invalid encoded_bits length. Expected {3*K + 12}, got {len(enc)}")
    d0 = np.concatenate([enc[0:3 * K:3], enc[3 * K:3 * K + 3], enc[3 * K + 6:3 * K + 9]])
    d1 = np.concatenate([enc[1:3 * K:3], enc[3 * K + 3:3 * K + 6]])
    d2 = np.concatenate([enc[2:3 * K:3], enc[3 * K + 9:3 * K + 12]])
    ml, Ncb, start = rm_params(K, rv_idx)
    cb = np.zeros(Ncb, dtype=np.uint8)
    cb[0::3] = d0[subblock_perm(K + 6)]
    cb[1:3 * (K + 3):3] = d1[subblock_perm(K + 3)]
    cb[2:3 * (K + 3):3] = d2[subblock_perm(K + 3)]
    return cb[(start + np.arange(E)) % Ncb]


def rate_dematch(llr, K, rv_idx=0):
    """rate_dematching_turbo (rate_matching.py:374-489): soft-combine into the
    circular buffer, unzip, inverse sub-block interleave; the 2 never-sent
    systematic positions keep LLR 0 (Q14)."""
    llr = np.asarray(llr, dtype=np.float64)
    ml, Ncb, start = rm_params(K, rv_idx)
    cb = np.zeros(Ncb)
    pos = (start + np.arange(len(llr))) % Ncb
    np.add.at(cb, pos, llr)
    v0 = cb[0::3][:K + 6]
    v1 = cb[1::3][:K + 3]
    v2 = cb[2::3][:K + 3]
    d0 = np.zeros(K + 6)
    d1 = np.zeros(K + 3)
    d2 = np.zeros(K + 3)
    d0[subblock_perm(K + 6)] = v0
    d1[subblock_perm(K + 3)] = v1
    d2[subblock_perm(K + 3)] = v2
    out = np.zeros(3 * K + 12)
    out[0:3 * K:3] = d0[:K]
    out[1:3 * K:3] = d1[:K]
    out[2:3 * K:3] = d2[:K]
    out[3 * K:3 * K + 3] = d0[K:K + 3]
    out[3 * K + 6:3 * K + 9] = d0[K + 3:K + 6]
    out[3 * K + 3:3 * K + 6] = d1[K:K + 3]
    out[3 * K + 9:3 * K + 12] = d2[K:K + 3]
    return out


def turbo_decode(llr, K, num_iterations=5, trace=False):
    """turbo_decode (turbo_decoder.py:338-450), max-log, via C (bit-exact f64)."""
    L = np.ascontiguousarray(np.asarray(llr, dtype=np.float64))
    perm = np.ascontiguousarray(qpp_perm(K))
    out = np.zeros(K, dtype=np.uint8)
    tr = np.zeros((num_iterations, K)) if trace else None
    lib().or_turbo_decode(_p(L, ctypes.c_double), K, num_iterations, _p(perm, ctypes.c_int32),
                          _p(out, ctypes.c_uint8),
                          _p(tr, ctypes.c_double) if trace else None)
    return (out, tr) if trace else out


def turbo_decode_f32_model(llr, K, num_iterations=8):
    """Kernel-verification model: the GPU decoder's float32 algorithm
    (coding_oracle.c or_turbo_decode_f32).  Not the reference semantics."""
    L = np.ascontiguousarray(np.asarray(llr, dtype=np.float32))
    perm = np.ascontiguousarray(qpp_perm(K))
    out = np.zeros(K, dtype=np.uint8)
    lib().or_turbo_decode_f32(_p(L, ctypes.c_float), K, num_iterations, _p(perm, ctypes.c_int32),
                              _p(out, ctypes.c_uint8))
    return out


def bcjr_app(ls, lp, la):
    """LogMAPDecoder.decode a-posteriori output (turbo_decoder.py:181-278)."""
    n = len(ls)
    a = [np.ascontiguousarray(np.asarray(x, dtype=np.float64)) for x in (ls, lp, la)]
    out = np.zeros(n)
    scr = np.zeros(lib().or_bcjr_scratch_doubles(n))
    lib().or_bcjr_maxlog(*[_p(x, ctypes.c_double) for x in a], n, _p(out, ctypes.c_double),
                         _p(scr, ctypes.c_double))
    return out


# --------------------------------------------------------------------------
def tf_interleave_perm(n_syms, cols):
    """T/F block interleaver (core/ofdm_core.py:1040-1060): write rows of `cols`,
    read columns.  Returns (perm, rows, total) with interleaved[j] = padded[perm[j]]."""
    rows = int(np.ceil(n_syms / cols))
    total = rows * cols
    perm = np.arange(total).reshape(rows, cols).T.reshape(-1)
    return perm, rows, total


def noise_var_per_symbol(H, snr_db, channel):
    """core/ofdm_core.py:1224-1243 (nominal sigma^2, clipped ZF amplification)."""
    s2 = 1.0 / (10 ** (snr_db / 10))
    if channel == 'awgn':
        return np.full(len(H), s2)
    hp = np.clip(np.abs(H) ** 2, 1e-6, 1e6)
    return np.maximum(s2 / hp, s2 / 4.0)


def coded_tx(num: Numerology, bits):
    """TX coding chain of simulate_siso_coded (core/ofdm_core.py:1003-1099)."""
    tbc = attach_crc24a(np.asarray(bits))
    cbs, plan = segment(tbc)
    rms = []
    for cb in cbs:
        enc = turbo_encode(cb)
        rms.append(rate_match(enc, len(enc), len(cb), 0))
    coded = np.concatenate(rms)
    qam = bits_to_symbols(coded, num.modulation)
    perm, rows, total = tf_interleave_perm(len(qam), num.Nd)
    padded = np.pad(qam, (0, total - len(qam))) if len(qam) < total else qam[:total]
    inter = padded[perm]
    n_ofdm = int(np.ceil(len(inter) / num.Nd))
    ds = np.pad(inter, (0, n_ofdm * num.Nd - len(inter))).reshape(n_ofdm, num.Nd)
    pil = pilots(0, num.Np)
    sig = ofdm_symbols_tx(num, ds, pil)
    return {'signal': sig, 'qam': qam, 'coded': coded, 'cbs': cbs, 'plan': plan,
            'rm_lens': [len(r) for r in rms], 'n_ofdm': n_ofdm}


def coded_rx_llrs(num: Numerology, rx, coded_len, snr_db, channel):
    """RX front end of simulate_siso_coded up to the LLRs (core/ofdm_core.py:1116-1261)."""
    Yf = demod_stream(num, rx)
    Hs, snr_est = estimate_periodic(num, Yf)
    eq = np.stack([Yf[i] / (Hs[i] + 1e-6) for i in range(Yf.shape[0])])
    Hd = np.stack(Hs)[:, num.data_idx].reshape(-1)
    sy = eq[:, num.data_idx].reshape(-1)
    ncs = coded_len // num.bps
    cols = num.Nd
    rows = int(np.ceil(ncs / cols))
    total = rows * cols
    if len(sy) < total:
        sy = np.pad(sy, (0, total - len(sy)))
        Hd = np.pad(Hd, (0, total - len(Hd)), 'edge')
    else:
        sy, Hd = sy[:total], Hd[:total]
    sd = sy.reshape(cols, rows).T.reshape(-1)[:ncs]
    hd = Hd.reshape(cols, rows).T.reshape(-1)[:ncs]
    nv = noise_var_per_symbol(hd, snr_db, channel)
    L = llrs(sd, nv, num.modulation)
    if len(L) > coded_len:
        L = L[:coded_len]
    elif len(L) < coded_len:
        L = np.pad(L, (0, coded_len - len(L)))
    return L, sd, hd, nv, snr_est


def coded_rx_decode(L, plan, rm_lens, iters=8, f32_model=False):
    """RX decoding chain (core/ofdm_core.py:1267-1299).  f32_model=True swaps
    the float64 reference decoder for the GPU kernel's float32 model."""
    off = 0
    dec = []
    for (K, F, info, o, crc), E in zip(plan, rm_lens):
        dm = rate_dematch(L[off:off + E], K, 0)
        off += E
        dec.append(turbo_decode_f32_model(dm, K, iters) if f32_model else turbo_decode(dm, K, iters))
    tbc = desegment(dec, plan)
    ok = check_crc24a(tbc)
    return (tbc[:-24] if len(tbc) >= 24 else tbc), ok


def simulate_siso_coded(num: Numerology, bits, snr_db, channel='awgn',
                        profile='Pedestrian_A', fD=0.0, draws=None, iters=8):
    """OFDMSimulator.simulate_siso_coded (core/ofdm_core.py:925-1338)."""
    bits = np.asarray(bits)
    if bits.size == 0:
        raise ValueError("Bits array cannot be empty")
    n0 = len(bits)
    tx = coded_tx(num, bits)
    pa = papr(tx['signal'])
    d = None if draws is None else draws[0]
    rx = channel_transmit(num, tx['signal'], channel, snr_db, profile, fD, d)
    L, sd, hd, nv, snr_est = coded_rx_llrs(num, rx, len(tx['coded']), snr_db, channel)
    dec, ok = coded_rx_decode(L, tx['plan'], tx['rm_lens'], iters)
    dec = np.pad(dec, (0, n0 - len(dec))) if len(dec) < n0 else dec[:n0]
    err = int(np.sum(bits != dec))
    return {'transmitted_bits': n0, 'received_bits': n0, 'bits_received_array': dec,
            'bit_errors': err, 'ber': float(err / n0), 'crc_pass': bool(ok),
            'snr_db': float(snr_db), 'papr_db': float(pa['papr_db']),
            'papr_linear': float(pa['papr_linear']), 'coded_bits_length': len(tx['coded']),
            'signal_tx': tx['signal'], 'signal_rx': rx, 'symbols_tx': tx['qam'],
            'symbols_rx': sd, 'H_estimate': hd, 'channel_snr_db': float(snr_est),
            'noise_var_mean': float(np.mean(nv)), 'llrs': L}
