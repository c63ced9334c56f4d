"""ORACLE — TEST INFRASTRUCTURE ONLY.

NumPy restatement of the device random streams of the Philox mode
(``bench.py``, ``OFDMSimulator.run_grid``): Philox4x32-10 and the mapping of
its outputs onto the reference's random draws, so that any frame the bench
times can be re-run on the CPU by ``lte_oracle`` with exactly the same inputs.

* Philox4x32-10 (Salmon et al., "Parallel random numbers: as easy as 1, 2, 3",
  SC'11; the Random123 reference constants).  Pinned by the published
  known-answer vectors (``tests/test_oracle_philox.py``) and, on the GPU, by the
  device's own outputs (``lte_philox_host``, ``tests/test_gpu_philox.py``).
  Device code: ``ofdm-lte_amd/csrc/lte_common.h`` ``philox4x32`` / ``rng4``.
* Counter = (index, stream, frame_lo, frame_hi), key = (seed_lo, seed_hi).
* What each stream feeds (the reference draw it replaces):
  - payload bits (``bits = np.random.randint(0, 2, n)`` in the reference's
    callers): word i of a frame = output (i mod 4) of counter i // 4 on
    ``STREAM_BITS``, MSB first (``k_payload``, lte_kernels.hip);
  - Jakes phases (``2*pi*np.random.rand(16)`` per path,
    core/rayleighchannel.py:31): phase m of (rx, path) = 2 pi (u + 0.5) 2^-32,
    u = output (m mod 4) of counter m // 4 on ``STREAM_FADE + 64 rx + path``
    (``k_fading``);
  - AWGN (``np.random.normal`` x 2, core/channel.py:227-228): stream sample n
    of RX r = the unit normal pair formed from outputs (x, y) (n even) or
    (z, w) (n odd) of counter n // 2 on ``STREAM_NOISE + r``, Box-Muller
    z = sqrt(-2 ln u) (cos 2 pi v, sin 2 pi v), u, v = (a + 0.5) 2^-32
    (``load_symbol_noisy2``, lte_dev.h).  The oracle forms it with libm
    (NumPy) float64 log / sqrt / cos / sin; the device's table-driven
    ``box_muller64t`` is checked against this formula
    (``tests/test_gpu_philox.py``).
  The reference consumes these as float64 values exactly like the injected
  draws of ref-compat mode (``lte_oracle.ref_compat_draws``), so
  ``lte_oracle.simulate_siso_coded(..., draws=siso_draws(...))`` is the
  reference's computation on the bench's own random numbers.
"""
from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = np.uint64(0xFFFFFFFF)

# lte_common.h RNG_STREAM_*
STREAM_BITS = 1
STREAM_FADE = 0x100          # + rx * 64 + path
STREAM_NOISE = 0x10000       # + rx
STREAM_MIMO_FADE = 0x20000   # + link * n_paths + path, link = rx * num_tx + tx
STREAM_MIMO_LINK = 0x30000   # + link
STREAM_BF = 0x40000          # + rx * num_tx + tx

TWO_M32 = 2.3283064365386962890625e-10   # 2^-32
TWO_PI = 6.283185307179586


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 on uint32 counter arrays (broadcast), key (k0, k1).
    Returns the four uint32 output words (lte_common.h philox4x32)."""
    c = [np.asarray(x, dtype=np.uint64) & MASK for x in (c0, c1, c2, c3)]
    c = list(np.broadcast_arrays(*c))
    k0, k1 = int(k0) & 0xFFFFFFFF, int(k1) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c[0]
        p1 = M1 * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        c = [hi1 ^ c[1] ^ np.uint64(k0), lo1, hi0 ^ c[3] ^ np.uint64(k1), lo0]
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return [x.astype(np.uint32) for x in c]


def rng4(seed: int, frame: int, stream: int, idx) -> np.ndarray:
    """rng4(seed, frame, stream, idx) of lte_common.h: [4, len(idx)] uint32."""
    idx = np.atleast_1d(np.asarray(idx, dtype=np.uint64))
    frame, seed = int(frame), int(seed)
    out = philox4x32_10(idx, np.uint64(stream), np.uint64(frame & 0xFFFFFFFF), np.uint64(frame >> 32),
                        seed & 0xFFFFFFFF, seed >> 32)
    return np.stack(out)


def payload_words(seed: int, frame: int, n_bits: int) -> np.ndarray:
    """The frame's payload words (k_payload): word i = output i % 4 of counter i // 4."""
    nwd = (n_bits + 31) // 32
    r = rng4(seed, frame, STREAM_BITS, np.arange((nwd + 3) // 4))
    return r.T.reshape(-1)[:nwd]


def payload_bits(seed: int, frame: int, n_bits: int) -> np.ndarray:
    """Payload bits, MSB first within each word: uint8 [n_bits]."""
    w = payload_words(seed, frame, n_bits)
    sh = np.arange(31, -1, -1, dtype=np.uint32)
    return ((w[:, None] >> sh[None, :]) & np.uint32(1)).astype(np.uint8).reshape(-1)[:n_bits]


def uniform_phase(u: np.ndarray) -> np.ndarray:
    """k_fading's float64 phase from a 32-bit output: 2 pi (u + 0.5) 2^-32."""
    return TWO_PI * ((u.astype(np.float64) + 0.5) * TWO_M32)


def fade_phases(seed: int, frame: int, rx: int, n_paths: int) -> np.ndarray:
    """Jakes phases [n_paths][16] of one RX (k_fading)."""
    out = np.empty((n_paths, 16))
    for p in range(n_paths):
        r = rng4(seed, frame, STREAM_FADE + 64 * rx + p, np.arange(4))
        out[p] = uniform_phase(r.T.reshape(-1))   # m = 4 * counter + component
    return out


def box_muller(a: np.ndarray, b: np.ndarray):
    """libm float64 Box-Muller of two 32-bit outputs: (r cos t, r sin t),
    r = sqrt(-2 ln u), t = 2 pi v, u, v = (a + 0.5) 2^-32 (both in (0, 1))."""
    u = (a.astype(np.float64) + 0.5) * TWO_M32
    v = (b.astype(np.float64) + 0.5) * TWO_M32
    r = np.sqrt(-2.0 * np.log(u))
    t = TWO_PI * v
    return r * np.cos(t), r * np.sin(t)


def normals(seed: int, frame: int, stream: int, n: int):
    """Unit normal pairs of samples 0..n-1 on one stream (sample n from
    counter n // 2, outputs (x, y) for even n, (z, w) for odd n)."""
    r = rng4(seed, frame, stream, np.arange((n + 1) // 2))
    e_re, e_im = box_muller(r[0], r[1])
    o_re, o_im = box_muller(r[2], r[3])
    z_re = np.empty(2 * len(e_re))
    z_im = np.empty(2 * len(e_re))
    z_re[0::2], z_re[1::2] = e_re, o_re
    z_im[0::2], z_im[1::2] = e_im, o_im
    return z_re[:n], z_im[:n]


def siso_draws(seed: int, frame: int, L: int, n_paths: int, n_rx: int = 1):
    """The draws of one SISO / SIMO frame in lte_oracle's `draws` format: per RX
    {'phases': [n_paths x 16], 'z_re': [L], 'z_im': [L]}."""
    out = []
    for r in range(n_rx):
        ph = fade_phases(seed, frame, r, n_paths) if n_paths else np.zeros((0, 16))
        zr, zi = normals(seed, frame, STREAM_NOISE + r, L)
        out.append({'phases': [ph[p] for p in range(n_paths)], 'z_re': zr, 'z_im': zi})
    return out


# --------------------------------------------------------------------------
# Multi-antenna links (lte_mimo.hip k_fading_mimo / link_noise_at): link = rx *
# num_tx + tx; path p of a Rayleigh link on STREAM_MIMO_FADE + link * n_paths + p
# (phase m = output m % 4 of counter m // 4, as k_fading); the 100 dB link noise
# of transmit_mimo on STREAM_MIMO_LINK + link (samples as the RX noise; the RX
# streams take one draw per RX on link (r, 0)'s stream, of standard deviation
# sqrt(sum_t s_rt^2): mimo_oracle.transmit_mimo 'combined_link_noise'); a flat
# spatial link h ~ CN(0, 1) = normal(0, 1/sqrt 2) re, im from outputs (x, y) of
# counter 0x7FFFFFFF on STREAM_MIMO_LINK + link; RX noise on STREAM_NOISE + rx.
def mimo_phases(seed: int, frame: int, link: int, n_paths: int) -> np.ndarray:
    out = np.empty((n_paths, 16))
    for p in range(n_paths):
        r = rng4(seed, frame, STREAM_MIMO_FADE + link * n_paths + p, np.arange(4))
        out[p] = uniform_phase(r.T.reshape(-1))
    return out


def flat_link_h(seed: int, frame: int, link: int) -> complex:
    r = rng4(seed, frame, STREAM_MIMO_LINK + link, [0x7FFFFFFF])
    zr, zi = box_muller(r[0], r[1])
    s = 1 / np.sqrt(2)
    return complex(s * zr[0], s * zi[0])


def sfbc_draws(seed: int, frame: int, L: int, num_rx: int, n_paths: int, num_tx: int = 2, merged: bool = False):
    """transmit_mimo's draws (mimo_oracle.transmit_mimo format), Rayleigh links.
    merged: config 4's full chain on the device (no capture of the received
    streams / noise powers): the link noise folded into the RX noise draw
    (lte_internal.h launch_npow_sfbc_merged; the link draws are then unused)."""
    out = []
    for r in range(num_rx):
        links = []
        for t in range(num_tx):
            link = r * num_tx + t
            ph = mimo_phases(seed, frame, link, n_paths)
            zr, zi = normals(seed, frame, STREAM_MIMO_LINK + link, L)
            links.append({'phases': [ph[p] for p in range(n_paths)], 'z_re': zr, 'z_im': zi})
        zr, zi = normals(seed, frame, STREAM_NOISE + r, L)
        out.append({'links': links, 'z_re': zr, 'z_im': zi, 'combined_link_noise': True, 'merged_link_noise': merged})
    return out


def sm_draws(seed: int, frame: int, L: int, num_tx: int, num_rx: int, channel: str, n_paths: int = 0):
    """transmit_spatial_multiplexing's draws (mimo_oracle.transmit_sm format).
    The impulse-response phases only form the reported channel_matrix (zeros)."""
    links = []
    for r in range(num_rx):
        row = []
        for t in range(num_tx):
            link = r * num_tx + t
            if channel == 'rayleigh_mp':
                ph = mimo_phases(seed, frame, link, n_paths)
                row.append({'phases': [ph[p] for p in range(n_paths)], 'ir_phases': [np.zeros(16)] * n_paths})
            else:
                row.append({'h': flat_link_h(seed, frame, link)})
        links.append(row)
    noise = []
    for r in range(num_rx):
        zr, zi = normals(seed, frame, STREAM_NOISE + r, L)
        noise.append({'z_re': zr, 'z_im': zi})
    return {'links': links, 'noise': noise}


# --------------------------------------------------------------------------
# Bench frames through the oracle
BENCH_SEED = 0x5EED
BENCH_SNRS = np.arange(0, 31, 2, dtype=np.float64)
BENCH_TB = 27760


def bench_snr(frame: int) -> float:
    """bench.py / lte_phy.dist.snr_index: frame id mod 16 on the 0:2:30 dB grid."""
    return float(BENCH_SNRS[int(frame) % len(BENCH_SNRS)])


def config2_frame(frame: int, seed: int = BENCH_SEED, snr_db=None, fD: float = 0.0):
    """One config-2 bench frame (SISO 20 MHz 64-QAM PedA + turbo x8, TB 27 760)
    through the float64 oracle on its Philox draws.  Returns (bit_errors, crc_ok)."""
    from . import lte_oracle as O
    num = O.Numerology(bandwidth=20.0, modulation='64-QAM')
    L = 14 * (num.N + num.cp)
    bits = payload_bits(seed, frame, BENCH_TB)
    snr = bench_snr(frame) if snr_db is None else float(snr_db)
    r = O.simulate_siso_coded(num, bits, snr, 'rayleigh_mp', fD=fD, draws=siso_draws(seed, frame, L, 4))
    return int(r['bit_errors']), bool(r['crc_pass'])


def config3_frame(frame: int, seed: int = BENCH_SEED, snr_db=None):
    """Config 3 (SIMO 1x4 MRC, 10 MHz 16-QAM, Vehicular-A, 14 symbols = 27 944
    bits, uncoded): simulate_simo on the frame's Philox draws.  (bit_errors, None)."""
    from . import lte_oracle as O
    num = O.Numerology(bandwidth=10.0, modulation='16-QAM')
    L = 14 * (num.N + num.cp)
    nb = 14 * num.Nd * num.bps
    snr = bench_snr(frame) if snr_db is None else float(snr_db)
    r = O.simulate_simo(num, payload_bits(seed, frame, nb), snr, 4, 'rayleigh_mp', 'Vehicular_A',
                        draws=siso_draws(seed, frame, L, 6, 4))
    return int(r['bit_errors']), None


def config4_frame(frame: int, seed: int = BENCH_SEED, snr_db=None):
    """Config 4 (SFBC 2x2 + turbo, 20 MHz 64-QAM PedA, TB 27 760): the oracle's
    composition (mimo_oracle.simulate_sfbc_coded) on the frame's Philox draws."""
    from . import lte_oracle as O, mimo_oracle as M
    num = O.Numerology(bandwidth=20.0, modulation='64-QAM')
    L = 14 * (num.N + num.cp)
    snr = bench_snr(frame) if snr_db is None else float(snr_db)
    r = M.simulate_sfbc_coded(num, payload_bits(seed, frame, BENCH_TB), snr, 2, 'rayleigh_mp',
                              draws=sfbc_draws(seed, frame, L, 2, 4, merged=True))
    return int(r['bit_errors']), bool(r['crc_pass'])


def config5_frame(frame: int, seed: int = BENCH_SEED, snr_db=None, channel: str = 'awgn', velocity_kmh=3.0):
    """Config 5 (spatial 4x4, rank 4, PMI 0, MMSE, 20 MHz 64-QAM, 14 symbols =
    83 916 bits) on flat CN(0,1) links (simulate_spatial_multiplexing's default
    channel) or PedA Rayleigh links at velocity_kmh: mimo_oracle.simulate_spatial
    on the frame's Philox draws."""
    from . import lte_oracle as O, mimo_oracle as M
    num = O.Numerology(bandwidth=20.0, modulation='64-QAM')
    L = 14 * (num.N + num.cp)
    nb = 14 * num.Nd * num.bps
    snr = bench_snr(frame) if snr_db is None else float(snr_db)
    r = M.simulate_spatial(num, payload_bits(seed, frame, nb), snr, 4, 4, 4, channel, 'Pedestrian_A',
                           velocity_kmh=velocity_kmh, draws=sm_draws(seed, frame, L, 4, 4, channel, 4))
    return int(r['bit_errors']), None


BENCH_FRAMES = {2: config2_frame, 3: config3_frame, 4: config4_frame, 5: config5_frame}
