"""ORACLE — TEST INFRASTRUCTURE ONLY (multi-antenna rows of SURVEY §8:
a12, a13, a33-a37; configs 4 and 5).  Same rules as lte_oracle.py: CPU
restatement with the reference's own operations in the reference's order;
only tests/ may import it.  Pinned by tests/golden/golden_mimo.npz
(tests/golden/make_golden_mimo.py runs the reference) in
tests/test_oracle_mimo.py.

Config 4 (SFBC) follows the reference with the documented estimator fix of
Appendix A Q19 (H0 = H[0,0,:], H1 = H[0,1,:] of estimate_channel_from_grid);
the unfixed reference raises (core/mimo_channel_estimator_periodic.py:219).
"""
from __future__ import annotations

import numpy as np

from .lte_oracle import (BPS, ITU_CHANNEL_MODELS, Numerology, attach_crc24a, bits_to_symbols, coded_rx_decode,
                         constellation, doppler_hz, interp_channel, itu_paths, jakes, llrs, multipath,
                         nearest_indices, indices_to_bits, pilots, rate_match, segment, tf_interleave_perm,
                         turbo_encode)


# --------------------------------------------------------------------------
# a33 SFBC Alamouti (core/sfbc_alamouti.py)
def sfbc_encode(s: np.ndarray):
    """SFBCAlamouti.encode (:45-78): pairs (s0,s1) -> TX0 [s0, -conj(s1)],
    TX1 [s1, conj(s0)]."""
    s = np.asarray(s, dtype=complex)
    if len(s) % 2:
        raise ValueError(f"Number of symbols must be even for Alamouti coding, got {len(s)}")
    t0 = np.zeros(len(s), dtype=complex)
    t1 = np.zeros(len(s), dtype=complex)
    t0[0::2] = s[0::2]
    t1[0::2] = s[1::2]
    t0[1::2] = -np.conj(s[1::2])
    t1[1::2] = np.conj(s[0::2])
    return t0, t1


def sfbc_decode(rx, H0, H1, reg=1e-10):
    """SFBCAlamouti.decode (:80-163): the per-pair loop with NumPy complex128
    scalars, exactly as the reference evaluates it (NumPy's scalar |z| and
    complex/real division round differently from the vectorised forms):
      s0 = conj(h0k) rk + h1k1 conj(rk1);  s1 = conj(h1k) rk - h0k1 conj(rk1)
      norm = |(h0k+h0k1)/2|^2 + |(h1k+h1k1)/2|^2 + reg."""
    rx, H0, H1 = (np.asarray(v, dtype=complex) for v in (rx, H0, H1))
    if len(rx) % 2:
        raise ValueError(f"Number of RX symbols must be even, got {len(rx)}")
    out = np.zeros(len(rx), dtype=complex)
    for i in range(0, len(rx), 2):
        rk, rk1 = rx[i], rx[i + 1]
        h0k, h1k, h0k1, h1k1 = H0[i], H1[i], H0[i + 1], H1[i + 1]
        s0 = np.conj(h0k) * rk + h1k1 * np.conj(rk1)
        s1 = np.conj(h1k) * rk - h0k1 * np.conj(rk1)
        norm = np.abs((h0k + h0k1) / 2) ** 2 + np.abs((h1k + h1k1) / 2) ** 2 + reg
        out[i] = s0 / norm
        out[i + 1] = s1 / norm
    return out


def sfbc_data_idx(num: Numerology) -> np.ndarray:
    """SFBCResourceMapper.__init__ (:186-200): an odd data-SC count drops the last."""
    d = num.data_idx
    return d[:len(d) - (len(d) % 2)]


def sfbc_map_grid(num: Numerology, t0, t1):
    """SFBCResourceMapper.map_sfbc_to_grid (:213-256): data on the (even) data
    SCs; TX0 pilots at pilot_idx[0::2] from cell 0, TX1 at [1::2] from cell 1
    (each generate_pilots reseeds the global RNG, Q1)."""
    d = sfbc_data_idx(num)
    g0 = np.zeros(num.N, dtype=complex)
    g1 = np.zeros(num.N, dtype=complex)
    g0[d] = t0[:len(d)]
    g1[d] = t1[:len(d)]
    p0, p1 = num.pilot_idx[::2], num.pilot_idx[1::2]
    g0[p0] = pilots(0, len(p0))
    g1[p1] = pilots(1, len(p1))
    return g0, g1


# --------------------------------------------------------------------------
# a34 MIMOChannelEstimatorPeriodic (core/mimo_channel_estimator_periodic.py)
def mimo_pilot_indices(num: Numerology, num_tx: int):
    """get_orthogonal_pilot_indices (:75-107): pilots_all[tx % step :: step],
    step = min(num_tx, 4)."""
    step = num_tx if num_tx <= 4 else 4
    return [num.pilot_idx[(t % step)::step] for t in range(num_tx)]


def mimo_estimate(num: Numerology, grids: np.ndarray, num_tx: int) -> np.ndarray:
    """estimate_channel_from_grid (:108-185), return_full_freq: LS at the TX's
    pilots (cell tx % 4, reseeding per link) + _interpolate_channel -> H[rx, tx, N]."""
    grids = np.atleast_2d(grids)
    pidx = mimo_pilot_indices(num, num_tx)
    H = np.zeros((grids.shape[0], num_tx, num.N), dtype=complex)
    for r in range(grids.shape[0]):
        for t in range(num_tx):
            pil = pilots(t % 4, len(pidx[t]))
            hp = grids[r, pidx[t]] / pil
            H[r, t] = interp_channel(pidx[t], hp, num.N)
    return H


# --------------------------------------------------------------------------
# a12 OFDMChannel.transmit_mimo (core/ofdm_core.py:434-543)
def transmit_mimo_draws(num_tx: int, num_rx: int, channel: str, L: int, profile='Pedestrian_A'):
    """Random numbers transmit_mimo consumes, in order: per RX, per TX link
    [rayleigh: per path rand(16); link noise normal(L) x 2 at 100 dB], then the
    RX noise normal(L) x 2 (unit scale; scaled at use)."""
    n_paths = len(ITU_CHANNEL_MODELS[profile]['delays_us'])
    out = []
    for _ in range(num_rx):
        links = []
        for _ in range(num_tx):
            if channel == 'rayleigh_mp':
                ph = [2 * np.pi * np.random.rand(16) for _ in range(n_paths)]
                links.append({'phases': ph, 'z_re': np.random.normal(0, 1.0, L),
                              'z_im': np.random.normal(0, 1.0, L)})
            else:
                links.append(None)
        out.append({'links': links, 'z_re': np.random.normal(0, 1.0, L), 'z_im': np.random.normal(0, 1.0, L)})
    return out


def transmit_mimo(num: Numerology, xs, num_rx: int, channel: str, snr_db: float, profile='Pedestrian_A',
                  draws=None):
    """OFDMChannel.transmit_mimo: awgn links h = exp(j tx pi/2) (h = 1 for tx 0);
    rayleigh links = a ChannelSimulator at 100 dB (fading + still-drawn link
    noise) with h estimated by power ratio and correlation phase; noise per RX
    with power (P_rx / num_tx) / SNR (Q5)."""
    num_tx = len(xs)
    L = len(xs[0])
    if draws is None:
        draws = transmit_mimo_draws(num_tx, num_rx, channel, L, profile)
    ys = []
    Hm = np.zeros((num_rx, num_tx), dtype=complex)
    for r in range(num_rx):
        acc = np.zeros(L, dtype=complex)
        # the device's Philox mode (draws[r]['combined_link_noise']): the links'
        # 100 dB noises enter the RX sum as one draw of standard deviation
        # sqrt(sum_t s_rt^2) on link (r, 0)'s numbers (lte_mimo.hip
        # rx_link_sigma); each link's own draw still forms its Hm entry
        comb = channel != 'awgn' and bool(draws[r].get('combined_link_noise'))
        # the device's merged mode (draws[r]['merged_link_noise'], config 4's full
        # chain: lte_internal.h launch_npow_sfbc_merged): no link-noise draw; its
        # power 2 s2 enters P in expectation and its variance the RX noise draw
        merged = comb and bool(draws[r].get('merged_link_noise'))
        s2, pl = 0.0, 0.0
        for t in range(num_tx):
            x = xs[t]
            if channel == 'awgn':
                h = 1.0 + 0j if t == 0 else np.exp(1j * (t * np.pi / 2))
                y = x * h
            else:
                dl, g = itu_paths(num, profile)
                d = draws[r]['links'][t]
                y0 = multipath(x, dl, g, d['phases'], 0.0, num.fs)
                p = np.mean(np.abs(y0) ** 2)
                pl = pl + p
                s = np.sqrt((p / 10 ** (100.0 / 10)) / 2)
                s2 = s2 + s * s
                y = y0 + (s * d['z_re'] + 1j * (s * d['z_im']))
                tp = np.mean(np.abs(x) ** 2)
                rp = np.mean(np.abs(y) ** 2)
                if tp > 1e-12:
                    h = np.sqrt(rp / tp) * np.exp(1j * np.angle(np.mean(y * np.conj(x))))
                else:
                    h = 1.0 + 0j
                if comb:
                    y = y0
            Hm[r, t] = h
            acc += y
        if merged:
            # the links' powers summed, then one sigma^2 (k_npow_sfbc_merged's order)
            s2 = (pl / 10 ** (100.0 / 10)) / 2
            sp = np.mean(np.abs(acc) ** 2) + 2.0 * s2
            npow = 2.0 * s2 + (sp / num_tx) / 10 ** (snr_db / 10)
            s = np.sqrt(npow / 2)
            ys.append(acc + (s * draws[r]['z_re'] + 1j * (s * draws[r]['z_im'])))
            continue
        if comb:
            s = np.sqrt(s2)
            z0 = draws[r]['links'][0]
            acc = acc + (s * z0['z_re'] + 1j * (s * z0['z_im']))
        sp = np.mean(np.abs(acc) ** 2)
        npow = (sp / num_tx) / 10 ** (snr_db / 10)
        s = np.sqrt(npow / 2)
        ys.append(acc + (s * draws[r]['z_re'] + 1j * (s * draws[r]['z_im'])))
    return ys, Hm


# --------------------------------------------------------------------------
# a13 ChannelSimulator.transmit_spatial_multiplexing (core/channel.py:397-493)
def transmit_sm_draws(num_tx: int, num_rx: int, channel: str, L: int, profile='Pedestrian_A'):
    """Draw order: rayleigh_mp: per (rx, tx) link: filter per path rand(16),
    then impulse_response per path rand(16); then per RX normal(L) x 2.
    awgn: per (rx, tx) normal() re, normal() im (CN(0,1)); then noise."""
    n_paths = len(ITU_CHANNEL_MODELS[profile]['delays_us'])
    links = []
    for _ in range(num_rx):
        row = []
        for _ in range(num_tx):
            if channel == 'rayleigh_mp':
                f = [2 * np.pi * np.random.rand(16) for _ in range(n_paths)]
                ir = [2 * np.pi * np.random.rand(16) for _ in range(n_paths)]
                row.append({'phases': f, 'ir_phases': ir})
            else:
                hr = np.random.normal(0, 1 / np.sqrt(2))
                hi = np.random.normal(0, 1 / np.sqrt(2))
                row.append({'h': hr + 1j * hi})
        links.append(row)
    noise = [{'z_re': np.random.normal(0, 1.0, L), 'z_im': np.random.normal(0, 1.0, L)} for _ in range(num_rx)]
    return {'links': links, 'noise': noise}


def transmit_sm(num: Numerology, xs, num_rx: int, channel: str, snr_db: float, profile='Pedestrian_A',
                fD=None, draws=None):
    """Rayleigh: per link RayleighChannel with the gains converted a third time
    (Q2) and fD from 3 km/h @ 2 GHz by default (Q3); channel_matrix = first
    impulse-response tap.  Noise per RX: P / SNR (no /num_tx here)."""
    num_tx = len(xs)
    L = min(len(x) for x in xs)
    xs = [np.asarray(x)[:L] for x in xs]
    if fD is None:
        fD = doppler_hz(2.0, 3)
    if draws is None:
        draws = transmit_sm_draws(num_tx, num_rx, channel, L, profile)
    ys = [np.zeros(L, dtype=complex) for _ in range(num_rx)]
    Hm = np.zeros((num_rx, num_tx), dtype=complex)
    snr_lin = 10 ** (snr_db / 10)
    if channel == 'rayleigh_mp':
        dl, g3 = itu_paths(num, profile, spatial=True)
        for r in range(num_rx):
            for t in range(num_tx):
                d = draws['links'][r][t]
                ys[r] += multipath(xs[t], dl, g3, d['phases'], fD, num.fs)
                Hm[r, t] = g3[0] * jakes(d['ir_phases'][0], fD, num.fs, 1)[0]
    else:
        for r in range(num_rx):
            for t in range(num_tx):
                hh = draws['links'][r][t]['h']
                Hm[r, t] = hh
                ys[r] += hh * xs[t]
    for r in range(num_rx):
        p = np.mean(np.abs(ys[r]) ** 2)
        s = np.sqrt((p / snr_lin) / 2)
        ys[r] += s * draws['noise'][r]['z_re'] + 1j * (s * draws['noise'][r]['z_im'])
    return ys, Hm


# --------------------------------------------------------------------------
# a35 / a36 layer mapping + MMSE (core/layer_mapper.py, core/mimo_detector.py)
def layer_map(symbols, rank):
    """LayerMapper.map_to_layers (:35-79): zero-pad to a multiple of rank,
    round-robin -> [rank, n/rank]."""
    s = np.asarray(symbols)
    if rank == 1:
        return s.reshape(1, -1)
    if len(s) % rank:
        s = np.concatenate([s, np.zeros(rank - len(s) % rank, dtype=s.dtype)])
    return s.reshape(len(s) // rank, rank).T


def layer_demap(layers, original_length=None):
    """LayerMapper.demap_from_layers (:81-115)."""
    layers = np.asarray(layers)
    s = layers.flatten() if layers.shape[0] == 1 else layers.T.flatten()
    return s if original_length is None else s[:original_length]


def mmse_detect(Y, H, sigma2, W):
    """MIMODetector._detect_per_subcarrier + _mmse_detect (:83-173), one
    subcarrier at a time with the same 2-D NumPy/LAPACK calls:
    s = inv(Heff^H Heff + s2 I) Heff^H y, Heff = H W."""
    nl = W.shape[1]
    out = np.zeros((nl, Y.shape[1]), dtype=complex)
    for sc in range(Y.shape[1]):
        He = H[:, :, sc] @ W
        HH = He.conj().T @ He
        try:
            Hi = np.linalg.inv(HH + sigma2 * np.eye(nl))
        except np.linalg.LinAlgError:
            Hi = np.linalg.pinv(HH + sigma2 * np.eye(nl))
        out[:, sc] = (Hi @ He.conj().T) @ Y[:, sc]
    return out


def hard_bits(symbols, mod):
    """Euclidean argmin (first index on ties) -> MSB-first bits."""
    return indices_to_bits(nearest_indices(np.asarray(symbols), mod), BPS[mod])


def _ofdm_time(num: Numerology, grid):
    t = np.fft.ifft(grid) * np.sqrt(num.N)
    return np.concatenate([t[-num.cp:], t])


def _fft_symbols(num: Numerology, y, n_sym):
    sl = num.N + num.cp
    return [np.fft.fft(y[i * sl + num.cp:(i + 1) * sl]) / np.sqrt(num.N) for i in range(n_sym)
            if (i + 1) * sl <= len(y)]


def _papr_db(s):
    p = np.abs(s) ** 2
    return 10 * np.log10(np.max(p) / np.mean(p))


# --------------------------------------------------------------------------
# G17 configs 4 / 5 end to end
def simulate_sfbc(num: Numerology, bits, snr_db, num_rx=2, channel='awgn', profile='Pedestrian_A', draws=None):
    """OFDMSimulator.simulate_miso (num_rx == 1, core/ofdm_core.py:1850-2047) /
    simulate_mimo (:2049-2258) with the Q19 estimator fix: per OFDM symbol QAM
    + SFBC encode + SFBC grid (pilot reseeds 0, 1) + IFFT/CP; transmit_mimo;
    per RX FFT + slot-0 estimate of H0/H1 reused for 14 symbols; per-RX SFBC
    decode averaged over RX; nearest-point hard decision."""
    bits = np.asarray(bits)
    n0 = len(bits)
    d_idx = sfbc_data_idx(num)
    bpo = len(d_idx) * num.bps
    n_sym = int(np.ceil(n0 / bpo))
    bp = np.pad(bits, (0, n_sym * bpo - n0)) if n0 < n_sym * bpo else bits.copy()
    s0, s1, chunks, pap0, pap1 = [], [], [], [], []
    for i in range(n_sym):
        ch = bp[i * bpo:(i + 1) * bpo]
        chunks.append(ch)
        t0, t1 = sfbc_encode(bits_to_symbols(ch, num.modulation))
        g0, g1 = sfbc_map_grid(num, t0, t1)
        x0, x1 = _ofdm_time(num, g0), _ofdm_time(num, g1)
        s0.append(x0)
        s1.append(x1)
        pap0.append(_papr_db(x0))
        pap1.append(_papr_db(x1))
    ys, Hm = transmit_mimo(num, [np.concatenate(s0), np.concatenate(s1)], num_rx, channel, snr_db, profile, draws)
    grids, H0s, H1s = [], [], []
    for r in range(num_rx):
        gr = _fft_symbols(num, ys[r], len(ys[r]) // (num.N + num.cp))
        h0l, h1l = [], []
        for st in range(0, len(gr), 14):
            H = mimo_estimate(num, gr[st], 2)
            for _ in range(min(14, len(gr) - st)):
                h0l.append(H[0, 0])
                h1l.append(H[0, 1])
        grids.append(gr)
        H0s.append(h0l)
        H1s.append(h1l)
    out_bits = []
    for i in range(min(n_sym, len(grids[0]))):
        dec = [sfbc_decode(grids[r][i][d_idx], H0s[r][i][d_idx], H1s[r][i][d_idx]) for r in range(num_rx)]
        z = np.mean(dec, axis=0)
        c = constellation(num.modulation)
        det = c[nearest_indices(z, num.modulation)]
        out_bits.append(hard_bits(det, num.modulation))
    rxb = np.concatenate(out_bits)[:n0]
    err = int(np.sum(bits[:n0] != rxb))
    p0, p1 = float(np.mean(pap0)), float(np.mean(pap1))
    return {'bits_received_array': rxb, 'bit_errors': err, 'ber': err / n0, 'channel_matrix': Hm,
            'papr_db_tx0': p0, 'papr_db_tx1': p1, 'papr_db': float(np.mean([p0, p1])), 'signals_rx': ys}


def simulate_spatial(num: Numerology, bits, snr_db, num_tx=4, num_rx=4, rank=4, channel='awgn',
                     profile='Pedestrian_A', velocity_kmh=3, frequency_ghz=2.0, draws=None):
    """simulate_spatial_multiplexing (core/ofdm_core.py:2489-2815), fixed rank,
    TM4 PMI 0 (rank 4 -> W = I4): H_initial draw (always), per symbol QAM ->
    layers -> precode on the first ceil(Nd/rank) data SCs (Q20) -> CRS pilots
    per TX (cell tx % 4, reseeding) -> IFFT/CP; transmit_spatial_multiplexing;
    per symbol: FFT, CRS estimate H[rx,tx,N] (every symbol), MMSE with the
    nominal sigma2 = 10^(-SNR/10), layer demap, hard bits."""
    bits = np.asarray(bits)
    n0 = len(bits)
    Nd = len(num.data_idx)
    bpo = Nd * num.bps
    n_sym = int(np.ceil(n0 / bpo))
    bp = np.pad(bits, (0, n_sym * bpo - n0)) if n0 < n_sym * bpo else bits.copy()
    if draws is None:
        np.random.randn(num_rx, num_tx)            # H_initial (core/ofdm_core.py:2581)
        np.random.randn(num_rx, num_tx)
    if rank != 4 or num_tx != 4:
        raise NotImplementedError('oracle restates TM4 rank 4 (W = I4) only')
    W = np.eye(4, dtype=complex)
    pidx = mimo_pilot_indices(num, num_tx)
    sig = [[] for _ in range(num_tx)]
    chunks = []
    for i in range(n_sym):
        ch = bp[i * bpo:(i + 1) * bpo]
        chunks.append(ch)
        q = bits_to_symbols(ch, num.modulation)
        lay = layer_map(q, rank)
        grids = [np.zeros(num.N, dtype=complex) for _ in range(num_tx)]
        for di, sc in enumerate(num.data_idx):
            if di < lay.shape[1]:
                xk = W @ lay[:, di]
                for t in range(num_tx):
                    grids[t][sc] = xk[t]
        for t in range(num_tx):
            grids[t][pidx[t]] = pilots(t % 4, len(pidx[t]))
        for t in range(num_tx):
            sig[t].append(_ofdm_time(num, grids[t]))
    xs = [np.concatenate(s) for s in sig]
    fD = doppler_hz(frequency_ghz, velocity_kmh)
    ys, Hm = transmit_sm(num, xs, num_rx, channel, snr_db, profile, fD, None if draws is None else draws)
    per_rx = [_fft_symbols(num, ys[r], n_sym) for r in range(num_rx)]
    s2 = 10 ** (-snr_db / 10)
    out_bits = []
    for i in range(min(n_sym, len(per_rx[0]))):
        g = np.array([per_rx[r][i] for r in range(num_rx)])
        H = mimo_estimate(num, g, num_tx)
        lay = mmse_detect(g[:, num.data_idx], H[:, :, num.data_idx], s2, W)
        sy = layer_demap(lay, original_length=Nd)
        out_bits.append(hard_bits(sy[:Nd], num.modulation)[:bpo])
    rxb = np.concatenate(out_bits)[:n0]
    err = int(np.sum(bits[:n0] != rxb))
    return {'bits_received_array': rxb, 'bit_errors': err, 'ber': err / n0, 'channel_matrix': Hm,
            'precoder_matrix': W, 'signals_rx': ys}


# --------------------------------------------------------------------------
# Config 4: SFBC 2 x num_rx + the coding chain (the build's composition; the
# reference has no function that composes them, SURVEY §8c / DESIGN.md §3a)
def simulate_sfbc_coded(num: Numerology, bits, snr_db, num_rx=2, channel='rayleigh_mp', profile='Pedestrian_A',
                        draws=None, iters=8):
    """simulate_siso_coded's coding chain (core/ofdm_core.py:925-1338: CRC-24A,
    segmentation, turbo, rate matching, QAM, T/F interleaver) with cols = the
    SFBC REs per OFDM symbol (Nd & ~1, Q18) around simulate_mimo's SFBC link
    (core/ofdm_core.py:2049-2258 with the Q19 estimator fix): per OFDM symbol
    SFBC encode + grid (cells 0 / 1) + IFFT/CP; transmit_mimo; per RX FFT +
    slot-0 estimate; per-RX SFBCAlamouti.decode averaged over RX.  Soft
    output: max-log LLRs (core/ofdm_core.py:791-923) with sigma^2_eff =
    max((sigma^2 / R^2) sum_r 1 / clip(norm_r, 1e-6, 1e6), sigma^2 / 4) per SC
    pair, sigma^2 = 1 / 10^(SNR/10) -- the SISO rule (:1224-1243) applied to the
    combined estimate; T/F de-interleave; dematch; the float64 reference turbo
    decoder (8 iterations); CRC-24A."""
    bits = np.asarray(bits)
    n0 = len(bits)
    tbc = attach_crc24a(bits)
    cbs, plan = segment(tbc)
    rms = []
    for cb in cbs:
        enc = turbo_encode(cb)
        rms.append(rate_match(enc, len(enc), len(cb), 0))
    coded = np.concatenate(rms)
    qam = bits_to_symbols(coded, num.modulation)
    d_idx = sfbc_data_idx(num)
    res = len(d_idx)
    perm, rows, total = tf_interleave_perm(len(qam), res)
    padded = np.pad(qam, (0, total - len(qam))) if len(qam) < total else qam[:total]
    inter = padded[perm]
    n_sym = rows
    s0, s1 = [], []
    for i in range(n_sym):
        t0, t1 = sfbc_encode(inter[i * res:(i + 1) * res])
        g0, g1 = sfbc_map_grid(num, t0, t1)
        s0.append(_ofdm_time(num, g0))
        s1.append(_ofdm_time(num, g1))
    ys, Hm = transmit_mimo(num, [np.concatenate(s0), np.concatenate(s1)], num_rx, channel, snr_db, profile, draws)
    grids, H0s, H1s = [], [], []
    for r in range(num_rx):
        gr = _fft_symbols(num, ys[r], n_sym)
        h0l, h1l = [], []
        for st in range(0, len(gr), 14):
            H = mimo_estimate(num, gr[st], 2)
            for _ in range(min(14, len(gr) - st)):
                h0l.append(H[0, 0])
                h1l.append(H[0, 1])
        grids.append(gr)
        H0s.append(h0l)
        H1s.append(h1l)
    s2 = 1.0 / (10 ** (snr_db / 10))
    z_all, nv_all = [], []
    for i in range(n_sym):
        dec, inv_g = [], np.zeros(res // 2)
        for r in range(num_rx):
            h0, h1 = H0s[r][i][d_idx], H1s[r][i][d_idx]
            dec.append(sfbc_decode(grids[r][i][d_idx], h0, h1))
            a0, a1 = (h0[0::2] + h0[1::2]) / 2, (h1[0::2] + h1[1::2]) / 2
            nrm = np.abs(a0) ** 2 + np.abs(a1) ** 2 + 1e-10
            inv_g += 1.0 / np.clip(nrm, 1e-6, 1e6)
        z_all.append(np.mean(dec, axis=0))
        nv_all.append(np.repeat(np.maximum((s2 / num_rx ** 2) * inv_g, s2 / 4.0), 2))
    z = np.concatenate(z_all)
    nv = np.concatenate(nv_all)
    ncs = len(coded) // num.bps
    rows_rx = int(np.ceil(ncs / res))
    tot = rows_rx * res
    sd = z[:tot].reshape(res, rows_rx).T.reshape(-1)[:ncs]
    nd = nv[:tot].reshape(res, rows_rx).T.reshape(-1)[:ncs]
    L = llrs(sd, nd, num.modulation)
    L = np.pad(L, (0, len(coded) - len(L))) if len(L) < len(coded) else L[:len(coded)]
    dec, ok = coded_rx_decode(L, plan, [len(r) for r in rms], iters)
    dec = np.pad(dec, (0, n0 - len(dec))) if len(dec) < n0 else dec[:n0]
    err = int(np.sum(bits != dec))
    return {'bits_received_array': dec, 'bit_errors': err, 'ber': err / n0, 'crc_pass': bool(ok),
            'channel_matrix': Hm, 'symbols_rx': sd, 'noise_var': nd, 'llrs': L}
