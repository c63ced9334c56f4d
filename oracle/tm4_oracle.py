"""ORACLE — TEST INFRASTRUCTURE ONLY (TM4 spatial
multiplexing with codebook precoding, rank adaptation and the MMSE / ZF /
SIC / MRC detectors).  Same rules as lte_oracle.py: a CPU restatement with
the reference's own operations in the reference's order; only tests/ may
import it.  Pinned by tests/golden/golden_tm4.npz (tests/golden/
make_golden_tm4.py runs the reference) in tests/test_oracle_tm4.py.
"""
from __future__ import annotations

import numpy as np

from .lte_oracle import Numerology, bits_to_symbols, constellation, doppler_hz, nearest_indices, pilots
from .mimo_oracle import (_fft_symbols, _ofdm_time, hard_bits, layer_demap, layer_map, mimo_estimate,
                          mimo_pilot_indices, transmit_sm)


# --------------------------------------------------------------------------
# LTECodebook (core/codebook_lte.py:14-311)
def _dft_columns(n_ant, n_vec, div):
    """Rank-1 DFT vectors exp(j 2 pi i a / 16) / div, a = antenna (:75-91)."""
    out = []
    for i in range(n_vec):
        ph = 2 * np.pi * i * np.arange(n_ant) / 16
        out.append(np.exp(1j * ph).reshape(-1, 1) / div)
    return out


def codebook(num_tx: int, mode: str = 'TM6', rank: int = 1):
    """LTECodebook._generate_codebook: the matrices of (:58-311), in order."""
    if mode == 'TM6' and rank != 1:
        raise ValueError(f"TM6 solo soporta rank=1, recibido rank={rank}")
    if mode == 'TM4' and (rank < 1 or rank > min(num_tx, 4)):
        raise ValueError(f"TM4 con {num_tx} antenas soporta rank 1-{min(num_tx, 4)}, recibido rank={rank}")
    if mode not in ('TM6', 'TM4'):
        raise ValueError(f"Modo {mode} no soportado")
    r2 = np.sqrt(2)
    if rank == 1:                                  # TM6 == TM4 rank 1 (:114-119)
        if num_tx == 2:
            return [np.array([[1], [v]]) / r2 for v in (1, -1, 1j, -1j)]
        if num_tx == 4:
            return _dft_columns(4, 16, 2)
        if num_tx == 8:
            return _dft_columns(8, 16, np.sqrt(8))
        raise ValueError(f"num_tx={num_tx} no soportado en TM6")
    if rank == 2:                                  # (:121-209)
        if num_tx == 2:
            return [np.array([[1, 0], [0, 1]]), np.array([[1, 1], [1, -1]]) / r2,
                    np.array([[1, 1], [1j, -1j]]) / r2]
        if num_tx == 4:
            out = []
            e = [np.exp(1j * (2 * np.pi * i / 4)) for i in range(4)]
            out += [np.array([[1, 0], [x, 0], [0, 1], [0, x]]) / r2 for x in e]
            out += [np.array([[1, 1], [x, -x], [1, -1], [x, x]]) / 2 for x in e]
            out += [np.array([[1, 0], [0, 1], [x, 0], [0, x]]) / r2 for x in e]
            out += [np.array([[1, 1], [1, -1], [x, x], [x, -x]]) / 2 for x in e]
            return out
        if num_tx == 8:
            out = []
            for i in range(16):
                v = np.exp(1j * (2 * np.pi * i / 16) * np.arange(4)) / np.sqrt(4)
                W = np.zeros((8, 2), dtype=complex)
                W[:4, 0], W[4:, 1] = v, v
                out.append(W)
            return out
        raise ValueError(f"num_tx={num_tx} no soportado en TM4 Rank-2")
    if rank == 3:                                  # (:211-253)
        if num_tx < 4:
            raise ValueError(f"Rank-3 requiere al menos 4 antenas TX, disponibles: {num_tx}")
        if num_tx == 4:
            out = []
            for i in range(8):
                x = np.exp(1j * (2 * np.pi * i / 8))
                out.append(np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1], [x, x, x]]) / r2)
            return out
        out = []
        for i in range(16):
            th = 2 * np.pi * i / 16
            v = np.array([1, np.exp(1j * th), np.exp(1j * 2 * th)]) / np.sqrt(3)
            W = np.zeros((8, 3), dtype=complex)
            W[0:3, 0], W[3:6, 1], W[5:8, 2] = v, v, v
            out.append(W)
        return out
    if num_tx < 4:                                 # rank 4 (:255-311)
        raise ValueError(f"Rank-4 requiere al menos 4 antenas TX, disponibles: {num_tx}")
    if num_tx == 4:
        dft = np.zeros((4, 4), dtype=complex)
        for i in range(4):
            for j in range(4):
                dft[i, j] = np.exp(-2j * np.pi * i * j / 4)
        return [np.eye(4, dtype=complex), dft / 2,
                np.array([[1, 1, 1, 1], [1, -1, 1, -1], [1, 1, -1, -1], [1, -1, -1, 1]]) / 2,
                np.array([[1, 1, 1, 1], [1, 1j, -1, -1j], [1, -1, 1, -1], [1, -1j, -1, 1j]]) / 2]
    out = []
    for i in range(8):
        th = 2 * np.pi * i / 8
        W = np.zeros((8, 4), dtype=complex)
        for lyr in range(4):
            W[2 * lyr:2 * lyr + 2, lyr] = np.array([1, np.exp(1j * th * (lyr + 1))]) / r2
        out.append(W)
    return out


def select_best_pmi(cb, H, metric='capacity'):
    """LTECodebook.select_best_pmi (:332-373): first PMI with the largest
    ||H W||_F^2 (capacity / sinr) or ||H W||_F (frobenius)."""
    best, best_v = 0, -np.inf
    for i, W in enumerate(cb):
        He = H @ W
        v = np.linalg.norm(He, 'fro') if metric == 'frobenius' else np.sum(np.abs(He) ** 2)
        if v > best_v:
            best, best_v = i, v
    return best, best_v


# --------------------------------------------------------------------------
# RankAdaptation (core/rank_adaptation.py:19-272)
def optimal_rank(H, num_tx, num_rx, snr_db, method='eigenvalue', threshold=0.15):
    """calculate_optimal_rank (:52-146): eigenvalues of H^H H above
    threshold * lambda_max, capped by min(tx, rx, 4), then SNR caps (< 5 dB ->
    1, < 10 dB -> 2); or the rank maximising sum log2(1 + snr s_i^2 / r)."""
    Ha = H.mean(axis=2) if H.ndim == 3 else H
    max_rank = min(num_tx, num_rx, 4)
    if method == 'capacity':
        sv = np.linalg.svd(Ha, full_matrices=False)[1][:max_rank]
        snr = 10 ** (snr_db / 10)
        best, best_c = 1, -np.inf
        for r in range(1, max_rank + 1):
            c = 0
            for i in range(r):
                if i < len(sv):
                    c += np.log2(1 + snr * sv[i] ** 2 / r)
            if c > best_c:
                best, best_c = r, c
        return best
    if method != 'eigenvalue':
        raise ValueError(f"Método '{method}' no soportado")
    ev = np.sort(np.linalg.eigvalsh(Ha.conj().T @ Ha))[::-1]
    if ev[0] < 1e-10:
        return 1
    ri = min(np.sum(ev / ev[0] > threshold), max_rank)
    if snr_db < 5:
        ri = 1
    elif snr_db < 10:
        ri = min(ri, 2)
    return max(1, ri)


def precoder_for_rank(H, num_tx, num_rx, snr_db, rank, metric='capacity'):
    """select_precoder_for_rank (:148-210): TM4 codebook of that rank; capacity
    log2(det(I + snr/rank H_e H_e^H)) (first maximum wins)."""
    cb = codebook(num_tx, 'TM4', rank)
    Ha = H.mean(axis=2) if H.ndim == 3 else H
    snr = 10 ** (snr_db / 10)
    best, best_v = 0, -np.inf
    for i, W in enumerate(cb):
        He = Ha @ W
        if metric == 'capacity':
            try:
                v = np.log2(np.linalg.det(np.eye(num_rx) + (snr / rank) * (He @ He.conj().T)))
            except Exception:      # the reference's bare except (:184-189)
                v = 0
        elif metric in ('frobenius', 'sinr'):
            v = np.linalg.norm(He, 'fro') ** 2 if metric == 'frobenius' else np.sum(np.abs(He) ** 2)
        else:
            raise ValueError(f"Métrica '{metric}' no soportada")
        if v > best_v:
            best, best_v = i, v
    return best, cb[best]


def feedback(H, num_tx, num_rx, snr_db, rank_method='eigenvalue', pmi_metric='capacity'):
    """get_feedback (:212-265)."""
    ri = optimal_rank(H, num_tx, num_rx, snr_db, rank_method)
    pmi, W = precoder_for_rank(H, num_tx, num_rx, snr_db, ri, pmi_metric)
    Ha = H.mean(axis=2) if H.ndim == 3 else H
    ev = np.sort(np.linalg.eigvalsh(Ha.conj().T @ Ha))[::-1]
    sv = np.linalg.svd(Ha, compute_uv=False)
    return {'ri': ri, 'pmi': pmi, 'W': W, 'eigenvalues': ev, 'condition_number': sv[0] / (sv[-1] + 1e-10)}


# --------------------------------------------------------------------------
# MIMODetector (core/mimo_detector.py:18-369)
def _mmse(y, He, s2):
    """_mmse_detect (:135-173): inv(He^H He + s2 I) He^H y (pinv on LinAlgError)."""
    nl = He.shape[1]
    A = He.conj().T @ He + s2 * np.eye(nl)
    try:
        Ai = np.linalg.inv(A)
    except np.linalg.LinAlgError:
        Ai = np.linalg.pinv(A)
    return (Ai @ He.conj().T) @ y


def _sic(y, He, s2, const):
    """_sic_detect (:200-306): order by ||h_i||^2 / (sum_{j!=i} ||h_j||^2 + s2
    + 1e-10) descending (np.argsort()[::-1]); per layer MMSE over the
    remaining columns (1 column: vdot(h, y) / (||h||^2 + s2)), nearest
    constellation point (first index on ties), cancel with the original column."""
    nl = He.shape[1]
    if const is None:
        return _mmse(y, He, s2)
    nrm = [np.linalg.norm(He[:, i]) ** 2 for i in range(nl)]
    sinr = np.zeros(nl)
    for i in range(nl):
        itf = 0
        for j in range(nl):
            if j != i:
                itf += np.linalg.norm(He[:, j]) ** 2
        sinr[i] = nrm[i] / (itf + s2 + 1e-10)
    order = np.argsort(sinr)[::-1]
    yr = y.copy()
    Hr = He.copy()
    left = list(range(nl))
    out = np.zeros(nl, dtype=complex)
    for it in range(nl):
        lyr = order[it]
        rel = left.index(lyr)
        if Hr.shape[1] == 1:
            h = Hr[:, 0]
            sm = np.vdot(h, yr) / (np.linalg.norm(h) ** 2 + s2)
        else:
            A = Hr.conj().T @ Hr + s2 * np.eye(Hr.shape[1])
            sm = (np.linalg.inv(A) @ Hr.conj().T @ yr)[rel]
        sh = const[np.argmin(np.abs(const - sm))]
        out[lyr] = sh
        yr = yr - He[:, lyr] * sh
        if it < nl - 1:
            keep = np.ones(len(left), dtype=bool)
            keep[rel] = False
            Hr = Hr[:, keep]
            left.pop(rel)
    return out


def detect_one(det, y, H, s2, W, num_layers, const=None):
    """_detect_single (:99-133)."""
    He = H @ W if W is not None else H[:, :num_layers]
    det = det.upper()
    if det in ('MMSE', 'IRC'):
        return _mmse(y, He, s2)
    if det == 'ZF':
        return np.linalg.pinv(He) @ y
    if det == 'SIC':
        return _sic(y, He, s2, const)
    if det == 'MRC':
        if num_layers != 1:
            raise ValueError("MRC solo soporta num_layers=1 (rank-1)")
        h = He[:, 0]
        return np.array([np.dot(h.conj() / np.linalg.norm(h) ** 2, y)])
    raise ValueError(f"Detector '{det}' no soportado")


def detect(det, Y, H, s2, W, num_layers, const=None):
    """MIMODetector.detect per subcarrier (:55-97): Y [rx, n], H [rx, tx, n]."""
    if Y.shape[0] < num_layers:
        raise ValueError(f"num_rx ({Y.shape[0]}) debe ser >= num_layers ({num_layers})")
    out = np.zeros((num_layers, Y.shape[1]), dtype=complex)
    for k in range(Y.shape[1]):
        out[:, k] = detect_one(det, Y[:, k], H[:, :, k], s2, W, num_layers, const)
    return out


# --------------------------------------------------------------------------
# simulate_spatial_multiplexing (core/ofdm_core.py:2489-2815), general TM4
def choose_rank_pmi(num_tx, num_rx, rank, snr_db, csi):
    """:2573-2589: H_initial = (randn + j randn) / sqrt(2 num_tx) is ALWAYS
    drawn; adaptive + CSI -> RankAdaptation.get_feedback(H_initial); otherwise
    rank (or min(tx, rx) for 'adaptive' without CSI) with PMI 0."""
    Hi = (np.random.randn(num_rx, num_tx) + 1j * np.random.randn(num_rx, num_tx)) / np.sqrt(2 * num_tx)
    if rank == 'adaptive' and csi:
        fb = feedback(Hi, num_tx, num_rx, snr_db)
        return fb['ri'], fb['pmi'], fb['W']
    r = int(rank) if rank != 'adaptive' else min(num_tx, num_rx)
    return r, 0, codebook(num_tx, 'TM4', r)[0]


def simulate_tm4(num: Numerology, bits, snr_db, num_tx=4, num_rx=2, rank='adaptive', detector='MMSE',
                 channel='awgn', profile='Pedestrian_A', velocity_kmh=3, frequency_ghz=2.0, csi=True):
    """The reference driver with its global-RNG order: H_initial -> TX pilot
    reseeds -> transmit_spatial_multiplexing draws -> RX pilot reseeds.  Per
    OFDM symbol: QAM, zero-pad to a multiple of rank, round-robin layers,
    x_k = W layers[:, k] on the first ceil(Nd/rank) data SCs, CRS pilots per
    TX; per RX FFT; per symbol CRS estimate H[rx, tx, N], detector with the
    nominal s2 = 10^(-SNR/10), layer demap, hard bits."""
    bits = np.asarray(bits)
    n0 = len(bits)
    Nd = len(num.data_idx)
    bpo = Nd * num.bps
    n_sym = int(np.ceil(n0 / bpo))
    bp = np.pad(bits, (0, n_sym * bpo - n0)) if n0 < n_sym * bpo else bits.copy()
    r, pmi, W = choose_rank_pmi(num_tx, num_rx, rank, snr_db, csi)
    if num_rx < r:
        raise ValueError(f"num_rx ({num_rx}) debe ser >= num_layers ({r})")
    pidx = mimo_pilot_indices(num, num_tx)
    sig = [[] for _ in range(num_tx)]
    for i in range(n_sym):
        q = bits_to_symbols(bp[i * bpo:(i + 1) * bpo], num.modulation)
        lay = layer_map(q, r)
        grids = np.zeros((num_tx, num.N), dtype=complex)
        for di, sc in enumerate(num.data_idx):
            if di < lay.shape[1]:
                grids[:, sc] = W @ lay[:, di]
        for t in range(num_tx):
            grids[t][pidx[t]] = pilots(t % 4, len(pidx[t]))
        for t in range(num_tx):
            sig[t].append(_ofdm_time(num, grids[t]))
    xs = [np.concatenate(s) for s in sig]
    fD = doppler_hz(frequency_ghz, velocity_kmh)
    ys, Hm = transmit_sm(num, xs, num_rx, channel, snr_db, profile, fD)
    per_rx = [_fft_symbols(num, ys[k], n_sym) for k in range(num_rx)]
    s2 = 10 ** (-snr_db / 10)
    const = constellation(num.modulation)
    out_bits, syms = [], []
    for i in range(min(n_sym, len(per_rx[0]))):
        g = np.array([per_rx[k][i] for k in range(num_rx)])
        H = mimo_estimate(num, g, num_tx)
        lay = detect(detector, g[:, num.data_idx], H[:, :, num.data_idx], s2, W, r, const)
        sy = layer_demap(lay, original_length=Nd)
        syms.append(sy[:Nd])
        out_bits.append(hard_bits(sy[:Nd], num.modulation)[:bpo])
    rxb = np.concatenate(out_bits)[:n0]
    err = int(np.sum(bits[:n0] != rxb))
    return {'bits_received_array': rxb, 'bit_errors': err, 'ber': err / n0, 'channel_matrix': Hm,
            'precoder_matrix': W, 'rank': r, 'pmi_used': pmi, 'signals_rx': ys, 'symbols_rx': np.concatenate(syms)}


__all__ = ['codebook', 'select_best_pmi', 'optimal_rank', 'precoder_for_rank', 'feedback', 'detect', 'detect_one',
           'choose_rank_pmi', 'simulate_tm4', 'nearest_indices']
