"""ORACLE — TEST INFRASTRUCTURE ONLY (beamforming --
codebook precoding with CSI feedback, MRT / eigen precoders, adaptive update,
OFDMSimulator.simulate_beamforming).  Same rules as lte_oracle.py: a CPU
restatement with the reference's own operations in the reference's order;
only tests/ may import it.  Pinned by tests/golden/golden_bf.npz
(tests/golden/make_golden_bf.py runs the reference) in tests/test_oracle_bf.py.
"""
from __future__ import annotations

import numpy as np

from .lte_oracle import Numerology, bits_to_symbols, symbols_to_bits
from .tm4_oracle import codebook, select_best_pmi


def mrt_weights(H):
    """BeamformingPrecoder.calculate_mrt_weights (core/beamforming_precoder.py:
    35-60): conj(mean over RX of H) / its norm -> [num_tx, 1]."""
    h = np.mean(H, axis=0) if H.ndim == 2 else H
    hc = np.conj(h)
    return (hc / np.sqrt(np.sum(np.abs(hc) ** 2))).reshape(-1, 1)


def eigen_weights(H):
    """calculate_eigenbeamforming (:62-89): eigenvector of H^H H with the
    largest |eigenvalue| (np.linalg.eig), unit norm."""
    w, v = np.linalg.eig(H.conj().T @ H)
    W = v[:, np.argmax(np.abs(w))]
    return (W / np.sqrt(np.sum(np.abs(W) ** 2))).reshape(-1, 1)


def bf_gain_db(H, W):
    """calculate_beamforming_gain (:155-180): ||H W||^2 / (||H||_F^2 / num_tx)."""
    if W is None:
        return 0.0
    return 10 * np.log10(np.sum(np.abs(H @ W) ** 2) / (np.sum(np.abs(H) ** 2) / H.shape[1]))


def update_period(velocity_kmh, frequency_ghz=2.0):
    """AdaptiveBeamforming._calculate_update_period (:238-266): 10 % of the
    coherence time 9 / (16 pi fD) in 66.67 us symbols, clipped to [1, 140]."""
    fd = (velocity_kmh / 3.6) * (frequency_ghz * 1e9) / 3e8
    if fd == 0:
        return 100
    return np.clip(int(0.1 * (9 / (16 * np.pi * fd)) / (1 / 15000)), 1, 140)


_CQI_EDGES = [-np.inf, -6.0, -4.0, -2.0, 0.0, 2.0, 4.0, 6.0, 8.0, 10.0, 12.0, 14.0, 16.0, 18.0, 20.0, 22.0]


def csi_feedback(H, num_tx, codebook_type='TM6', noise_variance=1.0):
    """CSIFeedback.generate_feedback (core/csi_feedback.py:64-190): PMI by the
    rank-1 codebook's largest ||H W||^2, CQI from the post-precoding SINR on the
    TS 36.213-like table, RI from the eigenvalue ratio (> 0.2 -> 2)."""
    cb = codebook(num_tx, codebook_type, 1)
    pmi, _ = select_best_pmi(cb, H, 'capacity')
    W = cb[pmi]
    sinr_db = 10 * np.log10(np.sum(np.abs(H @ W) ** 2) / noise_variance)
    cqi = 15
    for q in range(16):
        hi = _CQI_EDGES[q + 1] if q < 15 else np.inf
        if _CQI_EDGES[q] <= sinr_db < hi:
            cqi = q
            break
    ev = np.sort(np.linalg.eigvalsh(H.conj().T @ H))[::-1]
    ri = (2 if ev[1] / ev[0] > 0.2 else 1) if len(ev) >= 2 else 1
    return {'pmi': pmi, 'cqi': cqi, 'ri': ri, 'sinr_db': sinr_db, 'precoder': W}


def simulate_beamforming(num: Numerology, bits, snr_db, num_tx=2, num_rx=1, codebook_type='TM6',
                         update_mode='adaptive'):
    """OFDMSimulator.simulate_beamforming (core/ofdm_core.py:2260-2477), in the
    reference's global-RNG order: H = (randn + j randn)/sqrt 2 [num_rx, num_tx];
    per OFDM symbol: PMI feedback; W = codebook precoder (static) or MRT of H
    (adaptive); x = W s; y = H x + noise (randn(rx, Nd) + j randn(rx, Nd)) *
    sqrt(s2/2), s2 = 10^(-SNR/10); MRC with H_eff = H W; nearest-point bits."""
    bits = np.asarray(bits)
    n0 = len(bits)
    Nd = len(num.data_idx)
    bpo = Nd * num.bps
    n_sym = int(np.ceil(n0 / bpo))
    bp = np.concatenate([bits, np.zeros(n_sym * bpo - n0, dtype=int)]) if n0 < n_sym * bpo else bits
    q = bits_to_symbols(bp, num.modulation)
    H = (np.random.randn(num_rx, num_tx) + 1j * np.random.randn(num_rx, num_tx)) / np.sqrt(2)
    s2 = 10 ** (-snr_db / 10)
    rx_all, gains, pmis = [], [], []
    W = None
    for i in range(n_sym):
        d = q[i * Nd:(i + 1) * Nd]
        fb = csi_feedback(H, num_tx, codebook_type, 1.0)
        pmis.append(fb['pmi'])
        W = fb['precoder']
        Wg = None
        if update_mode == 'adaptive':
            W = mrt_weights(H)
            Wg = W
        x = W @ d.reshape(1, -1)
        gains.append(bf_gain_db(H, Wg))
        y = np.zeros((num_rx, Nd), dtype=complex)
        for r in range(num_rx):
            for t in range(num_tx):
                y[r, :] += H[r, t] * x[t, :]
        z = (np.random.randn(num_rx, Nd) + 1j * np.random.randn(num_rx, Nd)) * np.sqrt(s2 / 2)
        rx_all.append(y + z)
    He = H @ W
    eq = []
    for i in range(n_sym):
        comb = np.zeros(Nd, dtype=complex)
        for r in range(num_rx):
            comb += np.conj(He[r, 0]) * rx_all[i][r, :]
        eq.append(comb / np.sum(np.abs(He) ** 2))
    brx = symbols_to_bits(np.concatenate(eq), num.modulation)[:n0]
    err = int(np.sum(bits[:n0] != brx))
    return {'bits_received_array': brx, 'bit_errors': err, 'ber': err / n0, 'channel_matrix': H,
            'pmi_history': pmis, 'unique_pmis': len(set(pmis)), 'beamforming_gain_db': float(np.mean(gains)),
            'symbols_rx': np.concatenate(eq)}
