"""Beamforming: drop-ins for the reference's
core/beamforming_precoder.py (BeamformingPrecoder, AdaptiveBeamforming) and
core/csi_feedback.py (CSIFeedback), plus the simulate_beamforming driver the
OFDMSimulator mirror exposes.

The precoder / feedback classes are control logic on one small matrix per call
(the reference's own NumPy operations, so the PMI / RI / CQI decisions are
identical).  The per-RE work of simulate_beamforming -- QAM map, precoding,
flat-channel transmission, noise, MRC and slicing -- runs on the GPU in
LTE_CHAIN_BEAMFORMING (lte_bf.hip), which also recomputes PMI, W, H_eff and
the gain per frame on the device for batched Philox grids.
"""
from __future__ import annotations

from typing import Dict

import numpy as np

from . import _capi as C
from .tm4 import LTECodebook


class BeamformingPrecoder:
    """core/beamforming_precoder.py:15-215."""

    def __init__(self, num_tx, num_layers=1, precoder_type='MRT'):
        self.num_tx, self.num_layers, self.precoder_type = num_tx, num_layers, precoder_type
        self.W = None

    def calculate_mrt_weights(self, H_channel):
        h = np.mean(H_channel, axis=0) if H_channel.ndim == 2 else H_channel
        hc = np.conj(h)
        return (hc / np.sqrt(np.sum(np.abs(hc) ** 2))).reshape(-1, 1)

    def calculate_eigenbeamforming(self, H_channel):
        w, v = np.linalg.eig(H_channel.conj().T @ H_channel)
        W = v[:, np.argmax(np.abs(w))]
        return (W / np.sqrt(np.sum(np.abs(W) ** 2))).reshape(-1, 1)

    def apply_precoding(self, symbols, W_matrix=None):
        if W_matrix is None:
            if self.W is None:
                raise ValueError("Precoder W no ha sido calculado. Llamar a update_precoder() primero.")
            W_matrix = self.W
        if symbols.ndim == 1:
            symbols = symbols.reshape(1, -1)
        return W_matrix @ symbols

    def update_precoder(self, H_channel, method='MRT'):
        H = np.mean(H_channel, axis=2) if H_channel.ndim == 3 else H_channel
        if method == 'MRT':
            self.W = self.calculate_mrt_weights(H)
        elif method == 'eigen':
            self.W = self.calculate_eigenbeamforming(H)
        else:
            raise ValueError(f"Método '{method}' no soportado")
        return self.W

    def get_current_precoder(self):
        return self.W

    def get_effective_channel(self, H_channel):
        if self.W is None:
            raise ValueError("Precoder W no disponible")
        return H_channel @ self.W

    def calculate_beamforming_gain(self, H_channel):
        if self.W is None:
            return 0.0
        p_bf = np.sum(np.abs(H_channel @ self.W) ** 2)
        return 10 * np.log10(p_bf / (np.sum(np.abs(H_channel) ** 2) / self.num_tx))


class AdaptiveBeamforming(BeamformingPrecoder):
    """core/beamforming_precoder.py:218-292: MRT refreshed every 10 % of the
    coherence time 9 / (16 pi fD), counted in 66.67 us symbols, in [1, 140]."""

    def __init__(self, num_tx, velocity_kmh, frequency_ghz, num_layers=1):
        super().__init__(num_tx, num_layers, precoder_type='MRT')
        self.velocity_kmh, self.frequency_ghz = velocity_kmh, frequency_ghz
        self.update_period = self._calculate_update_period()
        self.symbols_since_update = 0

    def _calculate_update_period(self):
        fd = (self.velocity_kmh / 3.6) * (self.frequency_ghz * 1e9) / 3e8
        if fd == 0:
            return 100
        return np.clip(int(0.1 * (9 / (16 * np.pi * fd)) / (1 / 15000)), 1, 140)

    def should_update(self):
        return self.symbols_since_update >= self.update_period

    def process_symbol(self, symbols, H_channel):
        if self.should_update() or self.W is None:
            self.update_precoder(H_channel, method='MRT')
            self.symbols_since_update = 0
        out = self.apply_precoding(symbols)
        self.symbols_since_update += 1
        return out


_CQI_EDGES = [-np.inf, -6.0, -4.0, -2.0, 0.0, 2.0, 4.0, 6.0, 8.0, 10.0, 12.0, 14.0, 16.0, 18.0, 20.0, 22.0, np.inf]


class CSIFeedback:
    """core/csi_feedback.py:24-228: PMI (rank-1 codebook, largest ||H w||^2),
    CQI (post-precoding SINR table), RI (eigenvalue ratio > 0.2 -> 2)."""

    def __init__(self, num_tx, num_rx, codebook_type='TM6', feedback_mode='perfect'):
        self.num_tx, self.num_rx = num_tx, num_rx
        self.codebook_type, self.feedback_mode = codebook_type, feedback_mode
        self.codebook = LTECodebook(num_tx, transmission_mode=codebook_type)
        self.total_feedbacks = 0
        self.pmi_history = []

    def calculate_pmi(self, H_channel):
        pmi, _ = self.codebook.select_best_pmi(H_channel, metric='capacity')
        self.pmi_history.append(pmi)
        self.total_feedbacks += 1
        return pmi

    def calculate_cqi(self, H_channel, pmi, noise_variance=1.0):
        He = H_channel @ self.codebook.get_precoder(pmi)
        sinr_db = 10 * np.log10(np.sum(np.abs(He) ** 2) / noise_variance)
        return self._sinr_to_cqi(sinr_db), sinr_db

    @staticmethod
    def _sinr_to_cqi(sinr_db):
        for q in range(16):
            if _CQI_EDGES[q] <= sinr_db < _CQI_EDGES[q + 1]:
                return q
        return 15

    def calculate_rank_indicator(self, H_channel):
        ev = np.sort(np.linalg.eigvalsh(H_channel.conj().T @ H_channel))[::-1]
        return (2 if ev[1] / ev[0] > 0.2 else 1) if len(ev) >= 2 else 1

    def generate_feedback(self, H_channel, noise_variance=1.0) -> Dict:
        pmi = self.calculate_pmi(H_channel)
        cqi, sinr_db = self.calculate_cqi(H_channel, pmi, noise_variance)
        return {'pmi': pmi, 'cqi': cqi, 'ri': self.calculate_rank_indicator(H_channel), 'sinr_db': sinr_db,
                'precoder': self.codebook.get_precoder(pmi)}

    def get_statistics(self):
        if not self.pmi_history:
            return None
        return {'total_feedbacks': self.total_feedbacks, 'unique_pmis': len(set(self.pmi_history)),
                'most_common_pmi': max(set(self.pmi_history), key=self.pmi_history.count),
                'pmi_distribution': np.bincount(self.pmi_history, minlength=self.codebook.codebook_size)}

    def print_statistics(self):
        """core/csi_feedback.py:208-228 (printout of get_statistics)."""
        stats = self.get_statistics()
        if stats is None:
            print("[CSIFeedback] No hay estadísticas disponibles")
            return
        print(f"\n{'=' * 60}")
        print("Estadísticas CSI Feedback")
        print(f"{'=' * 60}")
        print(f"  Total feedbacks: {stats['total_feedbacks']}")
        print(f"  PMIs únicos usados: {stats['unique_pmis']} / {self.codebook.codebook_size}")
        print(f"  PMI más común: {stats['most_common_pmi']}")
        print("\n  Distribución PMI:")
        for pmi, count in enumerate(stats['pmi_distribution']):
            if count > 0:
                print(f"    PMI {pmi}: {count} ({100 * count / stats['total_feedbacks']:.1f}%)")
        print(f"{'=' * 60}\n")


def bf_plan(config, n_sym, n_bits, num_tx, num_rx, adaptive, max_frames=1, precision=None):
    from .engine import get_plan
    return get_plan(N=config.N, Nc=config.Nc, cp_len=config.cp_length, bps=config.bits_per_symbol, n_sym=n_sym,
                    chain=C.CHAIN_BEAMFORMING, channel=C.CH_AWGN, num_rx=num_rx, num_tx=num_tx, n_bits=n_bits,
                    max_frames=max_frames, bf_adaptive=int(adaptive), precision=precision)


def simulate_beamforming(sim, bits, snr_db=10.0, num_tx=2, num_rx=1, codebook_type='TM6', velocity_kmh=3.0,
                         update_mode='adaptive') -> Dict:
    """OFDMSimulator.simulate_beamforming (core/ofdm_core.py:2260-2477) -- one
    GPU call.  Global-RNG order as the reference: H = (randn(rx, tx) + j
    randn(rx, tx)) / sqrt 2, then per OFDM symbol randn(rx, Nd) (real) and
    randn(rx, Nd) (imag) of the noise.  The frame's H and the noise are
    injected; PMI (CSI feedback), the precoder (codebook vector for 'static',
    MRT for 'adaptive'), H_eff and the gain are computed on the device."""
    bits = np.asarray(bits)
    if bits.size == 0:
        raise ValueError("Bits array cannot be empty")
    if codebook_type not in ('TM6', 'TM4'):
        raise ValueError(f"Modo {codebook_type} no soportado")
    cfg = sim.config
    n0 = len(bits)
    Nd = sim.Nd
    n_sym = int(np.ceil(n0 / (Nd * cfg.bits_per_symbol)))
    adaptive = update_mode == 'adaptive'
    plan = bf_plan(cfg, n_sym, n0, num_tx, num_rx, adaptive, precision=sim.precision)
    H = (np.random.randn(num_rx, num_tx) + 1j * np.random.randn(num_rx, num_tx)) / np.sqrt(2)
    L = n_sym * Nd
    z = np.zeros((num_rx, 2, L))
    for i in range(n_sym):
        z[:, 0, i * Nd:(i + 1) * Nd] = np.random.randn(num_rx, Nd)
        z[:, 1, i * Nd:(i + 1) * Nd] = np.random.randn(num_rx, Nd)
    lh = np.stack([H.real, H.imag], axis=-1)
    r = plan.run([snr_db], bits=(bits & 1).astype(np.uint8)[None], noise=z[None], link_h=lh[None],
                 capture=('bits_rx', 'data_syms', 'pmi', 'bf_gain'))
    brx = r['bits_rx'][0].astype(np.int64)
    err = int(np.sum(bits != brx))
    pmi = int(r['pmi'][0])
    res = {'transmitted_bits': int(n0), 'received_bits': int(n0), 'bits_received_array': brx,
           'bit_errors': err, 'errors': err, 'ber': float(err / n0), 'snr_db': float(snr_db),
           'num_tx': num_tx, 'num_rx': num_rx, 'mode': 'Beamforming', 'codebook_type': codebook_type,
           'beamforming_gain_db': float(r['bf_gain'][0]), 'channel_matrix': H, 'pmi_history': [pmi] * n_sym,
           'unique_pmis': 1, 'velocity_kmh': velocity_kmh,
           'symbols_rx': r['data_syms'][0].astype(np.complex128)}
    sim.last_results = res
    return res


__all__ = ['BeamformingPrecoder', 'AdaptiveBeamforming', 'CSIFeedback', 'simulate_beamforming', 'bf_plan']
