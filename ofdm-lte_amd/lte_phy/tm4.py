"""TM4 closed-loop spatial multiplexing: the reference's codebook, rank
adaptation, layer mapper and MIMO detector classes.

Drop-ins for core.codebook_lte.LTECodebook (core/codebook_lte.py:14-433),
core.rank_adaptation.RankAdaptation (core/rank_adaptation.py:19-272),
core.layer_mapper.LayerMapper (core/layer_mapper.py:14-150) and
core.mimo_detector.MIMODetector (core/mimo_detector.py:18-369): same names,
arguments, return values and exceptions.  The codebook tables and the RI/PMI
search are host-side control logic on one small matrix per call (the
reference's own NumPy/LAPACK calls, so the decisions are identical);
MIMODetector.detect runs the per-subcarrier detectors on the GPU through
lte_mimo_detect_host (float64 on the device, lte_mimo.hip k_det_stage), the
same device code the spatial chain (LTE_CHAIN_SPATIAL) runs in-line.
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np

from . import _capi as C

DETECTORS = {'MMSE': C.DET_MMSE, 'IRC': C.DET_MMSE, 'ZF': C.DET_ZF, 'SIC': C.DET_SIC, 'MRC': C.DET_MRC}


class LTECodebook:
    """LTECodebook (core/codebook_lte.py:14-433): TM6 rank-1 and TM4 rank 1-4
    precoders for 2 / 4 / 8 TX antennas, in the reference's order."""

    def __init__(self, num_tx, transmission_mode='TM6', rank=1):
        self.num_tx, self.transmission_mode, self.rank = num_tx, transmission_mode, rank
        if transmission_mode == 'TM6' and rank != 1:
            raise ValueError(f"TM6 solo soporta rank=1, recibido rank={rank}")
        if transmission_mode == 'TM4' and (rank < 1 or rank > min(num_tx, 4)):
            raise ValueError(f"TM4 con {num_tx} antenas soporta rank 1-{min(num_tx, 4)}, recibido rank={rank}")
        if transmission_mode not in ('TM6', 'TM4'):
            raise ValueError(f"Modo {transmission_mode} no soportado")
        self.codebook = self._build()
        self.codebook_size = len(self.codebook)

    # -- tables (TS 36.211-style as the reference defines them, :58-311)
    def _rank1(self):
        n = self.num_tx
        if n == 2:
            return [np.array([[1], [1]]) / np.sqrt(2), np.array([[1], [-1]]) / np.sqrt(2),
                    np.array([[1], [1j]]) / np.sqrt(2), np.array([[1], [-1j]]) / np.sqrt(2)]
        if n in (4, 8):
            div = 2 if n == 4 else np.sqrt(8)
            return [np.exp(1j * (2 * np.pi * i * np.arange(n) / 16)).reshape(-1, 1) / div for i in range(16)]
        raise ValueError(f"num_tx={n} no soportado en TM6")

    def _rank2(self):
        n = self.num_tx
        if n == 2:
            return [np.array([[1, 0], [0, 1]]), np.array([[1, 1], [1, -1]]) / np.sqrt(2),
                    np.array([[1, 1], [1j, -1j]]) / np.sqrt(2)]
        if n == 4:
            ph = [np.exp(1j * (2 * np.pi * i / 4)) for i in range(4)]
            blocks = (lambda x: np.array([[1, 0], [x, 0], [0, 1], [0, x]]) / np.sqrt(2),
                      lambda x: np.array([[1, 1], [x, -x], [1, -1], [x, x]]) / 2,
                      lambda x: np.array([[1, 0], [0, 1], [x, 0], [0, x]]) / np.sqrt(2),
                      lambda x: np.array([[1, 1], [1, -1], [x, x], [x, -x]]) / 2)
            return [f(x) for f in blocks for x in ph]
        if n == 8:
            out = []
            for i in range(16):
                col = np.exp(1j * (2 * np.pi * i / 16) * np.arange(4)) / np.sqrt(4)
                W = np.zeros((8, 2), dtype=complex)
                W[0:4, 0] = col
                W[4:8, 1] = col
                out.append(W)
            return out
        raise ValueError(f"num_tx={n} no soportado en TM4 Rank-2")

    def _rank3(self):
        n = self.num_tx
        if n < 4:
            raise ValueError(f"Rank-3 requiere al menos 4 antenas TX, disponibles: {n}")
        if n == 4:
            return [np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1], [x, x, x]]) / np.sqrt(2)
                    for x in (np.exp(1j * (2 * np.pi * i / 8)) for i in range(8))]
        if n == 8:
            out = []
            for i in range(16):
                th = 2 * np.pi * i / 16
                v = np.array([1, np.exp(1j * th), np.exp(1j * 2 * th)]) / np.sqrt(3)
                W = np.zeros((8, 3), dtype=complex)
                W[0:3, 0] = v
                W[3:6, 1] = v
                W[5:8, 2] = v
                out.append(W)
            return out
        raise ValueError(f"num_tx={n} no soportado en TM4 Rank-3")

    def _rank4(self):
        n = self.num_tx
        if n < 4:
            raise ValueError(f"Rank-4 requiere al menos 4 antenas TX, disponibles: {n}")
        if n == 4:
            F = np.zeros((4, 4), dtype=complex)
            for i in range(4):
                for j in range(4):
                    F[i, j] = np.exp(-2j * np.pi * i * j / 4)
            return [np.eye(4, dtype=complex), F / 2,
                    np.array([[1, 1, 1, 1], [1, -1, 1, -1], [1, 1, -1, -1], [1, -1, -1, 1]]) / 2,
                    np.array([[1, 1, 1, 1], [1, 1j, -1, -1j], [1, -1, 1, -1], [1, -1j, -1, 1j]]) / 2]
        if n == 8:
            out = []
            for i in range(8):
                th = 2 * np.pi * i / 8
                W = np.zeros((8, 4), dtype=complex)
                for lyr in range(4):
                    W[2 * lyr:2 * lyr + 2, lyr] = np.array([1, np.exp(1j * th * (lyr + 1))]) / np.sqrt(2)
                out.append(W)
            return out
        raise ValueError(f"num_tx={n} no soportado en TM4 Rank-4")

    def _build(self):
        if self.transmission_mode == 'TM6':
            return self._rank1()
        return {1: self._rank1, 2: self._rank2, 3: self._rank3, 4: self._rank4}[self.rank]()

    # -- API (:313-433)
    def get_codebook(self):
        return self.codebook

    def get_precoder(self, pmi):
        if pmi < 0 or pmi >= self.codebook_size:
            raise ValueError(f"PMI {pmi} fuera de rango [0, {self.codebook_size-1}]")
        return self.codebook[pmi]

    def select_best_pmi(self, H_channel, metric='capacity'):
        if metric not in ('capacity', 'sinr', 'frobenius'):
            raise ValueError(f"Métrica '{metric}' no soportada")
        best_pmi, best = 0, -np.inf
        for pmi, W in enumerate(self.codebook):
            He = H_channel @ W
            v = np.linalg.norm(He, 'fro') if metric == 'frobenius' else np.sum(np.abs(He) ** 2)
            if v > best:
                best, best_pmi = v, pmi
        return best_pmi, best

    def calculate_quantization_error(self, H_channel, pmi):
        h = np.mean(H_channel, axis=0)
        w_opt = (np.conj(h) / np.linalg.norm(h)).reshape(-1, 1)
        return 1 - np.abs(np.vdot(w_opt.flatten(), self.get_precoder(pmi).flatten())) ** 2

    def print_codebook(self):
        """core/codebook_lte.py:413-433 (debug printout)."""
        print(f"\n{'=' * 60}")
        print(f"Codebook LTE - {self.transmission_mode} - {self.num_tx} TX")
        print(f"{'=' * 60}")
        for pmi, W in enumerate(self.codebook):
            print(f"\nPMI = {pmi}:")
            print(f"  W shape: {W.shape}")
            print("  W = ")
            for row in W:
                real = row.real if np.abs(row.real) > 1e-10 else 0
                imag = row.imag if np.abs(row.imag) > 1e-10 else 0
                if imag >= 0:
                    print(f"    {real:.3f} + {imag:.3f}j")
                else:
                    print(f"    {real:.3f} - {abs(imag):.3f}j")
        print(f"\n{'=' * 60}")

    def get_codebook_info(self):
        return {'num_tx': self.num_tx, 'transmission_mode': self.transmission_mode,
                'codebook_size': self.codebook_size, 'num_layers': self.codebook[0].shape[1],
                'pmi_bits': int(np.ceil(np.log2(self.codebook_size)))}


class RankAdaptation:
    """RankAdaptation (core/rank_adaptation.py:19-272): RI from the eigenvalues
    of H^H H (or capacity), PMI by the TM4 codebook search."""

    def __init__(self, num_tx, num_rx, snr_db=15.0, rank_threshold=0.15):
        self.num_tx, self.num_rx = num_tx, num_rx
        self.snr_db = snr_db
        self.snr_linear = 10 ** (snr_db / 10)
        self.rank_threshold = rank_threshold
        self.max_rank = min(num_tx, num_rx, 4)

    @staticmethod
    def _avg(H):
        return np.mean(H, axis=2) if H.ndim == 3 else H

    def calculate_optimal_rank(self, H_channel, method='eigenvalue'):
        H = self._avg(H_channel)
        if method == 'eigenvalue':
            ev = np.sort(np.linalg.eigvalsh(H.conj().T @ H))[::-1]
            if ev[0] < 1e-10:
                return 1
            ri = min(np.sum(ev / ev[0] > self.rank_threshold), self.max_rank)
            if self.snr_db < 5:
                ri = 1
            elif self.snr_db < 10:
                ri = min(ri, 2)
            return max(1, ri)
        if method == 'capacity':
            s = np.linalg.svd(H, full_matrices=False)[1][:self.max_rank]
            best_rank, best = 1, -np.inf
            for r in range(1, self.max_rank + 1):
                cap = 0
                for i in range(r):
                    if i < len(s):
                        cap += np.log2(1 + self.snr_linear * s[i] ** 2 / r)
                if cap > best:
                    best, best_rank = cap, r
            return best_rank
        raise ValueError(f"Método '{method}' no soportado")

    def select_precoder_for_rank(self, H_channel, rank, metric='capacity'):
        cb = LTECodebook(self.num_tx, transmission_mode='TM4', rank=rank)
        H = self._avg(H_channel)
        best_pmi, best = 0, -np.inf
        for pmi in range(cb.codebook_size):
            He = H @ cb.get_precoder(pmi)
            if metric == 'capacity':
                try:
                    v = np.log2(np.linalg.det(np.eye(self.num_rx) + (self.snr_linear / rank) * (He @ He.conj().T)))
                except Exception:
                    v = 0
            elif metric == 'frobenius':
                v = np.linalg.norm(He, 'fro') ** 2
            elif metric == 'sinr':
                v = np.sum(np.abs(He) ** 2)
            else:
                raise ValueError(f"Métrica '{metric}' no soportada")
            if v > best:
                best, best_pmi = v, pmi
        return best_pmi, cb.get_precoder(best_pmi)

    def get_feedback(self, H_channel, rank_method='eigenvalue', pmi_metric='capacity') -> Dict:
        ri = self.calculate_optimal_rank(H_channel, method=rank_method)
        pmi, W = self.select_precoder_for_rank(H_channel, ri, metric=pmi_metric)
        H = self._avg(H_channel)
        ev = np.sort(np.linalg.eigvalsh(H.conj().T @ H))[::-1]
        sv = np.linalg.svd(H, compute_uv=False)
        return {'ri': ri, 'pmi': pmi, 'W': W, 'eigenvalues': ev, 'condition_number': sv[0] / (sv[-1] + 1e-10)}

    def update_snr(self, new_snr_db):
        self.snr_db = new_snr_db
        self.snr_linear = 10 ** (new_snr_db / 10)


class LayerMapper:
    """LayerMapper (core/layer_mapper.py:14-150): round-robin over rank layers,
    zero-padded to a multiple of rank."""

    def __init__(self, num_layers):
        if num_layers < 1 or num_layers > 8:
            raise ValueError(f"num_layers debe estar en [1,8], recibido: {num_layers}")
        self.num_layers = num_layers

    def map_to_layers(self, symbols):
        s = np.asarray(symbols)
        if self.num_layers == 1:
            return s.reshape(1, -1)
        pad = (-len(s)) % self.num_layers
        if pad:
            s = np.concatenate([s, np.zeros(pad, dtype=s.dtype)])
        return s.reshape(len(s) // self.num_layers, self.num_layers).T

    def demap_from_layers(self, layers, original_length=None):
        layers = np.asarray(layers)
        s = layers.flatten() if self.num_layers == 1 else layers.T.flatten()
        return s if original_length is None else s[:original_length]

    def get_symbols_per_layer(self, total_symbols):
        return total_symbols if self.num_layers == 1 else int(np.ceil(total_symbols / self.num_layers))

    def get_padded_length(self, total_symbols):
        return total_symbols if self.num_layers == 1 else \
            int(np.ceil(total_symbols / self.num_layers)) * self.num_layers


class LayerDemapper:
    """LayerDemapper (core/layer_mapper.py:153-161): LayerMapper.demap_from_layers."""

    def __init__(self, num_layers):
        self.mapper = LayerMapper(num_layers)

    def demap(self, layers, original_length=None):
        return self.mapper.demap_from_layers(layers, original_length)


class MIMODetector:
    """MIMODetector (core/mimo_detector.py:18-369).  detect() runs on the GPU:
    per subcarrier H_eff = H W, then MMSE / IRC, ZF, SIC (ordered successive
    cancellation with hard decisions on `constellation`) or MRC (rank 1)."""

    def __init__(self, num_rx, num_layers, detector_type='MMSE', constellation=None):
        if num_rx < num_layers:
            raise ValueError(f"num_rx ({num_rx}) debe ser >= num_layers ({num_layers})")
        self.num_rx, self.num_layers = num_rx, num_layers
        self.detector_type = detector_type.upper()
        self.symbol_detector = constellation

    def _bps(self):
        c = self.symbol_detector
        if c is None or not isinstance(c, np.ndarray):
            return 0
        bps = {4: 2, 16: 4, 64: 6}.get(len(c), 0)
        if not bps:
            raise NotImplementedError("SIC on the GPU path slices to the QPSK / 16-QAM / 64-QAM constellations")
        return bps

    def detect(self, y_received, H_channel, noise_variance, W_precoder=None):
        det = DETECTORS.get(self.detector_type)
        if det is None:
            raise ValueError(f"Detector '{self.detector_type}' no soportado")
        if det == C.DET_MRC and self.num_layers != 1:
            raise ValueError("MRC solo soporta num_layers=1 (rank-1)")
        y = np.asarray(y_received)
        H = np.asarray(H_channel)
        per_sc = y.ndim == 2 and y.shape[1] > 1
        if not per_sc:
            y = y.reshape(-1, 1)
            H = (H[:, :, :1] if H.ndim == 3 else H[:, :, None])
        elif H.ndim == 2:
            H = np.repeat(H[:, :, None], y.shape[1], axis=2)
        W = W_precoder if W_precoder is not None else np.eye(H.shape[1], dtype=complex)[:, :self.num_layers]
        out = C.mimo_detect(det, y, H, float(noise_variance), np.asarray(W), self._bps())
        return out if per_sc else out[:, 0]


__all__: List[str] = ['LTECodebook', 'RankAdaptation', 'LayerMapper', 'MIMODetector', 'DETECTORS']
