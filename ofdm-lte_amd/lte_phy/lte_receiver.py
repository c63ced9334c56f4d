"""Drop-in mirror of core/lte_receiver.py: LTEChannelEstimator, LTEEqualizerZF
and LTEReceiver.

Each step runs on the GPU through a stage entry: FFT / sqrt(N)
(`lte_fft_host64`), LS estimation at the pilots + linear interpolation +
pilot statistics (`lte_chest_host64`), ZF (`lte_zf_host64`), SC-FDM IDFT
(`lte_dft_host64`), nearest-point decisions (`lte_nearest_host64`).  The host
slices symbols, gathers the data subcarriers and reproduces the reference's
global-RNG reseeds (quirk Q1).  The fused receivers of the simulators
(`k_rx_frame` & co.) compute the same rows in one pass per frame; this module
is the reference's class-level API over the same device arithmetic.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np

from . import _capi as C
from .dft_precoding import SC_FDMDecodifier
from .modulator import QAMModulator, bits_to_index, hard_bits
from .resource_mapper import LTEResourceGrid, PilotPattern


def chest(Y, pilot_indices, known, stats=True):
    """LS + np.linspace interpolation for a batch of grids Y [..., N] on the
    GPU (lte_chest_host64): (H [..., N], LS at the pilots [..., P],
    stats [..., 2] = mean |Y_p|^2, mean |Y_p - X_p|^2)."""
    Y = np.ascontiguousarray(Y, dtype=np.complex128)
    N = Y.shape[-1]
    pidx = np.ascontiguousarray(pilot_indices, dtype=np.int32)
    X = np.ascontiguousarray(known, dtype=np.complex128)
    if len(pidx) == 0:
        raise IndexError("index 0 is out of bounds for axis 0 with size 0")
    if len(X) != len(pidx):
        raise ValueError(f"operands could not be broadcast together with shapes ({len(pidx)},) ({len(X)},)")
    batch = Y.size // N
    H = np.empty_like(Y)
    hp = np.empty(Y.shape[:-1] + (len(pidx),), dtype=np.complex128)
    st = np.empty(Y.shape[:-1] + (2,), dtype=np.float64)
    C.device_init()
    C.check(C.load().lte_chest_host64(N, len(pidx), C.ptr(pidx, C.I32), C.ptr(X.view(np.float64), C.F64), batch,
                                      C.ptr(Y.view(np.float64), C.F64), C.ptr(H.view(np.float64), C.F64),
                                      C.ptr(hp.view(np.float64), C.F64), C.ptr(st, C.F64) if stats else None))
    return H, hp, st


def zf(Y, H, regularization):
    """Y / (H + regularization) on the GPU (lte_zf_host64)."""
    Y = np.ascontiguousarray(Y, dtype=np.complex128)
    Hb = np.ascontiguousarray(np.broadcast_to(np.asarray(H, dtype=np.complex128), Y.shape))
    out = np.empty_like(Y)
    if Y.size:
        C.device_init()
        C.check(C.load().lte_zf_host64(Y.size, C.ptr(Y.view(np.float64), C.F64), C.ptr(Hb.view(np.float64), C.F64),
                                       float(regularization), C.ptr(out.view(np.float64), C.F64)))
    return out


def ofdm_symbols(signal, N, cp):
    """_demodulate_ofdm_stream (core/lte_receiver.py:444-491): the stream cut
    into (N + CP)-sample symbols (at least one, the last zero-padded), CP
    removed, FFT / sqrt(N) on the GPU: [n_sym, N]."""
    sl = N + cp
    x = np.asarray(signal, dtype=np.complex128).ravel()
    n = max(1, len(x) // sl)
    buf = np.zeros(n * sl, dtype=np.complex128)
    m = min(len(x), n * sl)
    buf[:m] = x[:m]
    return C.fft(buf.reshape(n, sl)[:, cp:], inverse=False, precision='f64')


class LTEChannelEstimator:
    """LTEChannelEstimator (core/lte_receiver.py:20-133)."""

    def __init__(self, config, cell_id=0):
        self.config = config
        self.cell_id = cell_id
        self.resource_grid = LTEResourceGrid(config.N, config.Nc)
        self.pilot_pattern = PilotPattern(cell_id)

    def estimate_channel(self, received_signal: np.ndarray, tx_signal: Optional[np.ndarray] = None) -> Dict:
        N = self.config.N
        pilot_indices = self.resource_grid.get_pilot_indices()
        known = self.pilot_pattern.generate_pilots(len(pilot_indices))
        Y = np.asarray(received_signal, dtype=np.complex128)
        # the reference reads received_signal[pilot_indices] and interpolates onto N subcarriers
        if len(Y) <= pilot_indices[-1]:
            bad = int(pilot_indices[pilot_indices >= len(Y)][0])
            raise IndexError(f"index {bad} is out of bounds for axis 0 with size {len(Y)}")
        Yn = np.zeros(N, dtype=np.complex128)
        m = min(N, len(Y))
        Yn[:m] = Y[:m]
        H, hp, st = chest(Yn, pilot_indices, known)
        pilot_snr = st[0] / (st[1] + 1e-10)
        return {'channel_estimate': H, 'pilot_channel': hp, 'pilot_indices': pilot_indices,
                'pilot_snr_linear': pilot_snr, 'pilot_snr_db': 10 * np.log10(pilot_snr + 1e-10), 'interpolated': True}

    def _interpolate_channel(self, pilot_indices: np.ndarray, pilot_values: np.ndarray,
                             total_subcarriers: int) -> np.ndarray:
        """Edge hold + np.linspace between pilots (:98-133) on the GPU: the
        estimator kernel on a grid whose pilots are the values themselves
        (Y_p / 1 = Y_p exactly)."""
        pidx = np.asarray(pilot_indices)
        Y = np.zeros(int(total_subcarriers), dtype=np.complex128)
        Y[pidx] = pilot_values
        H, _, _ = chest(Y, pidx, np.ones(len(pidx), dtype=np.complex128), stats=False)
        return H


class LTEEqualizerZF:
    """LTEEqualizerZF (core/lte_receiver.py:136-180): Y / (H + reg)."""

    def __init__(self, config, regularization=1e-6):
        self.config = config
        self.regularization = regularization

    def equalize(self, received_symbols: np.ndarray, channel_estimate: np.ndarray) -> np.ndarray:
        return zf(received_symbols, channel_estimate, self.regularization)


class LTEReceiver:
    """LTEReceiver (core/lte_receiver.py:183-557): FFT, slot-periodic LS
    estimation (every 14 symbols), ZF, data extraction, optional SC-FDM IDFT,
    nearest-point detection."""

    def __init__(self, config, cell_id=0, enable_equalization=True, enable_sc_fdm=False):
        self.config = config
        self.cell_id = cell_id
        self.enable_equalization = enable_equalization
        self.enable_sc_fdm = enable_sc_fdm
        self.resource_grid = LTEResourceGrid(config.N, config.Nc)
        self.pilot_pattern = PilotPattern(cell_id)
        self.channel_estimator = LTEChannelEstimator(config, cell_id)
        self.equalizer = LTEEqualizerZF(config)
        self.qam_demodulator = QAMModulator(config.modulation)
        self.sc_fdm_decoder = (SC_FDMDecodifier(num_data_subcarriers=len(self.resource_grid.get_data_indices()),
                                                enable=True) if enable_sc_fdm else None)
        self.channel_estimates = []
        self.equalization_info = []
        self.slot_size = 14

    def receive_and_decode(self, received_ofdm_signal: np.ndarray) -> Dict:
        syms = self._demodulate_ofdm_stream(received_ofdm_signal)
        received_symbols = np.concatenate(syms)
        n_sym = len(syms)
        per_symbol, channel_snr_db = self._estimate_channel_periodic(syms)
        channel_estimate = per_symbol[0]
        if self.enable_equalization:
            symbols_equalized = self._equalize_with_periodic_estimates(syms, per_symbol)
        else:
            symbols_equalized = received_symbols
        data_indices = self.resource_grid.get_data_indices()
        all_idx = (data_indices[None, :] + self.config.N * np.arange(n_sym)[:, None]).ravel()
        symbols_data = symbols_equalized[all_idx[all_idx < len(symbols_equalized)]]
        if self.enable_sc_fdm and self.sc_fdm_decoder is not None:
            nd = len(data_indices)
            k = len(symbols_data) // nd
            if k:
                symbols_data = C.dft(symbols_data[:k * nd].reshape(k, nd), inverse=True, precision='f64').ravel()
        symbols_detected = self._detect_symbols(symbols_data)
        bits = self.qam_demodulator.symbols_to_bits(symbols_detected)
        self.channel_estimates.append(channel_estimate)
        self.equalization_info.append({'channel_snr_db': channel_snr_db, 'num_data_symbols': len(symbols_data)})
        return {'symbols_received': received_symbols, 'symbols_equalized': symbols_equalized,
                'symbols_data_only': symbols_data, 'symbols_detected': symbols_detected, 'bits': bits,
                'channel_estimate': channel_estimate, 'channel_snr_db': channel_snr_db,
                'pilot_snr_db': channel_snr_db, 'num_data_symbols': len(symbols_data),
                'num_pilot_symbols': len(self.resource_grid.get_pilot_indices()) * n_sym,
                'equalization_enabled': self.enable_equalization}

    def _estimate_channel_periodic(self, all_received_symbols: List[np.ndarray]) -> Tuple[List[np.ndarray], float]:
        """One estimate from the first symbol of every 14-symbol slot, reused
        for the slot (:360-411); all slots in one GPU call."""
        n = len(all_received_symbols)
        starts = list(range(0, n, self.slot_size))
        if not starts:
            return [], 0.0
        pidx = self.resource_grid.get_pilot_indices()
        known = None
        for _ in starts:   # one generate_pilots per slot, as the reference (RNG reseed each time)
            known = self.channel_estimator.pilot_pattern.generate_pilots(len(pidx))
        H, _, st = chest(np.stack([all_received_symbols[s] for s in starts]), pidx, known)
        snr = st[:, 0] / (st[:, 1] + 1e-10)
        snr_db = [10 * np.log10(v + 1e-10) for v in snr]
        per_symbol = []
        for i, s in enumerate(starts):
            per_symbol += [H[i]] * (min(s + self.slot_size, n) - s)
        return per_symbol, np.mean(snr_db)

    def _equalize_with_periodic_estimates(self, all_received_symbols: List[np.ndarray],
                                          channel_estimates_per_symbol: List[np.ndarray]) -> np.ndarray:
        if not all_received_symbols:
            return np.array([])
        Y = np.stack(all_received_symbols)
        H = np.stack([channel_estimates_per_symbol[min(i, len(channel_estimates_per_symbol) - 1)]
                      for i in range(len(all_received_symbols))])
        return self.equalizer.equalize(Y, H).ravel()

    def _demodulate_ofdm_stream(self, received_signal: np.ndarray) -> List[np.ndarray]:
        return list(ofdm_symbols(received_signal, self.config.N, self.config.cp_length))

    def _demodulate_ofdm(self, received_signal: np.ndarray) -> np.ndarray:
        s = self._demodulate_ofdm_stream(received_signal)
        return np.concatenate(s) if len(s) > 1 else s[0]

    def _detect_symbols(self, received_symbols: np.ndarray) -> np.ndarray:
        """Nearest constellation point (:508-521): GPU decisions, the point of
        each decided index."""
        y = np.asarray(received_symbols)
        if y.size == 0:
            return np.zeros_like(y)
        bps = int(np.log2(len(self.qam_demodulator.constellation)))
        idx = bits_to_index(hard_bits(y, bps), bps)
        return self.qam_demodulator.get_constellation()[idx].astype(y.dtype if np.iscomplexobj(y) else complex)

    def calculate_ber(self, transmitted_bits: np.ndarray, received_bits: np.ndarray) -> Dict:
        n = min(len(transmitted_bits), len(received_bits))
        errors = np.sum(transmitted_bits[:n] != received_bits[:n])
        return {'ber': errors / n if n > 0 else 0, 'errors': errors, 'total_bits': n}

    def reset_history(self):
        self.channel_estimates = []
        self.equalization_info = []

    def get_channel_estimate_history(self) -> np.ndarray:
        return np.array(self.channel_estimates)
