"""Drop-in mirror of core/demodulator.py: OFDMDemodulator ('simple' FFT
demodulation or the LTE receiver) and SymbolDetector.  FFTs, SC-FDM IDFTs and
decisions run on the GPU (lte_fft_host64, lte_dft_host64, lte_nearest_host64);
mode 'lte' is LTEReceiver.receive_and_decode."""
from __future__ import annotations

import numpy as np

from . import _capi as C
from .dft_precoding import SC_FDMDecodifier
from .lte_receiver import LTEReceiver
from .modulator import BPS_OF, QAMModulator, bits_to_index, constellation, hard_bits
from .resource_mapper import ResourceMapper


class OFDMDemodulator:
    """OFDMDemodulator (core/demodulator.py:15-188)."""

    def __init__(self, config, mode='simple', enable_equalization=False, enable_sc_fdm=False):
        self.config = config
        self.mode = mode
        self.enable_equalization = enable_equalization
        self.enable_sc_fdm = enable_sc_fdm
        self.qam_demodulator = QAMModulator(config.modulation)
        self.resource_mapper = None
        self.sc_fdm_decoder = None
        if self.mode == 'lte' or self.enable_sc_fdm:
            self.resource_mapper = ResourceMapper(config)
            if self.enable_sc_fdm:
                self.sc_fdm_decoder = SC_FDMDecodifier(
                    num_data_subcarriers=len(self.resource_mapper.get_data_indices()), enable=True)
        self.lte_receiver = (LTEReceiver(config, cell_id=0, enable_equalization=enable_equalization,
                                         enable_sc_fdm=enable_sc_fdm) if self.mode == 'lte' else None)

    def demodulate(self, received_signal):
        """One OFDM symbol: CP removal, FFT / sqrt(N), the data subcarriers
        through the SC-FDM IDFT or the first Nc subcarriers (:68-118)."""
        cfg = self.config
        L = cfg.N + cfg.cp_length
        x = np.asarray(received_signal)
        if len(x) < L:
            x = np.pad(x, (0, L - len(x)), 'constant')
        f = C.fft(np.asarray(x[cfg.cp_length:L], dtype=np.complex128), inverse=False, precision='f64')
        if self.enable_sc_fdm and self.sc_fdm_decoder is not None and self.resource_mapper is not None:
            return self.sc_fdm_decoder.decoding(f[self.resource_mapper.get_data_indices()])
        return f[:cfg.Nc]

    def demodulate_stream(self, received_signal, num_ofdm_symbols=None, resource_grid=None):
        """(symbols, bits) of a stream (:120-184): mode 'lte' through the LTE
        receiver, 'simple' symbol by symbol."""
        if self.mode == 'lte' and self.lte_receiver is not None:
            symbols_data = self.lte_receiver.receive_and_decode(received_signal)['symbols_data_only']
            return symbols_data, self.qam_demodulator.symbols_to_bits(symbols_data)
        spl = self.config.N + self.config.cp_length
        x = np.asarray(received_signal)
        if num_ofdm_symbols is None:
            num_ofdm_symbols = int(np.ceil(len(x) / spl))
        syms, bits = [], []
        for i in range(num_ofdm_symbols):
            a, e = i * spl, (i + 1) * spl
            chunk = np.pad(x[a:], (0, e - len(x)), 'constant') if e > len(x) else x[a:e]
            s = self.demodulate(chunk)
            syms.append(s)
            bits.append(self.qam_demodulator.symbols_to_bits(s))
        return np.concatenate(syms), np.concatenate(bits)

    def get_qam_demodulator(self):
        return self.qam_demodulator


class SymbolDetector:
    """SymbolDetector (core/demodulator.py:191-245): nearest constellation
    point (argmin |c - y|, ties -> the first).  The GPU slicer serves the LTE
    constellations (QPSK / 16-QAM / 64-QAM tables of QAMModulator)."""

    def __init__(self, constellation):
        self.constellation = constellation
        self._bps = None
        c = np.asarray(constellation)
        for mod, bps in BPS_OF.items():
            ref = globals()['constellation'](mod)
            if c.shape == ref.shape and np.array_equal(c, ref):
                self._bps = bps

    def _detect(self, y):
        if self._bps is None:
            raise NotImplementedError("the GPU slicer serves the QPSK / 16-QAM / 64-QAM constellations of "
                                      "QAMModulator")
        idx = bits_to_index(hard_bits(y, self._bps), self._bps)
        return np.asarray(self.constellation)[idx]

    def detect(self, received_symbol):
        return self._detect(np.atleast_1d(np.asarray(received_symbol, dtype=np.complex128)))[0]

    def detect_batch(self, received_symbols):
        y = np.asarray(received_symbols)
        detected = np.zeros_like(y)
        if y.size:
            detected[...] = self._detect(y.astype(np.complex128).ravel()).reshape(y.shape)
        return detected

    def calculate_error_rate(self, transmitted_symbols, received_symbols):
        return np.sum(transmitted_symbols != received_symbols) / len(transmitted_symbols)
