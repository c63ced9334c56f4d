"""Drop-in mirror of core/dft_precoding.py: the SC-FDM DFT precoder and IDFT
decoder.  Every transform runs on the GPU (lte_dft_host64: the unitary
M-point DFT / IDFT by Bluestein's chirp-z on the LDS FFT, M <= 1024 -- the
reference's matrix products are the same transform, equal to round-off);
no M x M matrix is ever built."""
from __future__ import annotations

from typing import Dict

import numpy as np

from . import _capi as C


def _check_len(symbols, M):
    if len(symbols) != M:
        raise ValueError(f"Tamaño de símbolos ({len(symbols)}) debe ser igual a M ({M})")


class DFTPrecodifier:
    """DFTPrecodifier (core/dft_precoding.py:20-130): X = DFT_M(x) / sqrt(M)."""

    def __init__(self, M: int = None, enable: bool = True):
        self.M = M
        self.enable = enable
        self._ready = M is not None and enable

    def set_size(self, M: int):
        self.M = M
        if self.enable:
            self._ready = True

    def precoding(self, symbols: np.ndarray) -> np.ndarray:
        if not self.enable or self.M is None:
            return symbols
        _check_len(symbols, self.M)
        return C.dft(np.asarray(symbols, dtype=np.complex128), inverse=False, precision='f64')

    def precoding_ifft(self, symbols: np.ndarray) -> np.ndarray:
        """np.fft.fft(x) / sqrt(M): the same transform (core/dft_precoding.py:95-122)."""
        return self.precoding(symbols)

    def get_statistics(self) -> Dict:
        return {'enabled': self.enable, 'dft_size': self.M, 'matrix_computed': self._ready}


class IDFTDecodifier:
    """IDFTDecodifier (core/dft_precoding.py:133-251): x = IDFT_M(X) * sqrt(M) / M."""

    def __init__(self, M: int = None, enable: bool = True):
        self.M = M
        self.enable = enable
        self._ready = M is not None and enable

    def set_size(self, M: int):
        self.M = M
        if self.enable:
            self._ready = True

    def decoding(self, precoded_symbols: np.ndarray) -> np.ndarray:
        if not self.enable or self.M is None:
            return precoded_symbols
        _check_len(precoded_symbols, self.M)
        return C.dft(np.asarray(precoded_symbols, dtype=np.complex128), inverse=True, precision='f64')

    def decoding_fft(self, precoded_symbols: np.ndarray) -> np.ndarray:
        """np.fft.ifft(X) * sqrt(M): the same transform (core/dft_precoding.py:218-243)."""
        return self.decoding(precoded_symbols)

    def get_statistics(self) -> Dict:
        return {'enabled': self.enable, 'idft_size': self.M, 'matrix_computed': self._ready}


class SC_FDMPrecodifier:
    """SC_FDMPrecodifier (core/dft_precoding.py:254-300)."""

    def __init__(self, num_data_subcarriers: int, enable: bool = True):
        self.num_data_subcarriers = num_data_subcarriers
        self.enable = enable
        self.dft_precoder = DFTPrecodifier(M=num_data_subcarriers, enable=enable)

    def precoding(self, data_symbols: np.ndarray) -> np.ndarray:
        return self.dft_precoder.precoding(data_symbols)

    def set_enable(self, enable: bool):
        self.enable = enable
        self.dft_precoder.enable = enable

    def get_statistics(self) -> Dict:
        return {'enabled': self.enable, 'num_data_subcarriers': self.num_data_subcarriers,
                'dft_info': self.dft_precoder.get_statistics()}


class SC_FDMDecodifier:
    """SC_FDMDecodifier (core/dft_precoding.py:303-348)."""

    def __init__(self, num_data_subcarriers: int, enable: bool = True):
        self.num_data_subcarriers = num_data_subcarriers
        self.enable = enable
        self.idft_decoder = IDFTDecodifier(M=num_data_subcarriers, enable=enable)

    def decoding(self, precoded_symbols: np.ndarray) -> np.ndarray:
        return self.idft_decoder.decoding(precoded_symbols)

    def set_enable(self, enable: bool):
        self.enable = enable
        self.idft_decoder.enable = enable

    def get_statistics(self) -> Dict:
        return {'enabled': self.enable, 'num_data_subcarriers': self.num_data_subcarriers,
                'idft_info': self.idft_decoder.get_statistics()}
