"""Drop-in for the reference's core/sfbc_alamouti.py.

`SFBCAlamouti` keeps the reference's class (core/sfbc_alamouti.py:15-175):
constructor checks, `enabled` pass-through, error messages and the
statistics dict.  `encode` / `decode` run on the MI355X through the C-ABI
stage entries `lte_sfbc_encode_host64` / `lte_sfbc_decode_host64`
(include/lte_phy.h) -- the pair rule and the combiner (`sfbc_combine`,
csrc/lte_mimo.hip) that the SFBC chains (`k_ofdm_tx_mimo<SFBC>`,
`k_det_sfbc`) run, in the reference's float64 arithmetic.

`SFBCResourceMapper` (:166-325) is index bookkeeping around a resource mapper
(data / pilot positions, even / odd pilot split, cell 0 / 1 pilots with the
reference's global-RNG reseed); the chains map on the device.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np

from . import _capi as C
from .ofdm_core import ResourceGrid, _reseed_pilots


class SFBCAlamouti:
    """SFBC Alamouti encoder / decoder for 2 TX antennas (core/sfbc_alamouti.py:15-175).

    Encoding, per pair (s0, s1) on subcarriers (k, k+1):
        TX0: [s0, -conj(s1)]    TX1: [s1, conj(s0)]
    """

    def __init__(self, num_tx: int = 2, enabled: bool = True):
        if num_tx != 2:
            raise ValueError("Alamouti SFBC requires exactly 2 TX antennas")
        self.num_tx = num_tx
        self.enabled = enabled

    def encode(self, symbols: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """SFBCAlamouti.encode (:45-78) on the GPU."""
        if not self.enabled:
            return symbols.copy(), symbols.copy()
        return C.sfbc_encode(np.asarray(symbols))

    def decode(self, rx_symbols: np.ndarray, H0: np.ndarray, H1: np.ndarray,
               regularization: float = 1e-10) -> np.ndarray:
        """SFBCAlamouti.decode (:80-163) on the GPU: per pair
        s0 = [conj(h0_k) r_k + h1_k+1 conj(r_k+1)] / norm,
        s1 = [conj(h1_k) r_k - h0_k+1 conj(r_k+1)] / norm,
        norm = |avg(h0)|^2 + |avg(h1)|^2 + regularization."""
        if not self.enabled:
            return rx_symbols.copy()
        N = len(rx_symbols)
        if N % 2 != 0:
            raise ValueError(f"Number of RX symbols must be even, got {N}")
        if len(H0) != N or len(H1) != N:
            raise ValueError(f"Channel estimates must have length {N}")
        return C.sfbc_decode(rx_symbols, H0, H1, regularization)

    def get_statistics(self) -> Dict:
        return {'enabled': self.enabled, 'num_tx': self.num_tx, 'coding_scheme': 'Alamouti SFBC',
                'rate': 1.0, 'diversity_order': 2}


class SFBCResourceMapper:
    """SFBCResourceMapper (core/sfbc_alamouti.py:166-325).  `resource_mapper`
    is the reference's ResourceMapper (anything with get_data_indices(),
    config.N and grid.get_pilot_indices()) or an LTEConfig, for which the
    LTEResourceGrid layout (ResourceGrid) is used."""

    def __init__(self, resource_mapper):
        if not hasattr(resource_mapper, 'get_data_indices'):
            resource_mapper = _GridMapper(resource_mapper)
        self.resource_mapper = resource_mapper
        self.data_indices = resource_mapper.get_data_indices()
        self.num_data = len(self.data_indices)
        if self.num_data % 2 != 0:
            print(f"[WARNING] Odd number of data subcarriers ({self.num_data}). "
                  f"Last subcarrier will be nulled for SFBC.")
            self.num_data -= 1
            self.data_indices = self.data_indices[:self.num_data]

    def prepare_data_for_sfbc(self, qam_symbols: np.ndarray) -> np.ndarray:
        if len(qam_symbols) < self.num_data:
            return np.pad(qam_symbols, (0, self.num_data - len(qam_symbols)), 'constant', constant_values=0)
        if len(qam_symbols) > self.num_data:
            return qam_symbols[:self.num_data]
        return qam_symbols

    def map_sfbc_to_grid(self, tx0_symbols: np.ndarray, tx1_symbols: np.ndarray,
                         pilot_symbols: Optional[np.ndarray] = None) -> Tuple[np.ndarray, np.ndarray]:
        """Data on the data SCs; TX0 pilots (cell 0) on the even pilot
        positions, TX1 pilots (cell 1) on the odd ones (:215-265).  Each
        PilotPattern reseeds the global NumPy RNG (quirk Q1), reproduced."""
        N = self.resource_mapper.config.N
        g0 = np.zeros(N, dtype=complex)
        g1 = np.zeros(N, dtype=complex)
        g0[self.data_indices] = tx0_symbols[:self.num_data]
        g1[self.data_indices] = tx1_symbols[:self.num_data]
        pil = self.resource_mapper.grid.get_pilot_indices()
        p0, p1 = pil[::2], pil[1::2]
        g0[p0] = C.pilots(0, len(p0))
        _reseed_pilots(0, len(p0))
        g1[p1] = C.pilots(1, len(p1))
        _reseed_pilots(1, len(p1))
        return g0, g1

    def extract_data_from_grid(self, rx_grid: np.ndarray) -> np.ndarray:
        return rx_grid[self.data_indices]

    def apply_generic_precoding(self, symbols: np.ndarray, W_matrix: np.ndarray) -> List[np.ndarray]:
        """tx[i] = sum_l W[i, l] symbols[l] (:267-325), layers accumulated in
        order onto zeros as the reference does."""
        if symbols.ndim == 1:
            symbols = symbols.reshape(1, -1)
        num_layers, num_data = symbols.shape
        if W_matrix.shape[1] != num_layers:
            raise ValueError(f"W_matrix shape {W_matrix.shape} no compatible con {num_layers} layers")
        out = []
        for t in range(W_matrix.shape[0]):
            s = np.zeros(num_data, dtype=complex)
            for l in range(num_layers):
                s += W_matrix[t, l] * symbols[l, :]
            out.append(s)
        return out


class _GridMapper:
    """The parts of ResourceMapper (core/resource_mapper.py:155-230) that
    SFBCResourceMapper reads, over an LTEConfig."""

    def __init__(self, config):
        self.config = config
        self.grid = ResourceGrid(config.N, config.Nc)

    def get_data_indices(self):
        return self.grid.get_data_indices()
