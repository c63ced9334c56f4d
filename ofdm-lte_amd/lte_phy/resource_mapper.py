"""Drop-in mirror of core/resource_mapper.py: the LTE resource grid, the pilot
pattern (with the reference's global-RNG reseed, quirk Q1) and the RE mapper.

The grid is index bookkeeping (host); pilot values come from the library's
native MT19937 (`lte_pilots`); the OFDM symbol of EnhancedOFDMModulator is
mapped on the GPU (`lte_qam_map_host64`) and transformed there
(`lte_fft_host64`).
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np

from . import _capi as C


def _reseed_pilots(cell_id, n):
    """PilotPattern.generate_pilots side effect (core/resource_mapper.py:148):
    the reference reseeds the GLOBAL NumPy RNG every time pilots are made."""
    np.random.seed(cell_id)
    np.random.choice([1, -1], size=n)


class LTEResourceGrid:
    """LTEResourceGrid (core/resource_mapper.py:17-111): guard bands, DC null
    at N/2, a pilot on every 6th useful subcarrier (offset 3), data elsewhere."""

    def __init__(self, N: int, Nc: int):
        self.N, self.Nc = N, Nc
        self.num_guard_left = (N - Nc) // 2
        self.num_guard_right = N - Nc - self.num_guard_left
        self.dc_index = N // 2
        self.pilot_spacing = 6
        self._init_subcarrier_types()

    def _init_subcarrier_types(self):
        """Subcarrier classes (core/resource_mapper.py:57-74), vectorised: the
        same index sets as the reference's per-k loop, and its dict."""
        N = self.N
        k = np.arange(N)
        guard = (k < self.num_guard_left) | (k >= N - self.num_guard_right)
        dc = (k == self.dc_index) & ~guard
        pilot = ~guard & ~dc & (((k - self.num_guard_left) % self.pilot_spacing) == self.pilot_spacing // 2)
        self._data = k[~guard & ~dc & ~pilot]
        self._pilot = k[pilot]
        self._guard = k[guard]
        types = np.where(guard, 'guard', np.where(dc, 'dc', np.where(pilot, 'pilot', 'data')))
        self.subcarrier_types = {int(i): str(t) for i, t in enumerate(types)}

    def get_subcarrier_type(self, k: int) -> str:
        return self.subcarrier_types.get(k, 'guard')

    def get_data_indices(self) -> np.ndarray:
        return self._data.copy()

    def get_pilot_indices(self) -> np.ndarray:
        return self._pilot.copy()

    def get_guard_indices(self) -> np.ndarray:
        return self._guard.copy()

    def get_statistics(self) -> Dict:
        return {'total_subcarriers': self.N, 'useful_subcarriers': self.Nc,
                'data_subcarriers': len(self._data), 'pilot_subcarriers': len(self._pilot),
                'guard_subcarriers': len(self._guard), 'dc_subcarriers': 1,
                'guard_left': self.num_guard_left, 'guard_right': self.num_guard_right,
                'pilot_spacing': self.pilot_spacing}


class PilotPattern:
    """PilotPattern (core/resource_mapper.py:114-152): np.random.seed(cell_id),
    choice([1, -1], n) times the pilot symbol ((1 + 1j) / sqrt 2 by default).
    Values from the library's MT19937 (lte_pilots, prefix-stable); the global
    NumPy RNG is left where the reference leaves it."""

    def __init__(self, cell_id: int = 0, pilot_symbol_value: complex = None):
        self.cell_id = cell_id
        self.pilot_symbol_value = (1 + 1j) / np.sqrt(2) if pilot_symbol_value is None else pilot_symbol_value

    def generate_pilots(self, num_pilots: int) -> np.ndarray:
        n = int(num_pilots)
        if n < 0:
            raise ValueError("negative dimensions are not allowed")
        base = C.pilots(int(self.cell_id), n) if n else np.zeros(0, dtype=np.complex128)
        _reseed_pilots(self.cell_id, n)
        phases = np.where(base.real < 0, -1, 1)
        return self.pilot_symbol_value * phases


class ResourceMapper:
    """ResourceMapper (core/resource_mapper.py:155-267): data on the data
    subcarriers, pilots on the pilot subcarriers, DC and guards null."""

    def __init__(self, config, cell_id: int = 0):
        self.config = config
        self.grid = LTEResourceGrid(config.N, config.Nc)
        self.pilot_pattern = PilotPattern(cell_id)
        self.stats = self.grid.get_statistics()

    def map_symbols(self, data_symbols: np.ndarray) -> Tuple[np.ndarray, Dict]:
        grid_mapped = np.zeros(self.config.N, dtype=complex)
        data_indices = self.grid.get_data_indices()
        pilot_indices = self.grid.get_pilot_indices()
        n = min(len(data_symbols), len(data_indices))
        grid_mapped[data_indices[:n]] = data_symbols[:n]
        grid_mapped[pilot_indices] = self.pilot_pattern.generate_pilots(len(pilot_indices))
        return grid_mapped, {
            'num_data_mapped': n, 'num_pilots_mapped': len(pilot_indices),
            'num_nulls': len(self.grid.get_guard_indices()) + 1, 'data_indices': data_indices[:n],
            'pilot_indices': pilot_indices, 'guard_indices': self.grid.get_guard_indices(),
            'dc_index': self.grid.dc_index, 'grid_statistics': self.stats}

    def extract_pilots(self, received_grid: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        pilot_indices = self.grid.get_pilot_indices()
        return pilot_indices, received_grid[pilot_indices]

    def get_data_indices(self) -> np.ndarray:
        return self.grid.get_data_indices()

    def get_statistics(self) -> Dict:
        return self.stats

    def print_grid_structure(self):
        s, N = self.stats, self.config.N
        print("\n" + "=" * 80)
        print("ESTRUCTURA DE GRID DE RECURSOS LTE")
        print("=" * 80)
        print(f"\nTamaño FFT (N): {N}")
        print(f"Subportadoras útiles (Nc): {self.config.Nc}")
        print("\nDistribución:")
        print(f"  Guard band izquierdo: {s['guard_left']} subportadoras")
        print(f"  Datos: {s['data_subcarriers']} subportadoras")
        print(f"  Pilotos: {s['pilot_subcarriers']} subportadoras")
        print(f"  DC (nulo): 1 subportadora (índice {self.grid.dc_index})")
        print(f"  Guard band derecho: {s['guard_right']} subportadoras")
        print(f"  Guardias totales (incluyendo DC): {s['guard_subcarriers'] + 1}")
        print("\nEficiencia espectral:")
        print(f"  Datos útiles: {s['data_subcarriers']} / {N} = {s['data_subcarriers'] / N * 100:.1f}%")
        print(f"  Overhead de pilotos: {s['pilot_subcarriers']} / {N} = {s['pilot_subcarriers'] / N * 100:.1f}%")
        print("\n" + "=" * 80)


def ofdm_symbol(grid_mapped, cp_length):
    """IFFT * sqrt(N) on the GPU (lte_fft_host64) and the cyclic prefix
    (core/modulator.py:242-248)."""
    t = C.fft(np.asarray(grid_mapped, dtype=np.complex128), inverse=True, precision='f64')
    return np.concatenate([t[-cp_length:], t])


class EnhancedOFDMModulator:
    """EnhancedOFDMModulator (core/resource_mapper.py:270-324): QAM map,
    resource mapping, IFFT, CP for one OFDM symbol."""

    def __init__(self, config, qam_modulator):
        self.config = config
        self.qam_modulator = qam_modulator
        self.resource_mapper = ResourceMapper(config)

    def modulate_with_mapping(self, bits: np.ndarray) -> Tuple[np.ndarray, Dict]:
        qam_symbols = self.qam_modulator.bits_to_symbols(bits)
        grid_mapped, mapping_info = self.resource_mapper.map_symbols(qam_symbols)
        return ofdm_symbol(grid_mapped, self.config.cp_length), mapping_info

    def get_resource_mapper(self) -> ResourceMapper:
        return self.resource_mapper
