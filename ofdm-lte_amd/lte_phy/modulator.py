"""Drop-in mirror of core/modulator.py: QAMModulator, OFDMModulator and the
QPSK soft demapper.

The arithmetic runs on the GPU through the library's stage entries: QAM map
(`lte_qam_map_host64`, the chains' constellation), nearest-point decisions
(`lte_nearest_host64`: the reference's own distance and argmin), LLRs
(`lte_llr_host64`), IFFT (`lte_fft_host64`), SC-FDM DFT (`lte_dft_host64`); a
whole LTE / SC-FDM stream is one plan call (`OFDMTransmitter`'s TX stage).
The host does index bookkeeping only.
"""
from __future__ import annotations

import numpy as np

from . import _capi as C
from .dft_precoding import SC_FDMPrecodifier
from .resource_mapper import ResourceMapper, ofdm_symbol

BPS_OF = {'QPSK': 2, '16-QAM': 4, '64-QAM': 6}


def constellation(mod):
    """QAMModulator._generate_constellation (core/modulator.py:28-59) (host table)."""
    if mod == 'QPSK':
        return np.array([1 + 1j, 1 - 1j, -1 + 1j, -1 - 1j]) / np.sqrt(2)
    if mod not in ('16-QAM', '64-QAM'):
        raise ValueError(f"Modulación no soportada: {mod}")
    lv = [-3, -1, 1, 3] if mod == '16-QAM' else [-7, -5, -3, -1, 1, 3, 5, 7]
    sc = np.sqrt(10) if mod == '16-QAM' else np.sqrt(42)
    return np.array([r + 1j * i for r in lv for i in lv]) / sc


def _bits_u8(bits):
    """0 / 1 bytes of a bit array; any other value is the reference's
    int(''.join(...), 2) failure (core/modulator.py:84)."""
    b = np.asarray(bits)
    if b.size and not np.all((b == 0) | (b == 1)):
        bad = b[(b != 0) & (b != 1)].ravel()[0]
        raise ValueError(f"invalid literal for int() with base 2: '{bad}'")
    return np.ascontiguousarray(b, dtype=np.uint8)


def map_bits(bits, bps):
    """bits (a whole number of symbols) -> constellation points on the GPU."""
    b = _bits_u8(bits)
    n = len(b) // bps
    out = np.empty(n, dtype=np.complex128)
    if n:
        C.device_init()
        C.check(C.load().lte_qam_map_host64(bps, n, C.ptr(b, C.U8), C.ptr(out.view(np.float64), C.F64)))
    return out


def hard_bits(symbols, bps):
    """Nearest-point decisions as the reference takes them (np.abs(c - y),
    np.argmin: the first of equal distances, decision boundaries included)
    as MSB-first bits, on the GPU (lte_nearest_host64): uint8 [n * bps]."""
    y = np.ascontiguousarray(symbols, dtype=np.complex128).ravel()
    out = np.empty(len(y) * bps, dtype=np.uint8)
    if len(y):
        C.device_init()
        C.check(C.load().lte_nearest_host64(bps, len(y), C.ptr(y.view(np.float64), C.F64), C.ptr(out, C.U8)))
    return out


def bits_to_index(bits, bps):
    b = np.asarray(bits, dtype=np.int64).reshape(-1, bps)
    return b @ (1 << np.arange(bps - 1, -1, -1))


class QAMModulator:
    """QAMModulator (core/modulator.py:15-116)."""

    def __init__(self, modulation_type='QPSK'):
        self.modulation_type = modulation_type
        self.constellation = self._generate_constellation()

    def _generate_constellation(self):
        return constellation(self.modulation_type)

    @property
    def _bps(self):
        return int(np.log2(len(self.constellation)))

    def bits_to_symbols(self, bits):
        """Pad to whole symbols with zeros, MSB-first index -> point (:61-88)."""
        bps = self._bps
        bits = np.asarray(bits)
        if len(bits) % bps != 0:
            bits = np.pad(bits, (0, bps - len(bits) % bps), 'constant')
        if self.modulation_type not in BPS_OF:   # a constellation set by hand: not the chains' table
            raise NotImplementedError("the GPU map serves the QPSK / 16-QAM / 64-QAM constellations")
        return map_bits(bits, bps)

    def symbols_to_bits(self, symbols):
        """Nearest point, index -> MSB-first bits (:90-112); an empty input gives
        the reference's np.array([])."""
        symbols = np.asarray(symbols)
        if symbols.size == 0:
            return np.array([])
        return hard_bits(symbols.ravel(), self._bps).astype(np.int64)

    def get_constellation(self):
        return self.constellation


class OFDMModulator:
    """OFDMModulator (core/modulator.py:119-420): 'simple' (sequential
    mapping), 'lte' (DC / guards / pilots) and 'sc-fdm' (LTE mapping after a
    DFT precoder)."""

    def __init__(self, config, mode='lte', enable_sc_fdm=False):
        self.config = config
        self.mode = 'sc-fdm' if enable_sc_fdm else mode
        self.enable_sc_fdm = enable_sc_fdm or (mode == 'sc-fdm')
        self.qam_modulator = QAMModulator(config.modulation)
        self.resource_mapper = ResourceMapper(config) if self.mode in ('lte', 'sc-fdm') else None
        if self.enable_sc_fdm and self.resource_mapper is not None:
            self.sc_fdm_precoder = SC_FDMPrecodifier(num_data_subcarriers=len(self.resource_mapper.get_data_indices()),
                                                     enable=self.enable_sc_fdm)
        else:
            self.sc_fdm_precoder = None

    def modulate(self, bits):
        qam_symbols = self.qam_modulator.bits_to_symbols(bits)
        if self.mode in ('lte', 'sc-fdm'):
            return self._modulate_lte(qam_symbols)
        return self._modulate_simple(qam_symbols)

    def _modulate_simple(self, qam_symbols):
        """First Nc symbols on subcarriers 0..Nc-1, IFFT, CP (:192-212)."""
        cfg = self.config
        par = np.zeros(cfg.N, dtype=complex)
        n = min(len(qam_symbols), cfg.Nc)
        par[:n] = qam_symbols[:n]
        return ofdm_symbol(par, cfg.cp_length), qam_symbols[:n], None

    def _modulate_lte(self, qam_symbols):
        """Pad / truncate to the data subcarriers, optional DFT precoding, RE
        mapping, IFFT, CP (:214-250)."""
        nd = len(self.resource_mapper.get_data_indices())
        if len(qam_symbols) < nd:
            qam_symbols = np.pad(qam_symbols, (0, nd - len(qam_symbols)), 'constant')
        elif len(qam_symbols) > nd:
            qam_symbols = qam_symbols[:nd]
        pre = (self.sc_fdm_precoder.precoding(qam_symbols) if self.enable_sc_fdm and self.sc_fdm_precoder is not None
               else qam_symbols)
        grid_mapped, mapping_info = self.resource_mapper.map_symbols(pre)
        return ofdm_symbol(grid_mapped, self.config.cp_length), qam_symbols, mapping_info

    def _bits_per_ofdm(self, lte):
        if lte:
            return len(self.resource_mapper.get_data_indices()) * self.config.bits_per_symbol
        return self.config.Nc * self.config.bits_per_symbol

    def modulate_stream(self, bits, num_ofdm_symbols=None):
        """Whole OFDM symbols from a bit stream (:252-302).  LTE / SC-FDM: one
        plan call for the stream (the TX stage the simulators use)."""
        lte = self.mode in ('lte', 'sc-fdm') and self.resource_mapper is not None
        bpo = self._bits_per_ofdm(lte)
        if num_ofdm_symbols is None:
            num_ofdm_symbols = int(np.ceil(len(bits) / bpo))
        total = num_ofdm_symbols * bpo
        bits = np.asarray(bits)
        if len(bits) < total:
            bits = np.pad(bits, (0, total - len(bits)), 'constant')
        if lte and num_ofdm_symbols > 0:
            from .ofdm_core import OFDMTransmitter
            tx = OFDMTransmitter(self.config, mode='lte', enable_sc_fdm=self.enable_sc_fdm)
            return tx.modulate(_bits_u8(bits[:total]).astype(np.int64))
        sig, syms, infos = [], [], ([] if lte else None)
        for i in range(num_ofdm_symbols):
            s, q, info = self.modulate(bits[i * bpo:(i + 1) * bpo])
            sig.append(s)
            syms.append(q)
            if lte:
                infos.append(info)
        return np.concatenate(sig), syms, infos

    def modulate_stream_vectorized(self, bits, num_ofdm_symbols=None):
        """The reference's vectorised variant (:304-403): LTE mapping only in
        mode 'lte' (mode 'sc-fdm' takes the sequential mapping there)."""
        lte = self.mode == 'lte' and self.resource_mapper is not None
        if lte:
            return self.modulate_stream(bits, num_ofdm_symbols)
        bpo = self._bits_per_ofdm(False)
        if num_ofdm_symbols is None:
            num_ofdm_symbols = int(np.ceil(len(bits) / bpo))
        total = num_ofdm_symbols * bpo
        bits = np.asarray(bits)
        if len(bits) < total:
            bits = np.pad(bits, (0, total - len(bits)), 'constant')
        sig, syms = [], []
        for i in range(num_ofdm_symbols):
            q = self.qam_modulator.bits_to_symbols(bits[i * bpo:(i + 1) * bpo])
            s, q2, _ = self._modulate_simple(q)
            sig.append(s)
            syms.append(q2)
        return np.concatenate(sig), syms, None

    def set_sc_fdm_enabled(self, enable: bool):
        self.enable_sc_fdm = enable
        self.mode = 'sc-fdm' if enable else 'lte'
        if self.sc_fdm_precoder is not None:
            self.sc_fdm_precoder.set_enable(enable)

    def get_qam_modulator(self):
        return self.qam_modulator


def qpsk_to_llrs(symbols: np.ndarray, noise_var: float) -> np.ndarray:
    """qpsk_to_llrs (core/modulator.py:423-475): interleaved [I0, Q0, I1, ...]
    = 2 sqrt(2) y / sigma^2 per component, on the GPU (lte_llr_host64, the
    chains' QPSK demapper)."""
    y = np.ascontiguousarray(symbols, dtype=np.complex128).ravel()
    if y.size == 0:
        return np.array([], dtype=np.float64)
    nv = np.ascontiguousarray(np.broadcast_to(np.asarray(noise_var, dtype=np.float64), y.shape))
    out = np.empty(2 * len(y), dtype=np.float64)
    C.device_init()
    C.check(C.load().lte_llr_host64(2, len(y), C.ptr(y.view(np.float64), C.F64), C.ptr(nv, C.F64),
                                    C.ptr(out, C.F64)))
    return out


def qam16_to_llrs(symbols: np.ndarray, noise_var: float) -> np.ndarray:
    """Placeholder in the reference (core/modulator.py:478-500)."""
    raise NotImplementedError("16-QAM LLR generation not yet implemented")


def qam64_to_llrs(symbols: np.ndarray, noise_var: float) -> np.ndarray:
    """Placeholder in the reference (core/modulator.py:503-525)."""
    raise NotImplementedError("64-QAM LLR generation not yet implemented")
