"""Drop-in mirror of the reference's orchestration layer (core/ofdm_core.py).

`OFDMTransmitter`, `OFDMReceiver`, `OFDMChannel` and `OFDMSimulator` keep the
reference's names, constructor arguments, defaults, return values and
result-dict keys; all signal processing runs on the MI355X through
liblte_hip.so (engine.Plan / _capi).

Random numbers: single-call methods reproduce the reference's frozen global
RNG exactly -- the host draws the same NumPy legacy-RNG values the reference
consumes (pilot reseed, Jakes phases, unit normals), leaving the global RNG in
the same final state, and the GPU consumes them ("ref-compat" injection).
`run_grid` is the device-resident Monte-Carlo driver (Philox per frame).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np

from . import _capi as C
from .dist import trial_shard
from .config import ITU_CHANNEL_MODELS, LTEConfig
from .engine import get_plan

SLOT_SIZE = 14


# ------------------------------------------------------------------ building blocks
# the reference's core/resource_mapper.py, core/modulator.py and
# core/demodulator.py classes (lte_phy.resource_mapper / .modulator / .demodulator)
from .resource_mapper import LTEResourceGrid as ResourceGrid, _reseed_pilots  # noqa: E402,F401
from .modulator import OFDMModulator, constellation  # noqa: E402,F401
from .demodulator import OFDMDemodulator  # noqa: E402
from .channel import AWGNChannel, FadingChannel, RayleighMultiPathChannel  # noqa: E402


def _check_mode(mode, enable_sc_fdm):
    """OFDMModulator mode rule (core/modulator.py:128-131): enable_sc_fdm or
    mode 'sc-fdm' -> LTE mapping + DFT precoding.  Returns the SC-FDM flag."""
    sc = bool(enable_sc_fdm) or mode == 'sc-fdm'
    if mode not in ('lte', 'sc-fdm'):
        raise NotImplementedError(f"mode '{mode}' is not on the GPU path (only 'lte' / 'sc-fdm' resource mapping)")
    return sc


def itu_paths(profile, fs, spatial=False):
    """RayleighMultiPathChannel._get_itu_profile_params (core/channel.py:162-186)
    followed by RayleighChannel.__init__'s second dB->linear conversion
    (core/rayleighchannel.py:16) -- quirk Q2 reproduced on purpose."""
    if profile not in ITU_CHANNEL_MODELS:
        raise ValueError(f"Perfil ITU no encontrado: {profile}. "
                         f"Opciones disponibles: {list(ITU_CHANNEL_MODELS.keys())}")
    d = ITU_CHANNEL_MODELS[profile]
    delays_s = np.array(d['delays_us']) * 1e-6
    g = 10 ** (np.array(d['power_db']) / 20)
    g = 10 ** (np.array(g) / 20)
    if spatial:
        g = 10 ** (np.array(g) / 20)
    return [int(np.round(t * fs)) for t in delays_s], [float(x) for x in g]


def doppler(frequency_ghz, velocity_kmh, profile):
    """RayleighMultiPathChannel fD rule (core/channel.py:113-143)."""
    if frequency_ghz is not None and velocity_kmh is not None:
        fc, v = frequency_ghz * 1e9, velocity_kmh / 3.6
    else:
        v = (5.0 if 'Pedestrian' in profile else 30.0 if 'Vehicular_A' in profile else
             120.0 if 'Vehicular_B' in profile else 10.0) / 3.6
        fc = 2e9
    return (v * fc) / 3e8


def papr(signal):
    """OFDMTransmitter.calculate_papr (core/ofdm_core.py:114-147)."""
    p = np.abs(signal) ** 2
    pk, av = np.max(p), np.mean(p)
    if av > 0:
        lin = pk / av
        return {'papr_db': 10 * np.log10(lin), 'papr_linear': lin, 'peak_power': pk, 'avg_power': av}
    return {'papr_db': 0.0, 'papr_linear': 1.0, 'peak_power': pk, 'avg_power': av}


# ------------------------------------------------------------------ TX
class OFDMTransmitter:
    """OFDMTransmitter (core/ofdm_core.py:42-155)."""

    def __init__(self, config: LTEConfig, mode: str = 'lte', enable_sc_fdm: bool = False):
        self.config, self.mode, self.enable_sc_fdm = config, mode, enable_sc_fdm
        self.modulator = OFDMModulator(config, mode=mode, enable_sc_fdm=enable_sc_fdm)
        self.grid = ResourceGrid(config.N, config.Nc)
        self.last_signal_tx = self.last_symbols_tx = self.last_mapping_infos = None

    def _mapping_info(self, n_data):
        g = self.grid
        return {'num_data_mapped': n_data, 'num_pilots_mapped': len(g._pilot),
                'num_nulls': len(g._guard) + 1, 'data_indices': g.get_data_indices()[:n_data],
                'pilot_indices': g.get_pilot_indices(), 'guard_indices': g.get_guard_indices(),
                'dc_index': g.dc_index, 'grid_statistics': g.get_statistics()}

    def modulate(self, bits) -> Tuple[np.ndarray, List[np.ndarray], List[Dict]]:
        """OFDMModulator.modulate_stream (core/modulator.py:252-302) on the GPU:
        an LTE / SC-FDM stream is one plan call (TX stage); mode 'simple'
        goes through the modulator's per-symbol GPU stages."""
        if not isinstance(bits, np.ndarray):
            bits = np.array(bits, dtype=int)
        if bits.size == 0:
            raise ValueError("Bits array cannot be empty")
        if self.modulator.mode not in ('lte', 'sc-fdm'):
            sig, syms, infos = self.modulator.modulate_stream(bits)
            self.last_signal_tx, self.last_symbols_tx, self.last_mapping_infos = sig, syms, infos
            return sig, syms, infos
        cfg = self.config
        Nd = len(self.grid._data)
        n_sym = int(np.ceil(len(bits) / (Nd * cfg.bits_per_symbol)))
        plan = get_plan(N=cfg.N, Nc=cfg.Nc, cp_len=cfg.cp_length, bps=cfg.bits_per_symbol, n_sym=n_sym,
                        chain=C.CHAIN_UNCODED, channel=C.CH_AWGN, n_bits=len(bits), max_frames=1,
                        sc_fdm=int(self.modulator.enable_sc_fdm))
        r = plan.run([np.inf], bits=(np.asarray(bits) & 1).astype(np.uint8)[None], stages=C.STAGE_TX,
                     capture=('signal_tx', 'tx_syms'))
        _reseed_pilots(0, len(self.grid._pilot))
        sig = r['signal_tx'][0].astype(np.complex128)
        ts = r['tx_syms'][0].astype(np.complex128)
        syms = [ts[i * Nd:(i + 1) * Nd] for i in range(n_sym)]
        infos = [self._mapping_info(Nd) for _ in range(n_sym)]
        self.last_signal_tx, self.last_symbols_tx, self.last_mapping_infos = sig, syms, infos
        return sig, syms, infos

    def calculate_papr(self, signal: np.ndarray) -> Dict:
        return papr(signal)

    def get_config(self) -> LTEConfig:
        return self.config

    def __repr__(self):
        return f"OFDMTransmitter({self.config.modulation}, {'SC-FDM' if self.enable_sc_fdm else 'OFDM'})"


# ------------------------------------------------------------------ RX
class OFDMReceiver:
    """OFDMReceiver (core/ofdm_core.py:158-276)."""

    def __init__(self, config: LTEConfig, mode: str = 'lte', enable_equalization: bool = True,
                 enable_sc_fdm: bool = False):
        self._sc = bool(enable_sc_fdm) or mode == 'sc-fdm'
        self.config, self.mode = config, mode
        self.enable_equalization, self.enable_sc_fdm = enable_equalization, enable_sc_fdm
        self.demodulator = OFDMDemodulator(config, mode=mode, enable_equalization=enable_equalization,
                                           enable_sc_fdm=enable_sc_fdm)
        self.grid = ResourceGrid(config.N, config.Nc)
        self.last_symbols_rx = self.last_bits_rx = self.channel_estimate = None

    def demodulate(self, signal_rx: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """OFDMDemodulator.demodulate_stream 'lte' path (core/demodulator.py:120-147):
        CP removal + FFT, slot-0 CRS estimation, ZF, nearest-point bits."""
        if signal_rx.size == 0:
            raise ValueError("Received signal cannot be empty")
        if self.mode != 'lte':   # 'simple' (and the reference's other modes): the demodulator's GPU stages
            syms, bits = self.demodulator.demodulate_stream(signal_rx)
            self.last_symbols_rx, self.last_bits_rx = syms, bits
            return syms, bits
        cfg = self.config
        sl = cfg.N + cfg.cp_length
        n_sym = max(1, len(signal_rx) // sl)
        sig = np.zeros(n_sym * sl, dtype=np.complex128)
        m = min(len(signal_rx), n_sym * sl)
        sig[:m] = signal_rx[:m]
        Nd = len(self.grid._data)
        nb = n_sym * Nd * cfg.bits_per_symbol
        plan = get_plan(N=cfg.N, Nc=cfg.Nc, cp_len=cfg.cp_length, bps=cfg.bits_per_symbol, n_sym=n_sym,
                        chain=C.CHAIN_UNCODED, channel=C.CH_AWGN, n_bits=nb, max_frames=1, sc_fdm=int(self._sc),
                        no_equalization=int(not self.enable_equalization))
        r = plan.run([0.0], stages=C.STAGE_RX, in_signal=sig[None], capture=('data_syms', 'bits_rx'))
        _reseed_pilots(0, len(self.grid._pilot))
        syms = r['data_syms'][0].astype(np.complex128)
        bits = r['bits_rx'][0].astype(np.int64)
        self.last_symbols_rx, self.last_bits_rx = syms, bits
        return syms, bits

    def estimate_channel(self) -> Dict:
        return {'estimated': False, 'method': 'none'}

    def calculate_ber(self, bits_tx: np.ndarray, bits_rx: np.ndarray) -> float:
        n = min(len(bits_tx), len(bits_rx))
        if n == 0:
            return 0.0
        return float(np.sum(bits_tx[:n] != bits_rx[:n]) / n)

    def get_config(self) -> LTEConfig:
        return self.config

    def __repr__(self):
        return f"OFDMReceiver({self.config.modulation}, {'SC-FDM' if self.enable_sc_fdm else 'OFDM'})"


# ------------------------------------------------------------------ channel
def _link_matrix(st, rayleigh):
    """channel_matrix of transmit_mimo (core/ofdm_core.py:476-518) from the
    per-link statistics [rx][tx][mean|x|^2, mean|y|^2, Re, Im mean(y x*)]:
    AWGN h = exp(j tx pi/2); Rayleigh sqrt(P_y / P_x) exp(j angle(mean(y x*)))
    (h = 1 if P_x <= 1e-12)."""
    st = np.asarray(st, dtype=np.float64)
    num_rx, num_tx = st.shape[:2]
    Hm = np.zeros((num_rx, num_tx), dtype=complex)
    for a in range(num_rx):
        for t in range(num_tx):
            if not rayleigh:
                Hm[a, t] = 1.0 + 0j if t == 0 else np.exp(1j * (t * np.pi / 2))
            elif st[a, t, 0] > 1e-12:
                Hm[a, t] = np.sqrt(st[a, t, 1] / st[a, t, 0]) * np.exp(1j * np.angle(st[a, t, 2] + 1j * st[a, t, 3]))
            else:
                Hm[a, t] = 1.0 + 0j
    return Hm


class OFDMChannel:
    """OFDMChannel (core/ofdm_core.py:279-557).  Any channel_type other than
    'rayleigh_mp' is AWGN, as in the reference (:322-332)."""

    def __init__(self, channel_type: str = 'awgn', snr_db: float = 10.0, fs: float = 15.36e6,
                 itu_profile: str = 'Pedestrian_A', frequency_ghz: float = 2.0, velocity_kmh: float = 0,
                 *, precision: Optional[str] = None):
        """precision (not in the reference): arithmetic type of the device channel,
        'f64' (default, LTE_PRECISION when unset) or 'f32'; OFDMSimulator passes its own."""
        self.precision = C.precision_of(precision)
        self.channel_type, self.snr_db, self.fs = channel_type, snr_db, fs
        self.profile, self.frequency_ghz, self.velocity_kmh = itu_profile, frequency_ghz, velocity_kmh
        self.rayleigh = channel_type == 'rayleigh_mp'
        if self.rayleigh:
            if fs is None:
                raise ValueError("Se requiere fs (frecuencia de muestreo) para canal Rayleigh")
            self.delays, self.gains = itu_paths(itu_profile, fs)
            self.fD = doppler(frequency_ghz, velocity_kmh, itu_profile)
        else:
            self.delays, self.gains, self.fD = [], [], 0.0

    def set_snr(self, snr_db: float) -> None:
        self.snr_db = snr_db

    @property
    def kind(self):
        return C.CH_RAYLEIGH if self.rayleigh else C.CH_AWGN

    def draw(self, L, num_rx=1):
        """Consume the global RNG like one ChannelSimulator.transmit per RX
        antenna (rayleighchannel.py:31, channel.py:227-228).  Returns
        phases [num_rx][P][16], unit normals [num_rx][2][L]."""
        P = len(self.delays)
        ph = np.zeros((num_rx, P, 16))
        z = np.zeros((num_rx, 2, L))
        for r in range(num_rx):
            for p in range(P):
                ph[r, p] = 2 * np.pi * np.random.rand(16)
            z[r, 0] = np.random.normal(0, 1.0, L)
            z[r, 1] = np.random.normal(0, 1.0, L)
        return ph, z

    def _apply(self, signal, num_rx):
        """Channel on an arbitrary stream on the GPU (lte_channel_host64; float32
        lte_channel_host in an f32 channel)."""
        C.device_init()
        f64 = self.precision == 'f64'
        cdt, rdt, ct = (np.complex128, np.float64, C.F64) if f64 else (np.complex64, np.float32, C.F32)
        x = np.ascontiguousarray(signal, dtype=cdt)
        L = len(x)
        ph, z = self.draw(L, num_rx)
        y = np.zeros((num_rx, L), dtype=cdt)
        npow = np.zeros(num_rx, dtype=rdt)
        P = len(self.delays)
        dl = np.array(self.delays, dtype=np.int32)
        g = np.array(self.gains, dtype=np.float64)
        fn = C.load().lte_channel_host64 if f64 else C.load().lte_channel_host
        C.check(fn(L, num_rx, self.kind, P, C.ptr(dl, C.I32) if P else None,
                   C.ptr(g, C.F64) if P else None, float(self.fD), float(self.fs or 0.0),
                   float(self.snr_db), 0, C.ptr(x.view(rdt), ct),
                   C.ptr(ph, C.F64) if P else None, C.ptr(z, C.F64),
                   C.ptr(y.view(rdt), ct), C.ptr(npow, ct)))
        return y.astype(np.complex128)

    def transmit(self, signal: np.ndarray) -> np.ndarray:
        """ChannelSimulator.transmit (core/channel.py:334-345)."""
        return self._apply(signal, 1)[0]

    def transmit_simo(self, signal_tx: np.ndarray, num_rx: int = 2) -> List[np.ndarray]:
        """Independent fading + noise per RX antenna (core/ofdm_core.py:361-412)."""
        if num_rx < 1:
            raise ValueError("num_rx must be >= 1")
        return list(self._apply(signal_tx, num_rx))

    def transmit_mimo(self, signals_tx, num_rx: int = 1):
        """OFDMChannel.transmit_mimo (core/ofdm_core.py:434-543) on the device
        (lte_channel_mimo_host).  AWGN links h = exp(j tx pi/2); Rayleigh links
        are each a 100 dB ChannelSimulator (fading + link noise); RX noise
        (P_rx / num_tx) / SNR.  The global RNG is consumed in the reference's
        order (per RX: per TX link [16 phases per path, link noise re, im],
        then the RX noise).  Returns (signals_rx list, channel_matrix
        [num_rx][num_tx]), the matrix by the reference's power-ratio /
        correlation-phase rule."""
        num_tx = len(signals_tx)
        if num_tx == 0:
            raise ValueError("No transmitted signals provided")
        L = len(signals_tx[0])
        for t, sg in enumerate(signals_tx):
            if len(sg) != L:
                raise ValueError(f"TX signal {t} length mismatch")
        C.device_init()
        f64 = self.precision == 'f64'
        cdt, rdt, ct = (np.complex128, np.float64, C.F64) if f64 else (np.complex64, np.float32, C.F32)
        x = np.ascontiguousarray(np.stack([np.asarray(sg) for sg in signals_tx]), dtype=cdt)
        P = len(self.delays)
        ph = np.zeros((num_rx, num_tx, max(P, 1), 16))
        lz = np.zeros((num_rx, num_tx, 2, L))
        z = np.zeros((num_rx, 2, L))
        for r in range(num_rx):
            for t in range(num_tx):
                if self.rayleigh:
                    for p in range(P):
                        ph[r, t, p] = 2 * np.pi * np.random.rand(16)
                    lz[r, t, 0] = np.random.normal(0, 1.0, L)
                    lz[r, t, 1] = np.random.normal(0, 1.0, L)
            z[r, 0] = np.random.normal(0, 1.0, L)
            z[r, 1] = np.random.normal(0, 1.0, L)
        y = np.zeros((num_rx, L), dtype=cdt)
        st = np.zeros((num_rx, num_tx, 4), dtype=rdt)
        dl = np.array(self.delays, dtype=np.int32)
        g = np.array(self.gains, dtype=np.float64)
        ray = self.rayleigh
        fn = C.load().lte_channel_mimo_host64 if f64 else C.load().lte_channel_mimo_host
        C.check(fn(
            L, num_tx, num_rx, 0, self.kind, P, C.ptr(dl, C.I32) if P else None, C.ptr(g, C.F64) if P else None,
            float(self.fD), float(self.fs or 0.0), float(self.snr_db), 0, C.ptr(x.view(rdt), ct),
            C.ptr(ph, C.F64) if ray else None, C.ptr(lz, C.F64) if ray else None, None, C.ptr(z, C.F64),
            C.ptr(y.view(rdt), ct), C.ptr(st, ct) if ray else None, None))
        return list(y.astype(np.complex128)), _link_matrix(st, ray)

    def get_config(self) -> Dict:
        return {'type': self.channel_type, 'snr_db': self.snr_db, 'fs': self.fs, 'profile': self.profile,
                'frequency_ghz': self.frequency_ghz, 'velocity_kmh': self.velocity_kmh}

    def __repr__(self):
        return f"OFDMChannel({self.channel_type}, SNR={self.snr_db}dB, {self.profile})"



class ChannelSimulator:
    """ChannelSimulator (core/channel.py:294-493) holding an AWGNChannel,
    FadingChannel or RayleighMultiPathChannel (lte_phy.channel) as
    `channel`.  The fD rule and gain conversions are the reference's
    (doppler(), Q2)."""

    def __init__(self, channel_type='awgn', snr_db=10.0, fs=None, itu_profile='Vehicular_A', frequency_ghz=None,
                 velocity_kmh=None, verbose=True, *, precision: Optional[str] = None):
        self.channel_type, self.fs, self.itu_profile = channel_type, fs, itu_profile
        self.frequency_ghz, self.velocity_kmh = frequency_ghz, velocity_kmh
        self.precision = C.precision_of(precision)
        if channel_type == 'awgn':
            self.channel = AWGNChannel(snr_db, precision=self.precision)
        elif channel_type == 'fading':
            self.channel = FadingChannel(snr_db, precision=self.precision)
        elif channel_type == 'rayleigh_mp':
            if fs is None:
                raise ValueError("Se requiere fs (frecuencia de muestreo) para canal Rayleigh")
            self.channel = RayleighMultiPathChannel(snr_db, fs, itu_profile, frequency_ghz=frequency_ghz,
                                                    velocity_kmh=velocity_kmh, verbose=verbose,
                                                    precision=self.precision)
        else:
            raise ValueError(f"Tipo de canal desconocido: {channel_type}")

    @property
    def snr_db(self):
        return self.channel.snr_db

    def set_snr(self, snr_db):
        self.channel.set_snr(snr_db)

    def transmit(self, signal):
        """core/channel.py:334-345."""
        received, _ = self.channel.transmit(signal)
        return received

    def set_channel_type(self, channel_type, **kwargs):
        """core/channel.py:351-373."""
        self.channel_type = channel_type
        snr = self.channel.snr_db if hasattr(self.channel, 'snr_db') else 10.0
        if channel_type == 'awgn':
            self.channel = AWGNChannel(snr, precision=self.precision)
        elif channel_type == 'fading':
            self.channel = FadingChannel(snr, precision=self.precision)
        elif channel_type == 'rayleigh_mp':
            if self.fs is None:
                raise ValueError("Se requiere fs para cambiar a canal Rayleigh")
            self.itu_profile = kwargs.get('itu_profile', self.itu_profile)
            self.channel = RayleighMultiPathChannel(snr, self.fs, self.itu_profile, precision=self.precision)
        else:
            raise ValueError(f"Tipo de canal desconocido: {channel_type}")

    def set_itu_profile(self, itu_profile):
        if isinstance(self.channel, RayleighMultiPathChannel):
            self.channel.set_profile(itu_profile)
            self.itu_profile = itu_profile
        else:
            raise ValueError("Solo se puede cambiar perfil ITU en canal Rayleigh")

    def get_channel(self):
        return self.channel

    def get_channel_info(self):
        if hasattr(self.channel, 'get_channel_info'):
            return self.channel.get_channel_info()
        return {'type': self.channel_type, 'SNR_dB': self.channel.snr_db if hasattr(self.channel, 'snr_db') else None}

    def transmit_spatial_multiplexing(self, tx_signals, num_rx=2):
        """core/channel.py:397-493 on the device (lte_channel_mimo_host mode 1).
        Streams are cut to the shortest.  rayleigh_mp: each link an independent
        RayleighChannel with the gains converted a third time (Q2) and this
        simulator's fD; H[rx, tx] = first tap of the link's impulse_response
        (its own 16 phases per path, drawn after the filter's).  awgn: h ~
        CN(0, 1) per link.  Noise per RX: P_rx / SNR.  Global RNG consumed in the
        reference's order."""
        num_tx = len(tx_signals)
        L = min(len(sg) for sg in tx_signals)
        if self.channel_type == 'fading':
            raise NotImplementedError("transmit_spatial_multiplexing on 'fading' links is outside the GPU path")
        ray = self.channel_type == 'rayleigh_mp'
        snr_db = self.channel.snr_db
        fD = self.channel.rayleigh.fD if ray else 0.0
        kind = C.CH_RAYLEIGH if ray else C.CH_AWGN
        C.device_init()
        f64 = self.precision == 'f64'
        cdt, rdt, ct = (np.complex128, np.float64, C.F64) if f64 else (np.complex64, np.float32, C.F32)
        x = np.ascontiguousarray(np.stack([np.asarray(sg)[:L] for sg in tx_signals]), dtype=cdt)
        if ray:
            delays, gains = itu_paths(self.itu_profile, self.fs, spatial=True)
        else:
            delays, gains = [], []
        P = len(delays)
        ph = np.zeros((num_rx, num_tx, max(P, 1), 16))
        lh = np.zeros((num_rx, num_tx, 2))
        Hm = np.zeros((num_rx, num_tx), dtype=complex)
        for r in range(num_rx):
            for t in range(num_tx):
                if ray:
                    for p in range(P):
                        ph[r, t, p] = 2 * np.pi * np.random.rand(16)
                    ir0 = 2 * np.pi * np.random.rand(16)     # impulse_response(N=1): path 0 is the tap kept
                    for _ in range(1, P):
                        np.random.rand(16)
                    Hm[r, t] = gains[0] * np.sqrt(2 / 16) * np.sum(np.exp(1j * ir0))
                else:
                    lh[r, t, 0] = np.random.normal(0, 1 / np.sqrt(2))
                    lh[r, t, 1] = np.random.normal(0, 1 / np.sqrt(2))
                    Hm[r, t] = lh[r, t, 0] + 1j * lh[r, t, 1]
        z = np.zeros((num_rx, 2, L))
        for r in range(num_rx):
            z[r, 0] = np.random.normal(0, 1.0, L)
            z[r, 1] = np.random.normal(0, 1.0, L)
        y = np.zeros((num_rx, L), dtype=cdt)
        dl = np.array(delays, dtype=np.int32)
        g = np.array(gains, dtype=np.float64)
        fn = C.load().lte_channel_mimo_host64 if f64 else C.load().lte_channel_mimo_host
        C.check(fn(
            L, num_tx, num_rx, 1, kind, P, C.ptr(dl, C.I32) if P else None, C.ptr(g, C.F64) if P else None,
            float(fD), float(self.fs or 0.0), float(snr_db), 0, C.ptr(x.view(rdt), ct),
            C.ptr(ph, C.F64) if ray else None, None, None if ray else C.ptr(lh, C.F64), C.ptr(z, C.F64),
            C.ptr(y.view(rdt), ct), None, None))
        return list(y.astype(np.complex128)), Hm


# ------------------------------------------------------------------ simulator
class OFDMSimulator:
    """OFDMSimulator (core/ofdm_core.py:560-2486): SISO, SISO+turbo and SIMO-MRC
    on the GPU, plus the device-resident Monte-Carlo grid `run_grid`."""

    def __init__(self, config: Optional[LTEConfig] = None, channel_type: str = 'awgn', mode: str = 'lte',
                 enable_sc_fdm: bool = False, enable_equalization: bool = True, num_channels: int = 1,
                 itu_profile: str = 'Pedestrian_A', frequency_ghz: float = 2.0, velocity_kmh: float = 0.0,
                 *, precision: Optional[str] = None):
        """precision (not in the reference): arithmetic type of the GPU chains
        (SISO, SIMO, SFBC, spatial multiplexing, beamforming) and of this
        simulator's channels, 'f64' (default; the reference's float64) or
        'f32' (fast mode)."""
        if config is None:
            config = LTEConfig()
        _check_mode(mode, enable_sc_fdm)   # the simulator chains map REs the LTE way
        self.precision = C.precision_of(precision)
        self.config, self.channel_type, self.mode = config, channel_type, mode
        self.enable_sc_fdm, self.enable_equalization = enable_sc_fdm, enable_equalization
        self.itu_profile, self.frequency_ghz, self.velocity_kmh = itu_profile, frequency_ghz, velocity_kmh
        self.tx = OFDMTransmitter(config, mode=mode, enable_sc_fdm=enable_sc_fdm)
        self.rx = OFDMReceiver(config, mode=mode, enable_equalization=enable_equalization,
                               enable_sc_fdm=enable_sc_fdm)
        fs = getattr(config, 'fs', 15.36e6)
        self.channels = []
        for _ in range(num_channels):
            if channel_type == 'rayleigh_mp':
                ch = OFDMChannel('rayleigh_mp', 10.0, fs, itu_profile, frequency_ghz, velocity_kmh,
                                 precision=self.precision)
            else:
                ch = OFDMChannel('awgn', snr_db=10.0, fs=fs, precision=self.precision)
            self.channels.append(ch)
        self.grid = ResourceGrid(config.N, config.Nc)
        self.last_results = None

    # -------------------------------------------------------------- helpers
    @property
    def Nd(self):
        return len(self.grid._data)

    def _plan(self, chain, n_sym, n_bits, num_rx=1, max_frames=1, iters=8):
        """SC-FDM (enable_sc_fdm / mode 'sc-fdm') reaches the uncoded SISO / SIMO
        transmitters and the SISO receiver; simulate_siso_coded ignores it, as
        the reference does (lte_plan_desc.sc_fdm, include/lte_phy.h)."""
        cfg, ch = self.config, self.channels[0]
        sc = int(self.tx.modulator.enable_sc_fdm and chain in (C.CHAIN_UNCODED, C.CHAIN_SIMO))
        # enable_equalization reaches simulate_siso's receiver only (the coded and SIMO
        # drivers build their own LTEReceivers, core/ofdm_core.py:1117-1122, 1369-1373)
        noeq = int(not self.enable_equalization and chain == C.CHAIN_UNCODED)
        return get_plan(N=cfg.N, Nc=cfg.Nc, cp_len=cfg.cp_length, bps=cfg.bits_per_symbol, n_sym=n_sym,
                        chain=chain, channel=ch.kind, num_rx=num_rx, delays=tuple(ch.delays),
                        gains=tuple(ch.gains), fD=ch.fD, fs=cfg.fs, n_bits=n_bits, turbo_iters=iters,
                        max_frames=max_frames, sc_fdm=sc, no_equalization=noeq, precision=self.precision)

    def _ref_draws(self, L, num_rx=1):
        """Exactly the global-RNG consumption of one reference simulate_* call:
        TX pilot reseed -> per antenna channel draws -> RX pilot reseed (Q1)."""
        np_ = len(self.grid._pilot)
        _reseed_pilots(0, np_)
        ph, z = self.channels[0].draw(L, num_rx)
        _reseed_pilots(0, np_)
        return ph, z

    @staticmethod
    def _bits_in(bits):
        if not isinstance(bits, np.ndarray):
            bits = np.array(bits, dtype=int)
        if bits.size == 0:
            raise ValueError("Bits array cannot be empty")
        return bits

    # -------------------------------------------------------------- SISO
    def simulate_siso(self, bits: np.ndarray, snr_db: float = 10.0) -> Dict:
        """core/ofdm_core.py:660-737"""
        bits = self._bits_in(bits)
        n0 = len(bits)
        n_sym = int(np.ceil(n0 / (self.Nd * self.config.bits_per_symbol)))
        plan = self._plan(C.CHAIN_UNCODED, n_sym, n0)
        ph, z = self._ref_draws(plan.L)
        r = plan.run([snr_db], bits=(bits & 1).astype(np.uint8)[None], phases=ph[None] if ph.size else None,
                     noise=z[None], capture=('signal_tx', 'signal_rx', 'data_syms', 'bits_rx', 'tx_syms'))
        brx = r['bits_rx'][0].astype(np.int64)
        err = int(np.sum(bits != brx))
        sig_tx = r['signal_tx'][0].astype(np.complex128)
        pa = papr(sig_tx)
        ts = r['tx_syms'][0].astype(np.complex128)
        res = {'transmitted_bits': int(n0), 'received_bits': int(n0), 'bits_received_array': brx,
               'bit_errors': err, 'errors': err, 'ber': float(err / n0), 'snr_db': float(snr_db),
               'papr_db': float(pa['papr_db']), 'papr_linear': float(pa['papr_linear']), 'signal_tx': sig_tx,
               'signal_rx': r['signal_rx'][0, 0].astype(np.complex128),
               'symbols_tx': [ts[i * self.Nd:(i + 1) * self.Nd] for i in range(n_sym)],
               'symbols_rx': r['data_syms'][0].astype(np.complex128)}
        self.tx.last_signal_tx = sig_tx
        self.rx.last_symbols_rx, self.rx.last_bits_rx = res['symbols_rx'], brx
        self.last_results = res
        return res

    def calculate_noise_var_zf(self, H_estimate: np.ndarray, snr_db: float) -> float:
        """core/ofdm_core.py:739-789 (harmonic-mean |H|^2)."""
        s2 = 1.0 / (10 ** (snr_db / 10))
        if H_estimate.size == 0:
            return s2
        hp = np.maximum(np.abs(np.atleast_1d(H_estimate)) ** 2, 1e-12)
        if len(hp) == 1:
            return s2 / hp[0]
        return s2 / (len(hp) / np.sum(1.0 / hp))

    # -------------------------------------------------------------- SISO + turbo
    def simulate_siso_coded(self, bits: np.ndarray, snr_db: float = 10.0) -> Dict:
        """core/ofdm_core.py:925-1338: CRC-24A -> segmentation -> turbo (rate 1/3)
        -> rate matching -> QAM -> T/F interleave -> OFDM -> channel -> ZF ->
        max-log LLRs -> dematch -> turbo max-log-MAP (8 it.) -> CRC."""
        bits = self._bits_in(bits)
        n0 = len(bits)
        plan = self._plan(C.CHAIN_CODED, 0, n0, iters=8)
        ph, z = self._ref_draws(plan.L)
        r = plan.run([snr_db], bits=(bits & 1).astype(np.uint8)[None], phases=ph[None] if ph.size else None,
                     noise=z[None], capture=('signal_tx', 'signal_rx', 'data_syms', 'bits_rx', 'tx_syms',
                                             'H', 'pilot_stats'))
        cfg = self.config
        bps, Nd = cfg.bits_per_symbol, self.Nd
        coded = plan.coded_bits
        dec = r['bits_rx'][0].astype(np.uint8)
        err = int(np.sum(bits != dec))
        sig_tx = r['signal_tx'][0].astype(np.complex128)
        pa = papr(sig_tx)
        # T/F de-interleave of the captured TX / RX REs (core/ofdm_core.py:1040-1060, 1174-1207)
        ncs_tx = -(-coded // bps)
        rows = -(-ncs_tx // Nd)
        q = np.arange(ncs_tx)
        qam = r['tx_syms'][0].astype(np.complex128)[(q % Nd) * rows + q // Nd]
        ncs = coded // bps
        rows_rx = -(-ncs // Nd)
        q = np.arange(ncs)
        src = (q % Nd) * rows_rx + q // Nd
        sy = r['data_syms'][0].astype(np.complex128)
        Hs = r['H'][0, 0].astype(np.complex128)                        # [n_grp][N]
        Hd = np.concatenate([Hs[l // SLOT_SIZE][self.grid._data] for l in range(plan.n_sym)])
        sd, hd = sy[src], Hd[src]
        s2 = 1.0 / (10 ** (snr_db / 10))
        if self.channels[0].channel_type == 'awgn':
            nv = np.full(len(sd), s2)
        else:
            nv = np.maximum(s2 / np.clip(np.abs(hd) ** 2, 1e-6, 1e6), s2 / 4.0)
        st = r['pilot_stats'][0, 0].astype(np.float64)
        ch_snr = float(np.mean(10 * np.log10(st[:, 0] / (st[:, 1] + 1e-10) + 1e-10)))
        res = {'transmitted_bits': int(n0), 'received_bits': int(n0), 'bits_received_array': dec,
               'bit_errors': err, 'ber': float(err / n0), 'crc_pass': bool(r['crc_ok'][0]),
               'snr_db': float(snr_db), 'papr_db': float(pa['papr_db']), 'papr_linear': float(pa['papr_linear']),
               'coded_bits_length': int(coded), 'signal_tx': sig_tx,
               'signal_rx': r['signal_rx'][0, 0].astype(np.complex128), 'symbols_tx': qam, 'symbols_rx': sd,
               'H_estimate': hd, 'channel_snr_db': ch_snr, 'noise_var_mean': float(np.mean(nv))}
        self.last_results = res
        return res

    # -------------------------------------------------------------- SIMO
    def simulate_simo(self, bits: np.ndarray, snr_db: float = 10.0, num_rx: int = 2, combining: str = 'mrc',
                      parallel: bool = True) -> Dict:
        """core/ofdm_core.py:1536-1679: independent channel per RX antenna, CRS
        estimation per antenna, MRC sum(conj(H_i) Y_i)/(sum|H_i|^2 + 1e-10)."""
        bits = self._bits_in(bits)
        if num_rx < 1:
            raise ValueError("num_rx must be >= 1")
        n0 = len(bits)
        n_sym = int(np.ceil(n0 / (self.Nd * self.config.bits_per_symbol)))
        plan = self._plan(C.CHAIN_SIMO, n_sym, n0, num_rx=num_rx)
        ph, z = self._ref_draws(plan.L, num_rx)
        r = plan.run([snr_db], bits=(bits & 1).astype(np.uint8)[None], phases=ph[None] if ph.size else None,
                     noise=z[None], capture=('signal_tx', 'signal_rx', 'data_syms', 'bits_rx', 'tx_syms', 'H'))
        brx = r['bits_rx'][0].astype(np.int64)
        err = int(np.sum(bits != brx))
        sig_tx = r['signal_tx'][0].astype(np.complex128)
        pa = papr(sig_tx)
        ts = r['tx_syms'][0].astype(np.complex128)
        H = r['H'][0].astype(np.complex128)
        res = {'transmitted_bits': int(n0), 'received_bits': int(n0), 'bits_received_array': brx,
               'bit_errors': err, 'errors': err, 'ber': float(err / n0), 'snr_db': float(snr_db),
               'papr_db': float(pa['papr_db']), 'papr_linear': float(pa['papr_linear']), 'signal_tx': sig_tx,
               'signal_rx_list': [r['signal_rx'][0, i].astype(np.complex128) for i in range(num_rx)],
               'symbols_tx': [ts[i * self.Nd:(i + 1) * self.Nd] for i in range(n_sym)],
               'symbols_rx_combined': r['data_syms'][0].astype(np.complex128),
               'symbols_rx_list': None,
               'channel_estimates_per_antenna': [[H[a, l // SLOT_SIZE] for l in range(n_sym)]
                                                 for a in range(num_rx)],
               'num_rx': num_rx, 'combining_method': combining, 'diversity_level': num_rx,
               'parallel_processing': parallel}
        self.last_results = res
        return res

    # -------------------------------------------------------------- SFBC (config 4)
    def _sfbc_plan(self, n_sym, n_bits, num_rx, coded=False, max_frames=1, iters=8):
        cfg, ch = self.config, self.channels[0]
        return get_plan(N=cfg.N, Nc=cfg.Nc, cp_len=cfg.cp_length, bps=cfg.bits_per_symbol, n_sym=n_sym,
                        chain=C.CHAIN_SFBC_CODED if coded else C.CHAIN_SFBC, channel=ch.kind, num_rx=num_rx,
                        num_tx=2, delays=tuple(ch.delays), gains=tuple(ch.gains), fD=ch.fD, fs=cfg.fs,
                        n_bits=n_bits, turbo_iters=iters, max_frames=max_frames, precision=self.precision)

    def _simulate_sfbc(self, bits, snr_db, num_rx, mode):
        """simulate_miso (core/ofdm_core.py:1850-2047) / simulate_mimo (:2049-2258)
        with the documented estimator fix (H0 = H[0,0,:],
        H1 = H[0,1,:] of MIMOChannelEstimatorPeriodic.estimate_channel_from_grid;
        the reference itself raises at core/mimo_channel_estimator_periodic.py:219).
        One GPU call; the global RNG is consumed exactly as the reference would:
        TX pilot reseeds (cells 0, 1 per OFDM symbol, core/sfbc_alamouti.py:248-256)
        -> transmit_mimo (per RX, per TX link: 16 phases per path + the link's
        100 dB noise; then the RX noise, core/ofdm_core.py:468-541) -> RX pilot
        reseeds (per RX per slot)."""
        bits = self._bits_in(bits)
        if num_rx < 1:
            raise ValueError("num_rx must be >= 1")
        n0 = len(bits)
        cfg, ch = self.config, self.channels[0]
        res = self.Nd & ~1
        n_sym = int(np.ceil(n0 / (res * cfg.bits_per_symbol)))
        plan = self._sfbc_plan(n_sym, n0, num_rx)
        L = plan.L
        pil = self.grid._pilot
        p0, p1 = len(pil[0::2]), len(pil[1::2])
        _reseed_pilots(0, p0)
        _reseed_pilots(1, p1)
        ray = ch.kind == C.CH_RAYLEIGH
        P = len(ch.delays)
        ph = np.zeros((num_rx, 2, max(P, 1), 16))
        lz = np.zeros((num_rx, 2, 2, L))
        z = np.zeros((num_rx, 2, L))
        for r in range(num_rx):
            for t in range(2):
                if ray:
                    for p in range(P):
                        ph[r, t, p] = 2 * np.pi * np.random.rand(16)
                    lz[r, t, 0] = np.random.normal(0, 1.0, L)
                    lz[r, t, 1] = np.random.normal(0, 1.0, L)
            z[r, 0] = np.random.normal(0, 1.0, L)
            z[r, 1] = np.random.normal(0, 1.0, L)
        _reseed_pilots(0, p0)
        _reseed_pilots(1, p1)
        r = plan.run([snr_db], bits=(bits & 1).astype(np.uint8)[None], phases=ph[None] if ray else None,
                     noise=z[None], link_noise=lz[None] if ray else None,
                     capture=('signal_tx', 'bits_rx', 'data_syms', 'link_stats'))
        brx = r['bits_rx'][0].astype(np.int64)
        err = int(np.sum(bits != brx))
        Hm = _link_matrix(r['link_stats'][0], ray)
        sig = r['signal_tx'][0].astype(np.complex128)
        sl = cfg.N + cfg.cp_length
        pap = []
        for t in range(2):
            syms = sig[t, :n_sym * sl].reshape(n_sym, sl)
            pw_ = np.abs(syms) ** 2
            pap.append(float(np.mean(10 * np.log10(np.max(pw_, axis=1) / np.mean(pw_, axis=1)))))
        res_d = {'transmitted_bits': int(n0), 'received_bits': int(n0), 'bits_received_array': brx,
                 'bit_errors': err, 'errors': err, 'ber': float(err / n0), 'snr_db': float(snr_db),
                 'num_tx': 2, 'num_rx': num_rx, 'mode': mode, 'diversity_order': 2 * num_rx,
                 'channel_matrix': Hm, 'papr_db_tx0': pap[0], 'papr_db_tx1': pap[1],
                 'papr_db': float(np.mean([pap[0], pap[1]])),
                 'papr_linear': 10 ** (np.mean([pap[0], pap[1]]) / 10),
                 'symbols_rx': r['data_syms'][0].astype(np.complex128)}
        self.last_results = res_d
        return res_d

    def simulate_miso(self, bits: np.ndarray, snr_db: float = 10.0) -> Dict:
        """core/ofdm_core.py:1850-2047: 2 TX SFBC Alamouti, 1 RX (see _simulate_sfbc)."""
        return self._simulate_sfbc(bits, snr_db, 1, 'MISO-SFBC')

    def simulate_mimo(self, bits: np.ndarray, snr_db: float = 10.0, num_rx: int = 2) -> Dict:
        """core/ofdm_core.py:2049-2258: 2 TX SFBC, num_rx RX, decodes averaged over RX."""
        return self._simulate_sfbc(bits, snr_db, num_rx, 'MIMO-SFBC')

    # -------------------------------------------------------------- sweeps
    def get_config(self) -> LTEConfig:
        """OFDMSimulator.get_config (core/ofdm_core.py:2479-2481)."""
        return self.config

    def __repr__(self) -> str:
        return (f"OFDMSimulator({self.config.modulation}, {'SC-FDM' if self.enable_sc_fdm else 'OFDM'}, "
                f"{self.channel_type}, {len(self.channels)}ch)")

    def run_ber_sweep(self, num_bits: int, snr_range, num_trials: int = 1,
                      progress_callback: Optional[callable] = None) -> Dict:
        """core/ofdm_core.py:1795-1846.  Bits are drawn once from the global RNG;
        every trial reuses the reference's frozen channel/noise draws, so the
        whole (SNR x trial) grid runs as ONE batched GPU call."""
        bits = np.random.randint(0, 2, num_bits)
        snrs = np.atleast_1d(snr_range)
        S, T = len(snrs), int(num_trials)
        if S * T == 0:
            return {'snr_db': snrs, 'ber_mean': np.array([]), 'ber_values': np.array([]),
                    'papr_values': np.array([])}
        n_sym = int(np.ceil(num_bits / (self.Nd * self.config.bits_per_symbol)))
        plan = self._plan(C.CHAIN_UNCODED, n_sym, num_bits, max_frames=S * T)
        ph, z = self._ref_draws(plan.L)
        snr_f = np.repeat(snrs.astype(np.float64), T)
        sidx = np.repeat(np.arange(S), T)
        r = plan.run(snr_f, snr_index=sidx, n_snr=S, bits=(bits & 1).astype(np.uint8)[None],
                     bits_broadcast=True, phases=ph[None] if ph.size else None, phases_broadcast=True,
                     noise=z[None], noise_broadcast=True, capture=('signal_tx',))
        pa = float(papr(r['signal_tx'][0].astype(np.complex128))['papr_db'])
        fe = r['frame_errors'].reshape(S, T)
        # same reduction as the reference: np.mean over the per-trial python floats
        ber = np.array([np.mean([float(int(e) / num_bits) for e in fe[i]]) for i in range(S)])
        papr_v = np.array([np.mean([pa] * T) for _ in range(S)])
        done = 0
        for si, snr in enumerate(snrs):
            for t in range(T):
                done += 1
                if progress_callback:
                    progress_callback(int(done / (S * T) * 100), f"SNR: {snr:.1f} dB - Trial {t+1}/{T}")
        return {'snr_db': snrs, 'ber_mean': ber, 'ber_values': ber.copy(), 'papr_values': papr_v}

    def simulate_beamforming(self, bits: np.ndarray, snr_db: float = 10.0, num_tx: int = 2, num_rx: int = 1,
                             codebook_type: str = 'TM6', velocity_kmh: float = 3.0,
                             update_mode: str = 'adaptive') -> Dict:
        """core/ofdm_core.py:2260-2477 (frequency-domain TM6 beamforming with
        CSI feedback; lte_phy/beamforming.py, LTE_CHAIN_BEAMFORMING)."""
        from .beamforming import simulate_beamforming
        return simulate_beamforming(self, self._bits_in(bits), snr_db, num_tx, num_rx, codebook_type, velocity_kmh,
                                    update_mode)

    def run_grid(self, snr_range, num_trials: int, seed: int = 0, coded: bool = False, num_rx: int = 1,
                 n_bits: Optional[int] = None, frames_per_call: int = 4096, rank: int = 0, world_size: int = 1,
                 turbo_iters: int = 8, mimo: Optional[str] = None, velocity_kmh: float = 3,
                 frequency_ghz: float = 2.0, spatial: Optional[Dict] = None,
                 beamforming: Optional[Dict] = None) -> Dict:
        """Device-resident Monte-Carlo BER/BLER grid (SNR x trials).  Frame
        (s, t) has global id s*num_trials + t; all randomness is Philox keyed by
        (seed, id), so results are identical for any sharding.  With
        world_size > 1 this process handles trials t = rank, rank+W, ... and
        the caller all-reduces the returned `counts`.

        mimo=None: SISO (coded: config 2) / SIMO MRC (num_rx > 1: config 3);
        mimo='sfbc': 2 x num_rx Alamouti (coded: config 4);
        mimo='spatial': TM4 (config 5 = 4x4 rank-4 PMI-0 MMSE; the spatial channel of
        simulate_spatial_multiplexing: gains converted once more, fD from
        velocity_kmh / frequency_ghz).  `spatial` overrides any of
        {'num_tx': 4, 'num_rx': 4, 'rank': 4, 'detector': 'MMSE', 'pmi': 0}.
        mimo='beamforming': simulate_beamforming's frequency-domain chain, H ~
        CN(0, 1) per frame; `beamforming` overrides {'num_tx': 4, 'num_rx': 1,
        'update_mode': 'adaptive'}."""
        snrs = np.atleast_1d(np.asarray(snr_range, dtype=np.float64))
        S, T = len(snrs), int(num_trials)
        cfg = self.config
        if mimo == 'sfbc':
            res = self.Nd & ~1
            if coded:
                nb = int(n_bits or 27760)
                plan = self._sfbc_plan(0, nb, num_rx, coded=True, max_frames=frames_per_call, iters=turbo_iters)
            else:
                nb = int(n_bits or SLOT_SIZE * res * cfg.bits_per_symbol)
                plan = self._sfbc_plan(int(np.ceil(nb / (res * cfg.bits_per_symbol))), nb, num_rx,
                                       max_frames=frames_per_call)
        elif mimo == 'spatial':
            if coded:
                raise NotImplementedError("config 5 is uncoded MMSE detection")
            nb = int(n_bits or SLOT_SIZE * self.Nd * cfg.bits_per_symbol)
            ch = self.channels[0]
            ctype = 'rayleigh_mp' if ch.kind == C.CH_RAYLEIGH else 'awgn'
            from .tm4 import DETECTORS, LTECodebook
            sp = {'num_tx': 4, 'num_rx': 4, 'rank': 4, 'detector': 'MMSE', 'pmi': 0}
            sp.update(spatial or {})
            W = LTECodebook(sp['num_tx'], transmission_mode='TM4', rank=sp['rank']).get_precoder(sp['pmi'])
            plan = _spatial_plan(cfg, ctype, ch.profile, velocity_kmh, frequency_ghz,
                                 int(np.ceil(nb / (self.Nd * cfg.bits_per_symbol))), nb, frames_per_call,
                                 num_tx=sp['num_tx'], num_rx=sp['num_rx'], rank=sp['rank'],
                                 detector=DETECTORS[sp['detector'].upper()], W=W, precision=self.precision)[0]
        elif mimo == 'beamforming':
            from .beamforming import bf_plan
            bfo = {'num_tx': 4, 'num_rx': 1, 'update_mode': 'adaptive'}
            bfo.update(beamforming or {})
            nb = int(n_bits or SLOT_SIZE * self.Nd * cfg.bits_per_symbol)
            plan = bf_plan(cfg, int(np.ceil(nb / (self.Nd * cfg.bits_per_symbol))), nb, bfo['num_tx'],
                           bfo['num_rx'], bfo['update_mode'] == 'adaptive', frames_per_call, precision=self.precision)
        elif mimo is not None:
            raise ValueError(f"unknown mimo mode {mimo!r}")
        elif coded:
            nb = int(n_bits or 27760)
            plan = self._plan(C.CHAIN_CODED, 0, nb, max_frames=frames_per_call, iters=turbo_iters)
        else:
            nb = int(n_bits or SLOT_SIZE * self.Nd * cfg.bits_per_symbol)
            n_sym = int(np.ceil(nb / (self.Nd * cfg.bits_per_symbol)))
            chain = C.CHAIN_SIMO if num_rx > 1 else C.CHAIN_UNCODED
            plan = self._plan(chain, n_sym, nb, num_rx=num_rx, max_frames=frames_per_call)
        ids = np.array([s * T + t for s in range(S) for t in trial_shard(T, rank, world_size)], dtype=np.uint64)
        counts = np.zeros((S, 4), dtype=np.uint64)
        for i in range(0, len(ids), frames_per_call):
            chunk = ids[i:i + frames_per_call]
            si = (chunk // T).astype(np.int32)
            r = plan.run(snrs[si], snr_index=si, n_snr=S, seed=seed, frame_ids=chunk)
            counts += r['counts']
        with np.errstate(divide='ignore', invalid='ignore'):
            ber = counts[:, 0] / np.maximum(counts[:, 1], 1)
            bler = counts[:, 2] / np.maximum(counts[:, 3], 1)
        return {'snr_db': snrs, 'counts': counts, 'ber': ber, 'bler': bler, 'bit_errors': counts[:, 0],
                'bits': counts[:, 1], 'block_errors': counts[:, 2], 'blocks': counts[:, 3], 'plan': plan}


def _spatial_plan(config, channel_type, itu_profile, velocity_kmh, frequency_ghz, n_sym, n_bits, max_frames=1,
                  num_tx=4, num_rx=4, rank=4, detector=C.DET_MMSE, W=None, precision=None):
    ch = {'awgn': C.CH_AWGN, 'rayleigh_mp': C.CH_RAYLEIGH}.get(channel_type)
    if ch is None:
        raise ValueError(f"Tipo de canal desconocido: {channel_type}")
    if ch == C.CH_RAYLEIGH:
        # transmit_spatial_multiplexing re-wraps the already-converted gains once
        # more (core/channel.py:435-444, Q2); fD from velocity and carrier (:113-143)
        delays, gains = itu_paths(itu_profile, config.fs, spatial=True)
        fD = doppler(frequency_ghz, velocity_kmh, itu_profile)
    else:
        delays, gains, fD = [], [], 0.0
    if W is None:
        W = np.eye(num_tx, dtype=complex)[:, :rank]
    Wt = tuple(complex(v) for v in np.asarray(W, dtype=complex).ravel())
    return get_plan(N=config.N, Nc=config.Nc, cp_len=config.cp_length, bps=config.bits_per_symbol, n_sym=n_sym,
                    chain=C.CHAIN_SPATIAL, channel=ch, num_rx=num_rx, num_tx=num_tx, delays=tuple(delays),
                    gains=tuple(gains), fD=fD, fs=config.fs, n_bits=n_bits, max_frames=max_frames, rank=rank,
                    detector=detector, precoder=Wt, precision=precision), gains, fD


def simulate_spatial_multiplexing(bits, num_tx=4, num_rx=2, rank='adaptive', detector_type='MMSE',
                                  modulation='64-QAM', snr_db=15, config=None, channel_type='awgn',
                                  itu_profile='Pedestrian_A', velocity_kmh=3, frequency_ghz=2.0,
                                  enable_csi_feedback=True, coherence_time_symbols=None, enable_parallel=False,
                                  codebook_type='TM4', *, precision: Optional[str] = None):
    """simulate_spatial_multiplexing (core/ofdm_core.py:2489-2815): TM4 with
    2 / 4 TX, 1-4 RX, rank 1-4 -- one GPU call.  Host: H_initial (:2573-2574,
    drawn even at fixed rank) -> RankAdaptation.get_feedback on it for
    rank='adaptive' with CSI (RI / PMI / W, core/rank_adaptation.py:212-265),
    else the TM4 codebook's PMI 0 of the given rank (min(tx, rx) for
    'adaptive' without CSI).  GPU: QAM -> layers (first ceil(Nd/rank) data
    SCs, Q20) -> x = W layers -> CRS pilots per TX (cell tx % 4) -> IFFT/CP
    -> transmit_spatial_multiplexing -> FFT -> CRS estimate per symbol ->
    H_eff = H W -> MMSE / IRC / ZF / SIC / MRC with the nominal sigma^2 =
    10^(-SNR/10) -> layer demap -> hard bits.  Global-RNG consumption as the
    reference: H_initial -> TX pilot reseeds per symbol and TX -> channel draws
    (core/channel.py:397-493: rayleigh_mp per link 16 phases per path for
    filter() and 16 per path for impulse_response(); 'awgn' per link h ~
    CN(0,1); then noise per RX) -> RX pilot reseeds."""
    from .tm4 import DETECTORS, LTECodebook, RankAdaptation
    bits = np.asarray(bits)
    if bits.size == 0:
        raise ValueError("Bits array cannot be empty")
    det = DETECTORS.get(str(detector_type).upper())
    if config is None:
        config = LTEConfig(modulation=modulation)
    n0 = len(bits)
    grid = ResourceGrid(config.N, config.Nc)
    Nd = len(grid._data)
    bpo = Nd * config.bits_per_symbol
    n_sym = int(np.ceil(n0 / bpo))
    H_initial = (np.random.randn(num_rx, num_tx) + 1j * np.random.randn(num_rx, num_tx)) / np.sqrt(2 * num_tx)
    if rank == 'adaptive' and enable_csi_feedback:
        fb = RankAdaptation(num_tx, num_rx, snr_db=snr_db).get_feedback(H_initial)
        rank_used, pmi_used, W = fb['ri'], fb['pmi'], fb['W']
    else:
        rank_used = int(rank) if rank != 'adaptive' else min(num_tx, num_rx)
        pmi_used = 0
        W = LTECodebook(num_tx, transmission_mode='TM4', rank=rank_used).get_precoder(0)
    if num_rx < rank_used:
        raise ValueError(f"num_rx ({num_rx}) debe ser >= num_layers ({rank_used})")
    if det is None:
        raise ValueError(f"Detector '{detector_type}' no soportado")
    if det == C.DET_MRC and rank_used != 1:
        raise ValueError("MRC solo soporta num_layers=1 (rank-1)")
    plan, gains, fD = _spatial_plan(config, channel_type, itu_profile, velocity_kmh, frequency_ghz, n_sym, n0,
                                    num_tx=num_tx, num_rx=num_rx, rank=rank_used, detector=det, W=W,
                                    precision=precision)
    L = plan.L
    ray = channel_type == 'rayleigh_mp'
    step = num_tx if num_tx <= 4 else 4
    pidx = [grid._pilot[t % step::step] for t in range(num_tx)]
    for t in range(num_tx):
        _reseed_pilots(t % 4, len(pidx[t]))
    P = len(plan.desc.delays[:plan.desc.n_paths]) if ray else 0
    ph = np.zeros((num_rx, num_tx, max(P, 1), 16))
    ir = np.zeros((num_rx, num_tx, max(P, 1), 16))
    lh = np.zeros((num_rx, num_tx, 2))
    for r in range(num_rx):
        for t in range(num_tx):
            if ray:
                for p in range(P):
                    ph[r, t, p] = 2 * np.pi * np.random.rand(16)
                for p in range(P):
                    ir[r, t, p] = 2 * np.pi * np.random.rand(16)
            else:
                lh[r, t, 0] = np.random.normal(0, 1 / np.sqrt(2))
                lh[r, t, 1] = np.random.normal(0, 1 / np.sqrt(2))
    z = np.zeros((num_rx, 2, L))
    for r in range(num_rx):
        z[r, 0] = np.random.normal(0, 1.0, L)
        z[r, 1] = np.random.normal(0, 1.0, L)
    for t in range(num_tx):
        _reseed_pilots(t % 4, len(pidx[t]))
    out = plan.run([snr_db], bits=(bits & 1).astype(np.uint8)[None], phases=ph[None] if ray else None,
                   noise=z[None], link_h=None if ray else lh[None], capture=('bits_rx', 'data_syms'))
    brx = out['bits_rx'][0].astype(np.int64)
    err = int(np.sum(bits != brx))
    Hm = np.zeros((num_rx, num_tx), dtype=complex)
    for r in range(num_rx):
        for t in range(num_tx):
            if ray:   # RayleighChannel.impulse_response(N=1) first tap (core/rayleighchannel.py:99-113)
                h = np.zeros(1, dtype=complex)
                for m in range(16):
                    h += np.exp(1j * (2 * np.pi * fD * np.cos(2 * np.pi * (m + 1) / 16) * np.zeros(1) + ir[r, t, 0, m]))
                Hm[r, t] = gains[0] * (h * np.sqrt(2 / 16))[0]
            else:
                Hm[r, t] = lh[r, t, 0] + 1j * lh[r, t, 1]
    return {'transmitted_bits': int(n0), 'received_bits': int(n0), 'bits_received_array': brx,
            'bit_errors': err, 'errors': err, 'ber': float(err / n0), 'snr_db': float(snr_db),
            'num_tx': num_tx, 'num_rx': num_rx, 'rank': int(rank_used), 'detector_type': detector_type,
            'mode': 'Spatial Multiplexing TM4', 'codebook_type': codebook_type, 'channel_matrix': Hm,
            'precoder_matrix': W, 'pmi_used': pmi_used, 'velocity_kmh': velocity_kmh,
            'modulation': modulation, 'symbols_rx': out['data_syms'][0].astype(np.complex128)}
