"""Drop-in mirror of core/channel.py's channel models: AWGNChannel,
RayleighMultiPathChannel and FadingChannel (ChannelSimulator, which holds
one of them, is in ofdm_core).

Each transmit is one GPU pass (lte_channel_host64: Jakes fading, multipath,
the measured power of the whole stream, noise = sqrt(P / SNR / 2) * z) on the
random numbers the reference draws from the global NumPy RNG, drawn here in
the reference's order (16 phases per path, then the real and the imaginary
noise vectors), so results and the RNG state after the call are the
reference's."""
from __future__ import annotations

from typing import Optional

import numpy as np

from . import _capi as C
from .config import ITU_CHANNEL_MODELS
from .rayleighchannel import RayleighChannel


def gpu_channel(x, num_rx, kind, delays, gains, fD, fs, snr_db, phases, noise, precision='f64'):
    """One lte_channel_host64 (f32: lte_channel_host) call: x [L] -> (y
    [num_rx][L], noise power [num_rx]); delays in samples, gains as
    amplitudes, phases [num_rx][P][16] radians, noise [num_rx][2][L] unit
    normals."""
    C.device_init()
    f64 = precision == 'f64'
    cdt, rdt, ct = (np.complex128, np.float64, C.F64) if f64 else (np.complex64, np.float32, C.F32)
    x = np.ascontiguousarray(x, dtype=cdt)
    L = len(x)
    y = np.zeros((num_rx, L), dtype=cdt)
    npow = np.zeros(num_rx, dtype=rdt)
    P = len(delays)
    dl = np.ascontiguousarray(delays, dtype=np.int32)
    g = np.ascontiguousarray(gains, dtype=np.float64)
    ph = np.ascontiguousarray(phases, dtype=np.float64) if P else None
    z = np.ascontiguousarray(noise, dtype=np.float64)
    fn = C.load().lte_channel_host64 if f64 else C.load().lte_channel_host
    C.check(fn(L, num_rx, kind, P, C.ptr(dl, C.I32) if P else None, C.ptr(g, C.F64) if P else None, float(fD),
               float(fs or 0.0), float(snr_db), 0, C.ptr(x.view(rdt), ct), C.ptr(ph, C.F64) if P else None,
               C.ptr(z, C.F64), C.ptr(y.view(rdt), ct), C.ptr(npow, ct)))
    return y.astype(np.complex128), npow.astype(np.float64)


def _noise_draws(L):
    """The reference's two legacy-normal vectors of one noise draw, as unit
    normals (normal(0, s, L) = 0 + s * gauss: the same gauss sequence)."""
    return np.stack([np.random.normal(0, 1.0, L), np.random.normal(0, 1.0, L)])


def _noise_vector(z, noise_power):
    s = np.sqrt(noise_power / 2)
    return (0 + s * z[0]) + 1j * (0 + s * z[1])


def _complex_only(signal):
    if not np.iscomplexobj(signal):
        raise NotImplementedError("the GPU channel serves complex baseband streams (real-valued signal given)")


class AWGNChannel:
    """AWGNChannel (core/channel.py:10-80): noise power = measured signal
    power / SNR.  transmit returns (received, noise)."""

    def __init__(self, snr_db=10.0, *, precision: Optional[str] = None):
        self.snr_db = snr_db
        self.snr_linear = 10 ** (snr_db / 10)
        self.noise_power = None
        self.precision = C.precision_of(precision)

    def set_snr(self, snr_db):
        self.snr_db = snr_db
        self.snr_linear = 10 ** (snr_db / 10)

    def transmit(self, signal):
        _complex_only(signal)
        x = np.asarray(signal)
        z = _noise_draws(len(x))
        y, npow = gpu_channel(x, 1, C.CH_AWGN, [], [], 0.0, 0.0, self.snr_db, None, z[None], self.precision)
        self.noise_power = npow[0]
        return y[0], _noise_vector(z, npow[0])

    def get_noise_power(self):
        return self.noise_power

    def get_snr_info(self):
        return {'SNR (dB)': self.snr_db, 'SNR (lineal)': self.snr_linear, 'Potencia de ruido': self.noise_power}


class RayleighMultiPathChannel:
    """RayleighMultiPathChannel (core/channel.py:83-245): ITU-R M.1225 taps
    (amplitudes, then converted again by RayleighChannel, quirk Q2), the fD
    rule of the reference, Jakes fading + measured-power AWGN."""

    def __init__(self, snr_db=10.0, fs=None, itu_profile='Vehicular_A', fD=None, frequency_ghz=None,
                 velocity_kmh=None, verbose=True, *, precision: Optional[str] = None):
        self.snr_db = snr_db
        self.snr_linear = 10 ** (snr_db / 10)
        self.itu_profile = itu_profile
        self.fs = fs
        self.noise_power = None
        self.frequency_ghz = frequency_ghz
        self.velocity_kmh = velocity_kmh
        self.verbose = verbose
        self.precision = C.precision_of(precision)
        delays, gains = self._get_itu_profile_params(itu_profile)
        if fD is None:
            if frequency_ghz is not None and velocity_kmh is not None:
                fc, v = frequency_ghz * 1e9, velocity_kmh / 3.6
            else:
                v = (5.0 if 'Pedestrian' in itu_profile else 30.0 if 'Vehicular_A' in itu_profile else
                     120.0 if 'Vehicular_B' in itu_profile else 10.0) / 3.6
                fc = 2e9
            fD = (v * fc) / 3e8
        self.rayleigh = RayleighChannel(fs, fD, delays, gains)
        if self.verbose:
            print(f"[RayleighMultiPathChannel] Perfil: {itu_profile}")
            print(f"  - Retardos: {[f'{d * 1e6:.2f}µs' for d in delays]}")
            print(f"  - Ganancias: {[f'{g:.1f}dB' for g in gains]}")
            print(f"  - Doppler máximo: {fD:.1f} Hz")
            if frequency_ghz is not None:
                print(f"  - Frecuencia: {frequency_ghz:.2f} GHz")
            if velocity_kmh is not None:
                print(f"  - Velocidad: {velocity_kmh:.1f} km/h")

    def _get_itu_profile_params(self, profile_name):
        if profile_name not in ITU_CHANNEL_MODELS:
            raise ValueError(f"Perfil ITU no encontrado: {profile_name}. "
                             f"Opciones disponibles: {list(ITU_CHANNEL_MODELS.keys())}")
        d = ITU_CHANNEL_MODELS[profile_name]
        return np.array(d['delays_us']) * 1e-6, 10 ** (np.array(d['power_db']) / 20)

    def set_snr(self, snr_db):
        self.snr_db = snr_db
        self.snr_linear = 10 ** (snr_db / 10)

    def set_profile(self, itu_profile):
        """The reference stores the new amplitudes without the second
        conversion here (core/channel.py:195-201); kept."""
        self.itu_profile = itu_profile
        delays, gains = self._get_itu_profile_params(itu_profile)
        self.rayleigh.delays = np.array(delays)
        self.rayleigh.gains = gains
        self.rayleigh.num_paths = len(delays)

    def transmit(self, signal):
        """rayleigh.filter, then AWGN on the measured power (:203-234): one
        GPU pass.  Returns (received, None)."""
        x = np.asarray(signal, dtype=np.complex128)
        rc = self.rayleigh
        P = rc.num_paths
        ph = np.stack([2 * np.pi * np.random.rand(16) for _ in range(P)])[None] if P else None
        z = _noise_draws(len(x))
        d = [int(np.round(t * rc.Fs)) for t in rc.delays]
        y, npow = gpu_channel(x, 1, C.CH_RAYLEIGH, d, rc.gains, rc.fD, rc.Fs, self.snr_db, ph, z[None],
                              self.precision)
        self.noise_power = npow[0]
        return y[0], None

    def get_channel_info(self):
        return {'type': 'Rayleigh MultiPath (ITU-R M.1225)', 'profile': self.itu_profile, 'SNR_dB': self.snr_db,
                'num_paths': self.rayleigh.num_paths, 'delays_us': self.rayleigh.delays * 1e6,
                'gains_dB': 20 * np.log10(self.rayleigh.gains)}


class FadingChannel:
    """FadingChannel (core/channel.py:248-291): per-sample h ~ CN(0, 1) (the
    reference's 'future extension'), then AWGN on the GPU.  The per-sample
    product x h is formed on the host before the GPU noise pass (this model
    is outside SURVEY §8's rows)."""

    def __init__(self, snr_db=10.0, fading_type='rayleigh', *, precision: Optional[str] = None):
        self.snr_db = snr_db
        self.snr_linear = 10 ** (snr_db / 10)
        self.fading_type = fading_type
        self.awgn_channel = AWGNChannel(snr_db, precision=precision)

    def transmit(self, signal):
        n = len(signal)
        h = np.random.normal(0, 1 / np.sqrt(2), n) + 1j * np.random.normal(0, 1 / np.sqrt(2), n)
        received, _ = self.awgn_channel.transmit(np.asarray(signal) * h)
        return received, h
