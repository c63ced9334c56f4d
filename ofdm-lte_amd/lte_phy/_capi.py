"""ctypes binding of liblte_hip.so (include/lte_phy.h).

The library is the product: every compute call of this package goes through
it.  There is no CPU fallback -- if the library is missing or no gfx950 GPU is
visible, calls raise loudly.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('LTE_HIP_LIB', os.path.join(_HERE, 'liblte_hip.so'))

LTE_OK, LTE_EINVAL, LTE_EHIP, LTE_ENOMEM, LTE_ENODEV, LTE_EUNSUP = 0, -1, -2, -3, -4, -5
CHAIN_UNCODED, CHAIN_CODED, CHAIN_SIMO, CHAIN_SFBC, CHAIN_SFBC_CODED, CHAIN_SPATIAL, CHAIN_BEAMFORMING = 0, 1, 2, 3, 4, 5, 6
CH_AWGN, CH_RAYLEIGH = 0, 1
DET_MMSE, DET_ZF, DET_SIC, DET_MRC = 0, 1, 2, 3
STAGE_TX, STAGE_CHANNEL, STAGE_RX, STAGE_ALL = 1, 2, 4, 7
MAX_PATHS = 16
PREC_DEFAULT, PREC_F32, PREC_F64 = 0, 32, 64
ABI_VERSION = 3   # LTE_ABI_VERSION of include/lte_phy.h that these ctypes layouts describe

c_i32, c_i64, c_u64, c_f64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double
P = ctypes.POINTER


class PlanDesc(ctypes.Structure):
    _fields_ = [('N', c_i32), ('Nc', c_i32), ('cp_len', c_i32), ('bps', c_i32), ('n_sym', c_i32),
                ('chain', c_i32), ('channel', c_i32), ('num_rx', c_i32), ('n_paths', c_i32),
                ('delays', c_i32 * MAX_PATHS), ('gains', c_f64 * MAX_PATHS), ('fD', c_f64), ('fs', c_f64),
                ('n_bits', c_i32), ('turbo_iters', c_i32), ('max_frames', c_i32), ('cell_id', c_i32),
                ('num_tx', c_i32), ('rank', c_i32), ('detector', c_i32), ('precoder', c_f64 * 32),
                ('sc_fdm', c_i32), ('bf_adaptive', c_i32), ('no_equalization', c_i32), ('precision', c_i32)]


class RunArgs(ctypes.Structure):
    _fields_ = [('n_frames', c_i32), ('snr_db', P(c_f64)), ('snr_index', P(c_i32)), ('n_snr', c_i32),
                ('seed', c_u64), ('frame_ids', P(c_u64)), ('frame_id0', c_u64),
                ('bits', P(ctypes.c_uint8)), ('bits_stride', c_i64),
                ('phases', P(c_f64)), ('phases_stride', c_i64),
                ('noise', P(c_f64)), ('noise_stride', c_i64),
                ('counts', P(c_u64)), ('frame_errors', P(ctypes.c_uint32)), ('frame_crc_ok', P(ctypes.c_uint8)),
                ('stages', c_i32), ('in_signal', ctypes.c_void_p), ('in_signal_stride', c_i64),
                ('cap_signal_tx', ctypes.c_void_p), ('cap_signal_rx', ctypes.c_void_p),
                ('cap_data_syms', ctypes.c_void_p), ('cap_H', ctypes.c_void_p),
                ('cap_pilot_stats', ctypes.c_void_p), ('cap_bits_rx', P(ctypes.c_uint8)),
                ('cap_llr', ctypes.c_void_p), ('cap_noise_power', ctypes.c_void_p),
                ('cap_tx_syms', ctypes.c_void_p),
                ('link_noise', P(c_f64)), ('link_noise_stride', c_i64),
                ('link_h', P(c_f64)), ('link_h_stride', c_i64),
                ('cap_link_stats', ctypes.c_void_p),
                ('cap_pmi', P(c_i32)), ('cap_bf_gain', P(c_f64))]


# every symbol include/lte_phy.h declares, with its ctypes signature
_SIGS = {
    'lte_strerror': (ctypes.c_char_p, [ctypes.c_int]),
    'lte_last_error': (ctypes.c_char_p, []),
    'lte_device_init': (ctypes.c_int, [ctypes.c_int]),
    'lte_version': (ctypes.c_int, []),
    'lte_abi_check': (ctypes.c_int, [ctypes.c_int]),
    'lte_plan_create': (ctypes.c_int, [P(PlanDesc), P(ctypes.c_void_p)]),
    'lte_plan_destroy': (ctypes.c_int, [ctypes.c_void_p]),
    'lte_plan_info': (ctypes.c_int, [ctypes.c_void_p, P(c_i64)]),
    'lte_plan_precision': (ctypes.c_int, [ctypes.c_void_p]),
    'lte_run': (ctypes.c_int, [ctypes.c_void_p, P(RunArgs)]),
    'lte_timing_enable': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    'lte_timing_read': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, P(c_f64), P(c_i64),
                                       ctypes.c_int]),
    'lte_timing_reset': (ctypes.c_int, [ctypes.c_void_p]),
    'lte_fft_host': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, P(ctypes.c_float), P(ctypes.c_float)]),
    'lte_fft_host64': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, P(c_f64), P(c_f64)]),
    'lte_pilots': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, P(c_f64)]),
    'lte_philox_host': (ctypes.c_int, [c_u64, ctypes.c_int, P(c_u64), ctypes.c_uint32, c_i64, P(ctypes.c_uint32),
                                       P(c_f64), P(ctypes.c_float)]),
    'lte_dft_host': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, P(ctypes.c_float), P(ctypes.c_float)]),
    'lte_dft_host64': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, P(c_f64), P(c_f64)]),
    'lte_llr_host': (ctypes.c_int, [ctypes.c_int, c_i64, P(ctypes.c_float), P(ctypes.c_float), P(ctypes.c_float)]),
    'lte_llr_host64': (ctypes.c_int, [ctypes.c_int, c_i64, P(c_f64), P(c_f64), P(c_f64)]),
    'lte_hard_host': (ctypes.c_int, [ctypes.c_int, c_i64, P(ctypes.c_float), P(ctypes.c_uint8)]),
    'lte_hard_host64': (ctypes.c_int, [ctypes.c_int, c_i64, P(c_f64), P(ctypes.c_uint8)]),
    'lte_qam_map_host64': (ctypes.c_int, [ctypes.c_int, c_i64, P(ctypes.c_uint8), P(c_f64)]),
    'lte_nearest_host64': (ctypes.c_int, [ctypes.c_int, c_i64, P(c_f64), P(ctypes.c_uint8)]),
    'lte_chest_host64': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, P(c_i32), P(c_f64), c_i64, P(c_f64), P(c_f64),
                                        P(c_f64), P(c_f64)]),
    'lte_zf_host64': (ctypes.c_int, [c_i64, P(c_f64), P(c_f64), c_f64, P(c_f64)]),
    'lte_rsc_encode_host': (ctypes.c_int, [c_i64, P(ctypes.c_uint8), ctypes.c_int, P(ctypes.c_uint8),
                                           P(ctypes.c_uint8)]),
    'lte_turbo_encode_host': (ctypes.c_int, [ctypes.c_int, c_i64, P(ctypes.c_uint8), P(ctypes.c_uint8)]),
    'lte_turbo_decode_host': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, P(ctypes.c_float),
                                             P(ctypes.c_uint8)]),
    'lte_bcjr_host': (ctypes.c_int, [ctypes.c_int, c_i64, P(ctypes.c_float), P(ctypes.c_float),
                                     P(ctypes.c_float), P(ctypes.c_float)]),
    'lte_turbo_decode_host64': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, P(c_f64), P(ctypes.c_uint8)]),
    'lte_bcjr_host64': (ctypes.c_int, [ctypes.c_int, c_i64, P(c_f64), P(c_f64), P(c_f64), P(c_f64)]),
    'lte_crc_host': (ctypes.c_int, [c_i64, P(ctypes.c_uint8), ctypes.c_uint32, ctypes.c_int,
                                    P(ctypes.c_uint32)]),
    'lte_mimo_detect_host': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            c_i64, P(c_f64), P(c_f64), P(c_f64), c_f64, P(c_f64)]),
    'lte_sfbc_encode_host64': (ctypes.c_int, [c_i64, P(c_f64), P(c_f64), P(c_f64)]),
    'lte_sfbc_decode_host64': (ctypes.c_int, [c_i64, P(c_f64), P(c_f64), P(c_f64), c_f64, P(c_f64)]),
    'lte_rate_dematch_map': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, P(c_i32)]),
    'lte_rate_dematch_host64': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, c_i64, P(c_f64), P(c_f64)]),
    'lte_qpp_perm': (ctypes.c_int, [ctypes.c_int, P(c_i32)]),
    'lte_subblock_perm': (ctypes.c_int, [ctypes.c_int, P(c_i32)]),
    'lte_set_decoder_mode': (ctypes.c_int, [ctypes.c_int]),
    'lte_channel_host': (ctypes.c_int, [c_i64, ctypes.c_int, ctypes.c_int, ctypes.c_int, P(c_i32), P(c_f64),
                                        c_f64, c_f64, c_f64, c_u64, P(ctypes.c_float), P(c_f64), P(c_f64),
                                        P(ctypes.c_float), P(ctypes.c_float)]),
    'lte_channel_host64': (ctypes.c_int, [c_i64, ctypes.c_int, ctypes.c_int, ctypes.c_int, P(c_i32), P(c_f64),
                                          c_f64, c_f64, c_f64, c_u64, P(c_f64), P(c_f64), P(c_f64),
                                          P(c_f64), P(c_f64)]),
    'lte_channel_mimo_host': (ctypes.c_int, [c_i64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, P(c_i32), P(c_f64), c_f64, c_f64, c_f64, c_u64,
                                             P(ctypes.c_float), P(c_f64), P(c_f64), P(c_f64), P(c_f64),
                                             P(ctypes.c_float), P(ctypes.c_float), P(ctypes.c_float)]),
    'lte_channel_mimo_host64': (ctypes.c_int, [c_i64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, P(c_i32), P(c_f64), c_f64, c_f64, c_f64, c_u64,
                                               P(c_f64), P(c_f64), P(c_f64), P(c_f64), P(c_f64),
                                               P(c_f64), P(c_f64), P(c_f64)]),
}

_lib = None
_lock = threading.Lock()
_device_ready = {}


def load():
    """Load liblte_hip.so (raises if it has not been built)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f"liblte_hip.so not found at {LIB_PATH}: build it with "
                                   f"`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in _SIGS.items():
                f = getattr(lib, name)
                f.restype = res
                f.argtypes = args
            if lib.lte_abi_check(ABI_VERSION) != LTE_OK:   # the RunArgs layout above is ABI 3's
                raise RuntimeError(f"{LIB_PATH}: {lib.lte_last_error().decode(errors='replace')}; rebuild it")
            _lib = lib
    return _lib


PRECISIONS = ('f64', 'f32')


def precision_of(p=None):
    """Arithmetic type of the GPU chains: 'f64' (the default -- the reference
    computes in float64 / complex128 throughout) or 'f32' (opt-in fast mode).
    LTE_PRECISION in the environment changes the default."""
    p = p or os.environ.get('LTE_PRECISION', 'f64')
    if p not in PRECISIONS:
        raise ValueError(f"precision must be one of {PRECISIONS}, got {p!r}")
    return p


def check(rc):
    if rc >= 0:
        return rc
    lib = load()
    msg = lib.lte_last_error().decode(errors='replace') or lib.lte_strerror(rc).decode()
    if rc == LTE_EINVAL:
        raise ValueError(msg)
    if rc == LTE_EUNSUP:
        raise NotImplementedError(msg)
    raise RuntimeError(f"liblte_hip: {lib.lte_strerror(rc).decode()}: {msg}")


def device_init(device=None):
    if device is None:
        device = int(os.environ.get('LOCAL_RANK', '0')) if 'LTE_DEVICE' not in os.environ else \
            int(os.environ['LTE_DEVICE'])
    if not _device_ready.get(device):
        check(load().lte_device_init(device))
        _device_ready[device] = True
    return device


def ptr(a, t):
    if a is None:
        return None
    return a.ctypes.data_as(P(t))


F32, U8, U32, U64, I32, F64 = ctypes.c_float, ctypes.c_uint8, ctypes.c_uint32, c_u64, c_i32, c_f64


def _cdtype(prec):
    return (np.complex128, np.float64, F64) if prec == 'f64' else (np.complex64, np.float32, F32)


def fft(x, inverse=False, precision=None):
    """Batched N-point FFT/sqrt(N) (inverse: IFFT*sqrt(N)) on the GPU; x [..., N] complex.
    precision 'f64' (default, complex128) or 'f32' (complex64)."""
    device_init()
    prec = precision_of(precision)
    cdt, rdt, ct = _cdtype(prec)
    x = np.ascontiguousarray(x, dtype=cdt)
    N = x.shape[-1]
    out = np.empty_like(x)
    f = load().lte_fft_host64 if prec == 'f64' else load().lte_fft_host
    check(f(N, 1 if inverse else 0, x.size // N, ptr(x.view(rdt), ct), ptr(out.view(rdt), ct)))
    return out


def dft(x, inverse=False, precision=None):
    """SC-FDM DFT (inverse: IDFT) of size M = x.shape[-1], unitary (1/sqrt(M)), on the GPU."""
    device_init()
    prec = precision_of(precision)
    cdt, rdt, ct = _cdtype(prec)
    x = np.ascontiguousarray(x, dtype=cdt)
    M = x.shape[-1]
    out = np.empty_like(x)
    f = load().lte_dft_host64 if prec == 'f64' else load().lte_dft_host
    check(f(M, 1 if inverse else 0, x.size // M, ptr(x.view(rdt), ct), ptr(out.view(rdt), ct)))
    return out


def pilots(cell_id, n):
    out = np.empty(2 * n, dtype=np.float64)
    check(load().lte_pilots(cell_id, n, ptr(out, F64)))
    return out[0::2] + 1j * out[1::2]


def philox(seed, frame_ids, stream, n_ctr):
    """The Philox mode's device streams (lte_philox_host): per frame and
    counter the four 32-bit outputs [nf, n_ctr, 4] uint32 and the unit normal
    pairs the noise kernels form from them, float64 and float32 [nf, n_ctr, 4]
    (re / im of the (x, y) pair, then of the (z, w) pair)."""
    device_init()
    fid = np.ascontiguousarray(np.atleast_1d(frame_ids), dtype=np.uint64)
    nf, n_ctr = len(fid), int(n_ctr)
    u = np.empty((nf, n_ctr, 4), dtype=np.uint32)
    g64 = np.empty((nf, n_ctr, 4), dtype=np.float64)
    g32 = np.empty((nf, n_ctr, 4), dtype=np.float32)
    check(load().lte_philox_host(int(seed) & 0xFFFFFFFFFFFFFFFF, nf, ptr(fid, U64), int(stream), n_ctr, ptr(u, U32),
                                 ptr(g64, F64), ptr(g32, F32)))
    return u, g64, g32


def rate_dematch_map(K, E, rv_idx=0):
    src = np.empty(3 * K + 12, dtype=np.int32)
    check(load().lte_rate_dematch_map(K, E, rv_idx, ptr(src, I32)))
    return src


def mimo_detect(det, y, H, sigma2, W, bps=0):
    """MIMODetector.detect per subcarrier on the GPU (lte_mimo_detect_host):
    y [num_rx, n] , H [num_rx, num_tx, n], W [num_tx, rank] -> [rank, n]."""
    device_init()
    y = np.ascontiguousarray(y, dtype=np.complex128)
    H = np.ascontiguousarray(H, dtype=np.complex128)
    W = np.ascontiguousarray(W, dtype=np.complex128)
    nr, n = y.shape
    nt, rank = W.shape
    if H.shape != (nr, nt, n):
        raise ValueError(f"H shape {H.shape} does not match y {y.shape} and W {W.shape}")
    out = np.empty((rank, n), dtype=np.complex128)
    check(load().lte_mimo_detect_host(int(det), nr, nt, rank, int(bps), n, ptr(y.view(np.float64), F64),
                                      ptr(H.view(np.float64), F64), ptr(W.view(np.float64), F64), float(sigma2),
                                      ptr(out.view(np.float64), F64)))
    return out


def sfbc_encode(symbols):
    """SFBCAlamouti.encode on the GPU (lte_sfbc_encode_host64): [n] complex -> (tx0, tx1)."""
    s = np.ascontiguousarray(symbols, dtype=np.complex128)
    if s.ndim != 1:
        raise ValueError(f"symbols must be 1-D, got shape {s.shape}")
    device_init()
    tx0, tx1 = np.empty_like(s), np.empty_like(s)
    check(load().lte_sfbc_encode_host64(len(s), ptr(s.view(np.float64), F64), ptr(tx0.view(np.float64), F64),
                                        ptr(tx1.view(np.float64), F64)))
    return tx0, tx1


def sfbc_decode(rx, H0, H1, regularization=1e-10):
    """SFBCAlamouti.decode on the GPU (lte_sfbc_decode_host64).  The C entry
    reads len(rx) values from each of H0 / H1: lengths are checked here."""
    r = np.ascontiguousarray(rx, dtype=np.complex128)
    h0 = np.ascontiguousarray(H0, dtype=np.complex128)
    h1 = np.ascontiguousarray(H1, dtype=np.complex128)
    if r.ndim != 1 or h0.ndim != 1 or h1.ndim != 1:
        raise ValueError(f"rx, H0, H1 must be 1-D, got shapes {r.shape}, {h0.shape}, {h1.shape}")
    if not (len(h0) == len(h1) == len(r)):
        raise ValueError(f"Channel estimates must have length {len(r)}")
    device_init()
    out = np.empty_like(r)
    check(load().lte_sfbc_decode_host64(len(r), ptr(r.view(np.float64), F64), ptr(h0.view(np.float64), F64),
                                        ptr(h1.view(np.float64), F64), float(regularization),
                                        ptr(out.view(np.float64), F64)))
    return out


precision = precision_of   # short alias used by the coding entry points
