"""Channel-coding API (drop-in names of core/channel_coding/__init__.py:15-40).

The compute-heavy functions (turbo encode / decode, CRC-24A, one BCJR pass)
run on the GPU through liblte_hip.so; segmentation and rate (de)matching are
index bookkeeping built from the library's native tables.
"""
import numpy as np

from . import _capi as C

CRC24A_POLYNOMIAL = 0x1864CFB
CRC24B_POLYNOMIAL = 0x1800063
USE_MAX_LOG_MAP = True


_TURBO_SIZES = ([40 + 8 * i for i in range(60)] + [528 + 16 * i for i in range(32)] +
                [1056 + 32 * i for i in range(32)] + [2112 + 64 * i for i in range(64)])


def segmentation_sizes(B):
    """Code-block sizes of segment_code_blocks (segmentation.py:74-263) for a
    transport block of B bits (CRC-24A included)."""
    Z, L = 6144, 24
    if B <= Z:
        return [next(k for k in _TURBO_SIZES if k >= B)]
    C_ = -(-B // (Z - L))
    Bp = B + C_ * L
    Kp = next(k for k in _TURBO_SIZES if k >= -(-Bp // C_))
    i = _TURBO_SIZES.index(Kp)
    Km = _TURBO_SIZES[i - 1] if i > 0 else Kp
    Cm = (C_ * Kp - Bp) // (Kp - Km) if Kp > Km else 0
    return [Km] * Cm + [Kp] * (C_ - Cm)


def set_decoder_mode(use_max_log_map: bool = True):
    """turbo_decoder.py:35-54.  Only max-log-MAP (the reference default) runs on the GPU."""
    if not use_max_log_map:
        raise NotImplementedError("exact log-MAP is not on the GPU path (the reference defaults to max-log)")


def calculate_crc24a(data_bits):
    """crc.py:137-159 on the GPU (same kernel that attaches the TB CRC)."""
    C.device_init()
    b = np.ascontiguousarray(np.asarray(data_bits), dtype=np.uint8)
    out = np.zeros(1, dtype=np.uint32)
    C.check(C.load().lte_crc_host(len(b), C.ptr(b, C.U8), CRC24A_POLYNOMIAL, 24, C.ptr(out, C.U32)))
    v = int(out[0])
    return np.array([(v >> (23 - i)) & 1 for i in range(24)], dtype=np.uint8)


def attach_crc24a(data_bits):
    return np.concatenate([np.asarray(data_bits), calculate_crc24a(data_bits)])


def check_crc24a(data_with_crc):
    d = np.asarray(data_with_crc)
    if len(d) < 24:
        return False
    return bool(np.array_equal(d[-24:], calculate_crc24a(d[:-24])))


def turbo_encode(input_bits):
    """turbo_encoder.py:214-313 on the GPU: [d0 d1 d2]*K + 12 tail bits."""
    C.device_init()
    b = np.ascontiguousarray(np.asarray(input_bits), dtype=np.uint8)
    K = len(b)
    out = np.zeros(3 * K + 12, dtype=np.uint8)
    C.check(C.load().lte_turbo_encode_host(K, 1, C.ptr(b, C.U8), C.ptr(out, C.U8)))
    return out


def turbo_decode(llr_encoded, K, num_iterations=5, debug=False, precision=None):
    """turbo_decoder.py:338-450 on the GPU (max-log BCJR).  precision 'f64'
    (default, bit-exact with the reference) or 'f32' (fast mode)."""
    return turbo_decode_batch(np.asarray(llr_encoded)[None], K, num_iterations, precision)[0]


def turbo_decode_batch(llrs, K, num_iterations=8, precision=None):
    """Decode many code blocks of the same K at once: llrs [ncb][3K+12]."""
    C.device_init()
    prec = C.precision(precision)
    out = np.zeros((np.asarray(llrs).size // (3 * K + 12), K), dtype=np.uint8)
    if prec == 'f64':
        L = np.ascontiguousarray(llrs, dtype=np.float64).reshape(-1, 3 * K + 12)
        C.check(C.load().lte_turbo_decode_host64(K, int(num_iterations), L.shape[0], C.ptr(L, C.F64),
                                                 C.ptr(out, C.U8)))
    else:
        L = np.ascontiguousarray(llrs, dtype=np.float32).reshape(-1, 3 * K + 12)
        C.check(C.load().lte_turbo_decode_host(K, int(num_iterations), L.shape[0], C.ptr(L, C.F32),
                                               C.ptr(out, C.U8)))
    return out


def rate_match_turbo(encoded_bits, E, K, rv_idx=0):
    """rate_matching.py:193-297 via the native dematch map (its inverse)."""
    enc = np.asarray(encoded_bits)
    if len(enc) != 3 * K + 12:
        raise ValueError(f"Invalid encoded_bits length. Expected {3*K + 12}, got {len(enc)}")
    Ncb = 3 * (K + 6)
    src = C.rate_dematch_map(K, min(E, Ncb), rv_idx)
    cb = np.zeros(min(E, Ncb), dtype=np.uint8)
    m = src >= 0
    cb[src[m]] = enc[m]
    return cb[np.arange(E) % len(cb)] if E > Ncb else cb


def rate_dematching_turbo(rate_matched_llrs, K, rv_idx=0, debug=False):
    """rate_matching.py:374-489 (no repetition: E <= N_cb)."""
    llr = np.asarray(rate_matched_llrs, dtype=np.float64)
    src = C.rate_dematch_map(K, len(llr), rv_idx)
    out = np.zeros(3 * K + 12)
    m = src >= 0
    out[m] = llr[src[m]]
    return out
