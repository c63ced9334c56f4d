"""Channel-coding API: every name of core/channel_coding/__init__.py:15-40.

The compute-heavy functions run on the GPU through liblte_hip.so:
  * CRC-24A / CRC-24B (the payload kernel's CRC, crc.py:89-347),
  * turbo encode (turbo_encoder.py:214-313),
  * turbo decode and LogMAPDecoder.decode (float64 max-log-MAP by default,
    bit-exact with the reference; exact log-MAP after set_decoder_mode(False);
    float32 fast mode on request),
  * rate_dematching_turbo for any E (repeats summed on the device).
Segmentation, the QPP / sub-block permutations and rate matching are index
bookkeeping; their permutations come from the library's native tables
(lte_qpp_perm, lte_subblock_perm, lte_rate_dematch_map).
"""
from typing import List, Tuple

import numpy as np

from . import _capi as C

CRC24A_POLYNOMIAL = 0x1864CFB
CRC24B_POLYNOMIAL = 0x1800063
CRC16_POLYNOMIAL = 0x11021
USE_MAX_LOG_MAP = True

__all__ = ['calculate_crc24a', 'calculate_crc24b', 'attach_crc24a', 'attach_crc24b', 'check_crc24a', 'check_crc24b',
           'segment_code_blocks', 'desegment_code_blocks', 'get_segmentation_info', 'turbo_encode', 'turbo_decode',
           'LogMAPDecoder', 'qpp_interleave', 'qpp_deinterleave', 'rate_match_turbo', 'rate_dematching_turbo',
           'sub_block_interleaver', 'sub_block_deinterleaver']

# segmentation.py:32-51 (TS 36.212 Table 5.1.3-3)
TURBO_INTERLEAVER_SIZES = ([40 + 8 * i for i in range(60)] + [528 + 16 * i for i in range(32)] +
                           [1056 + 32 * i for i in range(32)] + [2112 + 64 * i for i in range(64)])
_TURBO_SIZES = TURBO_INTERLEAVER_SIZES


def find_interleaver_size(min_size: int) -> int:
    """segmentation.py:53-71."""
    for size in TURBO_INTERLEAVER_SIZES:
        if size >= min_size:
            return size
    raise ValueError(f"No valid interleaver size found for min_size={min_size}")


# ---------------------------------------------------------------- CRC (GPU)
def _crc(data_bits, poly, length=24):
    C.device_init()
    b = np.ascontiguousarray(np.asarray(data_bits), dtype=np.uint8) & 1
    out = np.zeros(1, dtype=np.uint32)
    C.check(C.load().lte_crc_host(len(b), C.ptr(b, C.U8), poly, length, C.ptr(out, C.U32)))
    v = int(out[0])
    return np.array([(v >> (length - 1 - i)) & 1 for i in range(length)], dtype=np.uint8)


def calculate_crc24a(data_bits: np.ndarray) -> np.ndarray:
    """crc.py:137-159 on the GPU."""
    return _crc(data_bits, CRC24A_POLYNOMIAL)


def calculate_crc24b(data_bits: np.ndarray) -> np.ndarray:
    """crc.py:162-184 on the GPU."""
    return _crc(data_bits, CRC24B_POLYNOMIAL)


def attach_crc24a(data_bits: np.ndarray) -> np.ndarray:
    """crc.py:212-233."""
    return np.concatenate([data_bits, calculate_crc24a(data_bits)])


def attach_crc24b(data_bits: np.ndarray) -> np.ndarray:
    """crc.py:236-257."""
    return np.concatenate([data_bits, calculate_crc24b(data_bits)])


def check_crc24a(data_with_crc: np.ndarray) -> bool:
    """crc.py:277-307."""
    d = np.asarray(data_with_crc)
    if len(d) < 24:
        return False
    return bool(np.array_equal(d[-24:], calculate_crc24a(d[:-24])))


def check_crc24b(data_with_crc: np.ndarray) -> bool:
    """crc.py:310-347."""
    d = np.asarray(data_with_crc)
    if len(d) < 24:
        return False
    return bool(np.array_equal(d[-24:], calculate_crc24b(d[:-24])))


def calculate_crc16(data_bits: np.ndarray) -> np.ndarray:
    """crc.py:187-209 on the GPU (the serial CRC kernel, poly 0x11021)."""
    return _crc(data_bits, CRC16_POLYNOMIAL, 16)


def attach_crc16(data_bits: np.ndarray) -> np.ndarray:
    """crc.py:260-274."""
    return np.concatenate([data_bits, calculate_crc16(data_bits)])


def check_crc16(data_with_crc: np.ndarray) -> bool:
    """crc.py:343-367."""
    d = np.asarray(data_with_crc)
    if len(d) < 16:
        return False
    return bool(np.array_equal(d[-16:], calculate_crc16(d[:-16])))


def get_test_vectors_crc24a():
    """crc.py:370-394: (data, CRC-24A) for 40 zeros, 40 ones, alternating 0/1."""
    vecs = [np.zeros(40, dtype=np.uint8), np.ones(40, dtype=np.uint8),
            np.array([i % 2 for i in range(40)], dtype=np.uint8)]
    return [(v, calculate_crc24a(v)) for v in vecs]


# ---------------------------------------------------------------- segmentation
def _seg_params(B):
    """C, K-, K+, C-, C+, F of segmentation.py:147-187 (B > Z)."""
    Z, L = 6144, 24
    Cn = int(np.ceil(B / (Z - L)))
    Bp = B + Cn * L
    Kp = find_interleaver_size(int(np.ceil(Bp / Cn)))
    i = TURBO_INTERLEAVER_SIZES.index(Kp) - 1
    Km = TURBO_INTERLEAVER_SIZES[i] if i >= 0 else Kp
    dK = Kp - Km
    Cm = (Cn * Kp - Bp) // dK if dK > 0 else 0
    return Cn, Km, Kp, Cm, Cn - Cm, Cn * Kp - Bp + Cm * (Kp - Km)


def _bits_per_block(B, sizes):
    """Information bits of each code block (segmentation.py:193-214, 303-316)."""
    out, rem, Cn = [], B, len(sizes)
    for r, K in enumerate(sizes):
        n = rem if r == Cn - 1 else min(K - 24, rem // (Cn - r))
        out.append(n)
        rem -= n
    return out


def segmentation_sizes(B):
    """Code-block sizes of segment_code_blocks for a transport block of B bits
    (CRC-24A included)."""
    if B <= 6144:
        return [find_interleaver_size(B)]
    Cn, Km, Kp, Cm, Cp, _ = _seg_params(B)
    return [Km] * Cm + [Kp] * Cp


def segment_code_blocks(transport_block_with_crc: np.ndarray) -> Tuple[List[np.ndarray], dict]:
    """segmentation.py:74-263: fillers (zeros) first, then the information
    bits; CRC-24B (on the GPU) per block when C > 1."""
    tb = np.asarray(transport_block_with_crc)
    B = len(tb)
    if B <= 6144:
        K = find_interleaver_size(B)
        F = K - B
        cb = np.zeros(K, dtype=np.uint8)
        cb[F:] = tb
        return [cb], {'num_blocks': 1, 'block_sizes': [K], 'num_filler_bits': F,
                      'filler_positions': list(range(F)) if F > 0 else [], 'filler_per_block': [F],
                      'original_size': B, 'segmented': False}
    Cn, Km, Kp, Cm, Cp, F = _seg_params(B)
    sizes = [Km] * Cm + [Kp] * Cp
    info = _bits_per_block(B, sizes)
    blocks, fill, fpos, pos = [], [], [], 0
    for K, n in zip(sizes, info):
        cb = np.zeros(K - 24, dtype=np.uint8)
        Fr = (K - 24) - n
        fill.append(Fr)
        if n > 0:
            cb[Fr:Fr + n] = tb[pos:pos + n]
        if Fr > 0:
            fpos.extend(range(len(fpos), len(fpos) + Fr))
        pos += n
        blocks.append(attach_crc24b(cb))
    return blocks, {'num_blocks': Cn, 'block_sizes': sizes, 'num_filler_bits': F, 'filler_positions': fpos,
                    'filler_per_block': fill, 'original_size': B, 'segmented': True, 'K_plus': Kp,
                    'K_minus': Km, 'C_plus': Cp, 'C_minus': Cm}


def desegment_code_blocks(code_blocks: List[np.ndarray], metadata: dict) -> np.ndarray:
    """segmentation.py:266-359: drop CRC-24B and fillers, concatenate."""
    B = metadata['original_size']
    if not metadata['segmented']:
        F = metadata['num_filler_bits']
        return code_blocks[0][F:F + B]
    sizes = metadata['block_sizes']
    out = []
    for cb, K, n in zip(code_blocks, sizes, _bits_per_block(B, sizes)):
        Fr = (K - 24) - n
        out.append(cb[:-24][Fr:Fr + n])
    return np.concatenate(out)


def get_segmentation_info(transport_block_size: int) -> dict:
    """segmentation.py:362-420."""
    sizes = segmentation_sizes(transport_block_size)
    return {'num_blocks': len(sizes), 'block_sizes': sizes, 'total_coded_bits': sum(3 * K + 12 for K in sizes)}


# ---------------------------------------------------------------- turbo encode (GPU)
def _qpp(K):
    perm = np.empty(int(K), dtype=np.int32)
    C.check(C.load().lte_qpp_perm(int(K), C.ptr(perm, C.I32)))
    return perm


def qpp_interleave(data: np.ndarray, K: int) -> np.ndarray:
    """turbo_encoder.py:76-103: out[i] = data[(f1 i + f2 i^2) mod K]."""
    return np.asarray(data)[_qpp(K)]


def qpp_deinterleave(data: np.ndarray, K: int) -> np.ndarray:
    """turbo_encoder.py:105-134 (inverse permutation)."""
    perm = _qpp(K)
    inv = np.zeros(int(K), dtype=int)
    inv[perm] = np.arange(int(K))
    return np.asarray(data)[inv]


def rsc_encode(input_bits: np.ndarray, trellis_termination: bool = True) -> Tuple[np.ndarray, np.ndarray]:
    """turbo_encoder.py:137-211 on the GPU (lte_rsc_encode_host): the
    'systematic' output is the feedback bit, the termination feeds s1 ^ s2."""
    C.device_init()
    b = np.ascontiguousarray(np.asarray(input_bits), dtype=np.uint8) & 1
    m = len(b) + (3 if trellis_termination else 0)
    sys_, par = np.zeros(m, dtype=np.uint8), np.zeros(m, dtype=np.uint8)
    C.check(C.load().lte_rsc_encode_host(len(b), C.ptr(b, C.U8), 1 if trellis_termination else 0,
                                         C.ptr(sys_, C.U8), C.ptr(par, C.U8)))
    return sys_, par


def turbo_encode_block_list(code_blocks: list) -> list:
    """turbo_encoder.py:316-329."""
    return [turbo_encode(block) for block in code_blocks]


def turbo_encode(input_bits):
    """turbo_encoder.py:214-313 on the GPU: [d0 d1 d2]*K + 12 tail bits."""
    C.device_init()
    b = np.ascontiguousarray(np.asarray(input_bits), dtype=np.uint8)
    K = len(b)
    out = np.zeros(3 * K + 12, dtype=np.uint8)
    C.check(C.load().lte_turbo_encode_host(K, 1, C.ptr(b, C.U8), C.ptr(out, C.U8)))
    return out


# ---------------------------------------------------------------- turbo decode (GPU)
def set_decoder_mode(use_max_log_map: bool = True):
    """turbo_decoder.py:35-54: True = max-log-MAP (default), False = exact
    log-MAP (log_sum_exp max*), for every float64 decode on the GPU."""
    global USE_MAX_LOG_MAP
    USE_MAX_LOG_MAP = bool(use_max_log_map)
    C.check(C.load().lte_set_decoder_mode(1 if use_max_log_map else 0))
    mode = "Max-Log-MAP (fast)" if use_max_log_map else "True Log-MAP (exact)"
    print(f"Turbo Decoder mode set to: {mode}")


def log_sum_exp(a: float, b: float) -> float:
    """turbo_decoder.py:64-88 (the scalar max* of exact log-MAP; the GPU
    decoders evaluate the same expression per trellis branch)."""
    if np.isinf(a) and a < 0:
        return b
    if np.isinf(b) and b < 0:
        return a
    if a > b:
        return a + np.log1p(np.exp(b - a))
    return b + np.log1p(np.exp(a - b))


def max_star(a: float, b: float) -> float:
    """turbo_decoder.py:91-115: max(a, b) in max-log-MAP mode, else log_sum_exp."""
    if USE_MAX_LOG_MAP:
        return max(a, b)
    return log_sum_exp(a, b)


def turbo_decode(llr_encoded, K, num_iterations=5, debug=False, *, precision=None):
    """turbo_decoder.py:338-450 on the GPU.  precision 'f64' (default,
    bit-exact with the reference) or 'f32' (fast mode, max-log only)."""
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


class LogMAPDecoder:
    """turbo_decoder.py:118-335: one BCJR pass of the 8-state RSC over any
    length (tail steps included), float64 on the GPU (lte_bcjr_host64), max*
    per set_decoder_mode.  The trellis tables mirror _build_trellis."""

    def __init__(self):
        self.num_states = 8
        self.num_memory = 3
        self._build_trellis()

    def _build_trellis(self):
        self.next_state = np.zeros((8, 2), dtype=int)
        self.output_systematic = np.zeros((8, 2), dtype=int)
        self.output_parity = np.zeros((8, 2), dtype=int)
        for s in range(8):
            s0, s1, s2 = (s >> 2) & 1, (s >> 1) & 1, s & 1
            for u in range(2):
                fb = (u + s1 + s2) % 2
                self.next_state[s, u] = (fb << 2) | (s0 << 1) | s1
                self.output_systematic[s, u] = fb
                self.output_parity[s, u] = (fb + s0 + s2) % 2

    def decode(self, llr_systematic: np.ndarray, llr_parity: np.ndarray, llr_apriori: np.ndarray = None,
               return_extrinsic: bool = True) -> Tuple[np.ndarray, np.ndarray]:
        ls = np.ascontiguousarray(llr_systematic, dtype=np.float64)
        K = len(ls)
        lp = np.ascontiguousarray(llr_parity, dtype=np.float64)[:K]
        la = np.zeros(K) if llr_apriori is None else np.ascontiguousarray(llr_apriori, dtype=np.float64)[:K]
        if len(lp) < K or len(la) < K:
            raise ValueError("llr_parity / llr_apriori shorter than llr_systematic")
        if K == 0:   # the reference's recursions run zero steps: empty decisions and LLRs
            return np.zeros(0, dtype=np.uint8), np.zeros(0)
        C.device_init()
        app = np.zeros(K)
        C.check(C.load().lte_bcjr_host64(K, 1, C.ptr(ls, C.F64), C.ptr(np.ascontiguousarray(lp), C.F64),
                                         C.ptr(np.ascontiguousarray(la), C.F64), C.ptr(app, C.F64)))
        out = (app - la - ls) if return_extrinsic else app
        return (app < 0).astype(np.uint8), out


# ---------------------------------------------------------------- rate matching
def _sbi(n):
    perm = np.empty(int(n), dtype=np.int32)
    C.check(C.load().lte_subblock_perm(int(n), C.ptr(perm, C.I32)))
    return perm


def sub_block_interleaver(input_bits: np.ndarray, D: int = 32) -> np.ndarray:
    """rate_matching.py:25-94 (D = 32 columns; <NULL>s removed)."""
    if D != 32:
        raise ValueError("the LTE sub-block interleaver has D = 32 columns")
    x = np.asarray(input_bits)
    if len(x) == 0:
        return np.array([], dtype=np.uint8)
    return x[_sbi(len(x))].astype(np.uint8)


def sub_block_deinterleaver(input_bits: np.ndarray, original_length: int, D: int = 32) -> np.ndarray:
    """rate_matching.py:97-190: the inverse permutation; like the reference
    the output is uint8 (its int matrix truncates), and missing input leaves
    its positions out."""
    if D != 32:
        raise ValueError("the LTE sub-block interleaver has D = 32 columns")
    n = int(original_length)
    if n == 0:
        return np.array([], dtype=np.uint8)
    x = np.asarray(input_bits)
    perm = _sbi(n)
    m = min(len(x), n)
    out = np.full(n, -1, dtype=np.int64)
    out[perm[:m]] = np.asarray(x[:m]).astype(np.int64)
    return out[out != -1].astype(np.uint8)


def sub_block_deinterleaver_llr(interleaved_data: np.ndarray, K_original: int) -> np.ndarray:
    """rate_matching.py:300-371, an index permutation: NULL cells are the
    last of R x 32 in column-major order of the original matrix, moved by the
    column permutation; the values fill the permuted matrix row-major around
    them, the inverse column permutation is applied and the matrix is read
    column-major without the NULLs (NaN inputs are dropped like NULLs, as
    the reference does), truncated to K_original."""
    x = np.asarray(interleaved_data, dtype=np.float64).ravel()
    D, Kpi = 32, len(x)
    R = int(np.ceil(Kpi / D))
    P = np.array([0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30,
                  1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31])
    P_inv = np.argsort(P)
    rows, cols = np.meshgrid(np.arange(R), np.arange(D), indexing='ij')
    null_orig = cols * R + rows >= Kpi
    null_perm = np.zeros((R, D), dtype=bool)
    null_perm[:, P] = null_orig
    perm = np.full((R, D), np.nan)
    slots = np.flatnonzero(~null_perm.ravel())
    n = min(len(slots), Kpi)
    perm.ravel()[slots[:n]] = x[:n]
    out = perm[:, P_inv].T.ravel()
    return np.array(out[~np.isnan(out)][:K_original], dtype=np.float64)


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
    """rate_matching.py:374-489 on the GPU for any E: punctured positions 0.0,
    repeats (E > N_cb) summed in order onto 0.0."""
    llr = np.ascontiguousarray(rate_matched_llrs, dtype=np.float64)
    out = np.zeros(3 * K + 12)
    if len(llr) == 0:   # E = 0: every position punctured (the reference returns zeros(3K + 12))
        return out
    C.device_init()
    C.check(C.load().lte_rate_dematch_host64(int(K), len(llr), int(rv_idx), 1, C.ptr(llr, C.F64), C.ptr(out, C.F64)))
    return out
