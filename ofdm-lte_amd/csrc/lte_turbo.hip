// Channel-coding kernels around the turbo decoder (lte_decoder.hip) for
// gfx950: RX rate dematch into the decoder's row layout (with the soft
// demapper fused in), TX code-block construction + turbo encoding, and the
// RX CRC-24A / desegmentation / bit-error count.
#include "lte_common.h"
#include "lte_internal.h"
#include "lte_dev.h"

namespace lte {


// ---------------------------------------------------------------------------
// RX rate-dematch + transpose into the decoder layout, rows of R (double: the
// default float64 chain; float: fast mode).
// Replaces rate_dematching_turbo (rate_matching.py:374-489) composed with the
// T/F de-interleaver (core/ofdm_core.py:1174-1207): rx_map[layer][t] gives, for
// LLR t of a frame in RE order, the destination (r<<24 | row) or -1.  Layer 0
// writes 0.5 * (0 + llr) (the circular buffer starts at zero); layers 1.. hold
// the repeats of E > N_cb and ADD in order (circular_buffer[pos] += llr[i],
// rate_matching.py:433-436), one launch per layer so the sums keep the
// reference's order.  Rows hold LLR/2: x/2 commutes with every rounded add.
// A block loads a [64 frames][DM_CH t] tile (coalesced rows), then every wave
// writes whole decoder rows (64 frames of one LLR).
constexpr int DM_CH = 64;
// LTE_DM_NT (A/B): 1 = non-temporal decoder-row stores, 3 = also non-temporal
// loads of the equalised symbols / noise variances (k_dematch_zn)
#ifndef LTE_DM_NT
#define LTE_DM_NT 0
#endif
template <class R>
__device__ __forceinline__ void dm_store(R* dst, R v, bool add) {
  if (add) *dst = *dst + (R)0.5 * v;
  else if (LTE_DM_NT & 1) __builtin_nontemporal_store((R)0.5 * ((R)0 + v), dst);
  else *dst = (R)0.5 * ((R)0 + v);
}

template <class R>
__global__ __launch_bounds__(256) void k_dematch(const R* __restrict__ llr, int T, int B,
                                                 const int32_t* __restrict__ rx_map, int add,
                                                 R* const* __restrict__ blk, const int64_t* __restrict__ rows,
                                                 int ch, int g0) {
  __shared__ R tile[64][DM_CH + 1];   // [frame][t], +1: conflict-free column reads
  const int g = g0 + blockIdx.y;
  const int t0 = blockIdx.x * DM_CH;
  const int nt = min(DM_CH, T - t0);
  // load: 16 lanes x 4 LLRs per frame row (coalesced); scalar tail
  const int c4 = (threadIdx.x & 15) * 4;
  for (int f = threadIdx.x >> 4; f < 64; f += 16) {
    const int b = g * 64 + f;
    const R* src = llr + (size_t)b * T + t0;
    R v[4] = {(R)0, (R)0, (R)0, (R)0};
    if (b < B) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (c4 + e < nt) v[e] = src[c4 + e];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) tile[f][c4 + e] = v[e];
  }
  __syncthreads();
  // store: each wave writes whole decoder rows (64 frames of one LLR)
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), f = threadIdx.x & 63;
  for (int c = wv; c < nt; c += 4) {
    const int m = rx_map[t0 + c];
    if (m < 0) continue;
    const int r = m >> 24, row = m & 0xFFFFFF;
    dm_store(&blk[r][turbo_elem_ch(ch, rows[r], g, row) + f], tile[f][c], add != 0);
  }
}

template <class R>
int launch_dematch(hipStream_t s, const R* llr, int T, int B, const int32_t* rx_map, int n_layers, R* const* blk,
                   const int64_t* rows, int ch, int g0) {
  const int G = (B + 63) / 64 - g0;   // groups g0 .. ceil(B/64)-1
  if (G < 1 || G > 65535 || n_layers < 1) return (int)hipErrorInvalidValue;
  for (int k = 0; k < n_layers; ++k) {
    hipLaunchKernelGGL(k_dematch<R>, dim3((T + DM_CH - 1) / DM_CH, G), dim3(256), 0, s, llr, T, B,
                       rx_map + (size_t)k * T, k > 0 ? 1 : 0, blk, rows, ch, g0);
    const int e = (int)hipGetLastError();
    if (e) return e;
  }
  return 0;
}

// Soft demap + dematch in one pass: a block covers DZ_RE resource elements of
// 64 frames; it reads their equalised symbols and noise variances (instead of
// bps LLRs per RE), computes the max-log LLRs (soft_demap, the function
// k_rx_data uses) into an LDS tile [frame][LLR], then writes whole decoder
// rows exactly as k_dematch.  f64 covers 8 REs per block (49 KB tile at 16).
// The noise variance is per (frame, 14-symbol group, data subcarrier): RE re =
// l * nd + j of a frame reads nv[b * n_nv + (l / 14) * nd + j].
#ifndef LTE_DZ_RE64   // REs per block for float64 (A/B: 16 = 256-B symbol spans per frame, 50 KB tile)
#define LTE_DZ_RE64 8
#endif
template <class R> constexpr int dz_re() { return sizeof(R) == 8 ? LTE_DZ_RE64 : 16; }
template <class R, int BPS>
__global__ __launch_bounds__(256) void k_dematch_zn(const cx<R>* __restrict__ z, const R* __restrict__ nv, int n_re,
                                                    int nd, int n_nv, int nv_grp, int nv_sh, int B,
                                                    const int32_t* __restrict__ rx_map, int add,
                                                    R* const* __restrict__ blk, const int64_t* __restrict__ rows,
                                                    int ch, int g0) {
  using V = cx<R>;
  constexpr int DZ_RE = dz_re<R>(), TC = DZ_RE * BPS, PER = 64 * DZ_RE / 256;
  __shared__ R tile[64][TC + 1];
  const int g = g0 + blockIdx.y;
  const int re0 = blockIdx.x * DZ_RE;
  const int nr = min(DZ_RE, n_re - re0);
  // every (z, nv) load of this thread issued before the demapping
  V zv[PER];
  R nvv[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = threadIdx.x + k * 256, f = e / DZ_RE, r = e % DZ_RE, b = g * 64 + f;
    const bool ok = b < B && r < nr;
    const size_t i = (size_t)b * n_re + re0 + r;
    const int l = (re0 + r) / nd, j = re0 + r - l * nd;
    if (LTE_DM_NT & 2) {
      zv[k] = ok ? mkc(__builtin_nontemporal_load(&z[i].x), __builtin_nontemporal_load(&z[i].y)) : mkc((R)0, (R)0);
      nvv[k] = ok ? __builtin_nontemporal_load(&nv[(size_t)b * n_nv + (l / nv_grp) * (nd >> nv_sh) + (j >> nv_sh)])
                  : (R)1;
    } else {
      zv[k] = ok ? z[i] : mkc((R)0, (R)0);
      nvv[k] = ok ? nv[(size_t)b * n_nv + (l / nv_grp) * (nd >> nv_sh) + (j >> nv_sh)] : (R)1;
    }
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = threadIdx.x + k * 256, f = e / DZ_RE, r = e % DZ_RE;
    R o[BPS];
    soft_demap<BPS>(zv[k], nvv[k], o);
#pragma unroll
    for (int m = 0; m < BPS; ++m) tile[f][r * BPS + m] = o[m];
  }
  __syncthreads();
  const int t0 = re0 * BPS, nt = nr * BPS;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), f = threadIdx.x & 63;
  for (int c = wv; c < nt; c += 4) {
    const int m = rx_map[t0 + c];
    if (m < 0) continue;
    const int r = m >> 24, row = m & 0xFFFFFF;
    dm_store(&blk[r][turbo_elem_ch(ch, rows[r], g, row) + f], tile[f][c], add != 0);
  }
}

template <class R>
int launch_dematch_zn(hipStream_t s, const cx<R>* z, const R* nv, int n_re, int nd, int bps, int B,
                      const int32_t* rx_map, int n_layers, R* const* blk, const int64_t* rows, int ch, int g0,
                      int nv_pairs) {
  const int G = (B + 63) / 64 - g0;
  if (G < 1 || G > 65535 || (bps != 4 && bps != 6) || n_layers < 1 || nd < 1) return (int)hipErrorInvalidValue;
  if (nv_pairs && (nd & 1)) return (int)hipErrorInvalidValue;
  // nv per (14-symbol group, data subcarrier) (SISO), or per (symbol, RE pair) (SFBC)
  const int nv_grp = nv_pairs ? 1 : 14, nv_sh = nv_pairs ? 1 : 0;
  const int n_nv = ((n_re / nd + nv_grp - 1) / nv_grp) * (nd >> nv_sh);
  constexpr int DZ = dz_re<R>();
  const dim3 grid((n_re + DZ - 1) / DZ, G);
  const int T = n_re * bps;
  for (int k = 0; k < n_layers; ++k) {
    const int32_t* mp = rx_map + (size_t)k * T;
    if (bps == 4)
      hipLaunchKernelGGL((k_dematch_zn<R, 4>), grid, dim3(256), 0, s, z, nv, n_re, nd, n_nv, nv_grp, nv_sh, B, mp,
                         k > 0 ? 1 : 0, blk, rows, ch, g0);
    else
      hipLaunchKernelGGL((k_dematch_zn<R, 6>), grid, dim3(256), 0, s, z, nv, n_re, nd, n_nv, nv_grp, nv_sh, B, mp,
                         k > 0 ? 1 : 0, blk, rows, ch, g0);
    const int e = (int)hipGetLastError();
    if (e) return e;
  }
  return 0;
}

template int launch_dematch<float>(hipStream_t, const float*, int, int, const int32_t*, int, float* const*,
                                   const int64_t*, int, int);
template int launch_dematch<double>(hipStream_t, const double*, int, int, const int32_t*, int, double* const*,
                                    const int64_t*, int, int);
template int launch_dematch_zn<float>(hipStream_t, const float2*, const float*, int, int, int, int, const int32_t*,
                                      int, float* const*, const int64_t*, int, int, int);
template int launch_dematch_zn<double>(hipStream_t, const double2*, const double*, int, int, int, int,
                                       const int32_t*, int, double* const*, const int64_t*, int, int, int);

// ---------------------------------------------------------------------------
// Stage entry: rate_dematching_turbo (rate_matching.py:374-489) for any E,
// repetition included.  One thread per (code block, output j of [3K+12]):
// src0[j] is the first rate-matched index feeding j (-1: punctured, stays
// 0.0); the repeats i0 + m N_cb (m >= 1, E > N_cb) are summed in order of i
// onto 0.0, exactly as circular_buffer[pos] += llr[i] (:433-436).
__global__ __launch_bounds__(256) void k_rate_dematch(const double* __restrict__ llr, int E, int Ncb, int n_out,
                                                      const int32_t* __restrict__ src0, int64_t ncb,
                                                      double* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= ncb * n_out) return;
  const int64_t c = t / n_out;
  const int j = (int)(t - c * n_out);
  double v = 0.0;
  const double* l = llr + c * E;
  for (int i = src0[j]; i >= 0 && i < E; i += Ncb) v = v + l[i];
  out[t] = v;
}

int launch_rate_dematch(hipStream_t s, const double* llr, int E, int Ncb, int n_out, const int32_t* src0, int64_t ncb,
                        double* out) {
  const int64_t n = ncb * n_out;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_rate_dematch, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, llr, E, Ncb, n_out, src0, ncb,
                     out);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// TX: CB construction (segmentation.py:212-247 + CRC-24B crc.py:162-184) and
// turbo encoding (turbo_encoder.py:137-313).  One lane = one (CB slot, frame).
struct BitWriter {   // MSB-first stream writer; one store per completed word
  uint32_t* p;
  uint64_t acc;
  int n;
  __device__ __forceinline__ void put(uint32_t bits, int nb) {   // nb in [1, 32]
    acc = (acc << nb) | (nb == 32 ? (uint64_t)bits : (uint64_t)(bits & ((1u << nb) - 1u)));
    n += nb;
    if (n >= 32) {
      *p++ = (uint32_t)(acc >> (n - 32));
      n -= 32;
    }
  }
  __device__ __forceinline__ void flush() {
    if (n) *p = (uint32_t)(acc << (32 - n));
  }
};

// CRC-24 byte table (MSB-first, zero init; poly without the x^24 term)

// RSC code (turbo_encoder.py:137-211) 32 bits at a time, in closed form.  The
// feedback ("systematic", Q13) sequence obeys a_k = u_k ^ a_{k-2} ^ a_{k-3}, i.e.
// a = u / g0(D) with g0 = 1 + D^2 + D^3.  Since (1 + D^7) = g0 (1 + D^2 + D^3 +
// D^4), 1/g0 = (1 + D^2 + D^3 + D^4) / (1 + D^7): four shifted XORs, then a
// stride-7 prefix XOR in three doubling steps.  The state (s0, s1, s2) =
// (a_{-1}, a_{-2}, a_{-3}) adds its zero-input response (period 7; the three
// basis words below).  Parity q_k = a_k ^ a_{k-1} ^ a_{k-3}.  Words are
// MSB-first (time runs toward bit 0); u holds nb (multiple of 8) bits
// left-aligned, bits past nb are ignored.  Returns q, *fw = a (left-aligned),
// and leaves the state at time nb-1.
__device__ __forceinline__ uint32_t rsc_word(uint32_t u, int nb, uint32_t& s0, uint32_t& s1, uint32_t& s2,
                                             uint32_t* fw) {
  uint32_t y = u ^ (u >> 2) ^ (u >> 3) ^ (u >> 4);
  y ^= y >> 7;
  y ^= y >> 14;
  y ^= y >> 28;
  const uint32_t a = y ^ (s0 ? 0x72e5cb97u : 0u) ^ (s1 ? 0xe5cb972eu : 0u) ^ (s2 ? 0xb972e5cbu : 0u);
  const uint32_t q = a ^ ((a >> 1) | (s0 << 31)) ^ ((a >> 3) | (s2 << 31) | (s1 << 30) | (s0 << 29));
  s0 = (a >> (32 - nb)) & 1u;
  s1 = (a >> (33 - nb)) & 1u;
  s2 = (a >> (34 - nb)) & 1u;
  *fw = a;
  return q;
}

// one trellis-termination step (turbo_encoder.py:190-211): input s1 ^ s2 makes
// the feedback bit 0; returns fb | parity << 1
__device__ __forceinline__ uint32_t rsc_tail(uint32_t& s0, uint32_t& s1, uint32_t& s2) {
  const uint32_t fb = 0u, par = fb ^ s0 ^ s2;
  s2 = s1; s1 = s0; s0 = fb;
  return fb | (par << 1);
}

// TX coding in one kernel (k_encode): a workgroup of ENC_SEG waves owns 64
// consecutive frames (lanes) of one code-block slot r, so K, F, f1, f2 and the
// QPP permutation are uniform.  Wave q owns the CB words [q SW, (q+1) SW): the
// frame's word chain is ENC_SEG times shorter and a CU holds 4x the waves of a
// one-wave-per-64-blocks design (whose 45-KB LDS copy of the blocks allowed 3
// waves per CU).  Both serial recursions are linear over GF(2), so each wave
// runs them over its words from a zero start and the true starts are formed
// from the other waves' partial results, exchanged through LDS:
//  * CRC-24B (crc.py:162-184) over CB bits [0, Kd): crc = sum_q crc_q *
//    x^(Kd - end_q) mod P (lte_common.h CRC-24 algebra; x^(2^j) table below);
//  * the RSC encoders (turbo_encoder.py:137-313, rsc_word): the state after a
//    segment is A^len s_in ^ f_q, f_q the state reached from 0 and A the
//    zero-input step, of order 7 (g0 = 1 + D^2 + D^3 is primitive).  Encoder
//    2's f_q are summed bit by bit over the natural-order block (qmask), so
//    its interleaved walk runs once, from the true start.
// The code blocks (CB construction: segmentation.py:212-247) are parked in LDS
// as [word][lane] for encoder 2's QPP gathers (pi(i) is uniform: one
// conflict-free LDS read per bit).
constexpr int ENC_SEG = 4;
constexpr int ENC_MAXSW = 48;   // K <= 6144: 192 words, at most 48 per wave
constexpr int ENC_CH = 16;      // whole output words stored per bunch (each lane completes its line pieces)

struct X2Tab { uint32_t v[16]; };
constexpr X2Tab make_x2tab(uint32_t poly) {   // x^(2^j) mod P, j < 16
  X2Tab t{};
  uint32_t b = 2u;
  for (int j = 0; j < 16; ++j) {
    t.v[j] = b;
    uint32_t r = 0u;   // b * b mod P
    for (int i = 23; i >= 0; --i) {
      r = ((r << 1) & 0xFFFFFFu) ^ ((r & 0x800000u) ? poly : 0u);
      r ^= ((b >> i) & 1u) ? b : 0u;
    }
    b = r;
  }
  return t;
}
__constant__ X2Tab kX2B = make_x2tab((uint32_t)CRC24B_POLY);

__device__ __forceinline__ uint32_t crcb_xpow(int e) {   // x^e mod P_24B, 0 <= e < 65536
  uint32_t r = 1u;
  for (int j = 0; j < 16; ++j)
    if ((e >> j) & 1) r = gf24_mul(r, kX2B.v[j], (uint32_t)CRC24B_POLY);
  return r;
}

// RSC state (s0, s1, s2) packed as s0 | s1 << 1 | s2 << 2, advanced n steps with zero input
__device__ __forceinline__ uint32_t rsc_zero_steps(uint32_t st, int n) {
  uint32_t s0 = st & 1u, s1 = (st >> 1) & 1u, s2 = (st >> 2) & 1u;
  for (int k = n % 7; k > 0; --k) {
    const uint32_t fb = s1 ^ s2;
    s2 = s1; s1 = s0; s0 = fb;
  }
  return s0 | (s1 << 1) | (s2 << 2);
}

// Exclusive prefix of the segment-final states: the state entering wave q's
// words.  fin = [ENC_SEG][64] packed states reached from 0; len(q') = bits of
// segment q'.
__device__ __forceinline__ uint32_t rsc_seg_start(const uint32_t* fin, int q, int lane, int K, int SW) {
  uint32_t st = 0u;
  for (int p = 0; p < q; ++p) {
    const int len = max(0, min(K, 32 * (p + 1) * SW) - 32 * p * SW);
    st = rsc_zero_steps(st, len) ^ fin[p * 64 + lane];
  }
  return st;
}

__global__ __launch_bounds__(64 * ENC_SEG) void k_encode(const uint32_t* __restrict__ pw, int PW, int KWmax,
                                                         uint32_t* __restrict__ enc, int EW,
                                                         const CbInfo* __restrict__ cbi, int B,
                                                         const uint16_t* __restrict__ qmask, int qstride) {
  extern __shared__ uint32_t esm[];
  uint32_t* cwl = esm;                        // [KWmax][64] code blocks
  uint32_t* xch = esm + (size_t)KWmax * 64;   // [3][ENC_SEG][64] exchange: CRC, encoder-1 states, encoder-2 sums
  __shared__ uint32_t crc_t[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) crc_t[i] = crc24_table_entry(i, (uint32_t)CRC24B_POLY);
  const int G = (B + 63) >> 6;                // 64-frame groups per slot
  const int r = blockIdx.x / G;
  // wave index as a scalar: the segment bounds, K and the QPP walk stay in SGPRs
  const int lane = threadIdx.x & 63, q = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = (blockIdx.x - r * G) * 64 + lane;
  const bool act = b < B;
  const CbInfo ci = cbi[r];
  const int K = ci.K, F = ci.F, C = gridDim.x / G;
  const int KW = (K + 31) >> 5, KWf = K >> 5;
  const int SW = (KW + ENC_SEG - 1) / ENC_SEG;
  const int w0 = min(KW, q * SW), w1 = min(KW, w0 + SW);
  const bool last = w0 < w1 && w1 == KW;   // the wave holding the block's end writes the tails
  const uint32_t* tb = pw + (size_t)(act ? b : 0) * PW;
  uint32_t* e = enc + ((size_t)(act ? b : 0) * C + r) * 3 * EW;
  const int Kd = ci.crc ? K - 24 : K;   // every LTE K (and so Kd) is a multiple of 8
  // CB bit p in [F, Kd) is TB bit (off - F + p): the 32 bits of word w are a
  // fixed-offset window over TB words i00 + w, i00 + w + 1
  const int64_t base = (int64_t)ci.off - F;
  const int64_t i00 = base >> 5;   // arithmetic shift: floor for negative base
  const int o = (int)(base & 31);
  auto ldw = [&](int64_t i) -> uint32_t { return (i >= 0 && i < PW) ? tb[i] : 0u; };
  __syncthreads();   // crc_t
  // ---- 1. this wave's CB words (data bits) into LDS, their CRC from 0
  uint32_t crc = 0u;
  {
    uint32_t wa = ldw(i00 + w0), wb = ldw(i00 + w0 + 1);
    for (int w = w0; w < w1; ++w) {
      const uint32_t wn = ldw(i00 + w + 2);   // next window word, in flight during this one
      const int p0 = w * 32;
      uint32_t t = o ? ((wa << o) | (wb >> (32 - o))) : wa;
      if (p0 < F) t &= (F - p0 >= 32) ? 0u : (0xFFFFFFFFu >> (F - p0));   // filler bits are 0
      const int db = min(32, max(0, Kd - p0));                         // data bits of this word
      t &= db >= 32 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> db);
      if (ci.crc)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (8 * k < db) crc = ((crc << 8) & 0xFFFFFFu) ^ crc_t[((crc >> 16) ^ (t >> (24 - 8 * k))) & 0xFFu];
      cwl[w * 64 + lane] = t;
      wa = wb;
      wb = wn;
    }
  }
  xch[q * 64 + lane] = (ci.crc && 32 * w0 < Kd)
                           ? gf24_mul(crc, crcb_xpow(Kd - min(32 * w1, Kd)), (uint32_t)CRC24B_POLY) : 0u;
  __syncthreads();
  if (ci.crc) {   // the CB's CRC-24B into bits [Kd, K) of the words this wave owns
    crc = 0u;
#pragma unroll
    for (int p = 0; p < ENC_SEG; ++p) crc ^= xch[p * 64 + lane];
    const uint32_t L = crc << 8;   // left-aligned, MSB first
    for (int w = max(w0, Kd >> 5); w < w1; ++w) {
      const int p0 = 32 * w;
      cwl[w * 64 + lane] |= p0 <= Kd ? (L >> (Kd - p0)) : (L << (p0 - Kd));
    }
  }
  // ---- 2. encoder 1: the segment's end state from 0, then the real pass.
  // The same walk over the natural-order bits forms encoder 2's segment end
  // states from 0, by linearity: CB bit p enters the interleaved stream at
  // k = pi^-1(p), in segment t, and moves segment t's end state by
  // A^(end_t - 1 - k) (1, 0, 0); qmask[p] holds that 3-bit vector at bits 3t
  // (encode_qmask, host).  So encoder 2 later runs once, from its true start.
  uint32_t s0 = 0u, s1 = 0u, s2 = 0u, f;
  uint32_t F2 = 0u;
  const uint16_t* qm = qmask + (size_t)r * qstride;
  for (int w = w0; w < w1; ++w) {
    const uint32_t cwv = cwl[w * 64 + lane];
    const int nb = min(32, K - 32 * w);
    (void)rsc_word(cwv, nb, s0, s1, s2, &f);
    const uint32_t* qw = reinterpret_cast<const uint32_t*>(qm + 32 * w);   // uniform: scalar loads
#pragma unroll
    for (int j = 0; j < 32; j += 2) {
      const uint32_t pr = qw[j >> 1];   // qmask[32w + j] | qmask[32w + j + 1] << 16 (zero past K)
      F2 ^= (pr & 0xFFFFu) & (0u - ((cwv >> (31 - j)) & 1u));
      F2 ^= (pr >> 16) & (0u - ((cwv >> (30 - j)) & 1u));
    }
  }
  xch[(ENC_SEG + q) * 64 + lane] = s0 | (s1 << 1) | (s2 << 2);
  xch[(2 * ENC_SEG + q) * 64 + lane] = F2;
  __syncthreads();   // (also publishes the finished code blocks to encoder 2)
  uint32_t st = rsc_seg_start(xch + ENC_SEG * 64, q, lane, K, SW);
  s0 = st & 1u; s1 = (st >> 1) & 1u; s2 = (st >> 2) & 1u;
  uint32_t pf = 0, pq = 0;   // the last, partial word (K % 32 bits), if any
  int pnb = 0;
  for (int wc = w0; wc < w1; wc += ENC_CH) {
    uint32_t fb[ENC_CH], qb[ENC_CH];
#pragma unroll
    for (int j = 0; j < ENC_CH; ++j) {
      const int w = wc + j;
      fb[j] = qb[j] = 0u;
      if (w >= w1) continue;
      const int nb = min(32, K - 32 * w);
      const uint32_t qq = rsc_word(cwl[w * 64 + lane], nb, s0, s1, s2, &f);
      if (nb == 32) { fb[j] = f; qb[j] = qq; }
      else { pf = f; pq = qq; pnb = nb; }
    }
    if (act) {
#pragma unroll
      for (int j = 0; j < ENC_CH; ++j)
        if (wc + j < min(w1, KWf)) e[wc + j] = fb[j];
#pragma unroll
      for (int j = 0; j < ENC_CH; ++j)
        if (wc + j < min(w1, KWf)) e[EW + wc + j] = qb[j];
    }
  }
  if (last && act) {
    BitWriter wr0{e + KWf, 0, 0}, wr1{e + EW + KWf, 0, 0};
    if (pnb) {
      wr0.put(pf >> (32 - pnb), pnb);
      wr1.put(pq >> (32 - pnb), pnb);
    }
    for (int t = 0; t < 3; ++t) {   // trellis termination, encoder 1
      const uint32_t v = rsc_tail(s0, s1, s2);
      wr0.put(v & 1u, 1);
      wr1.put(v >> 1, 1);
    }
    wr0.flush();   // d0[K+3..K+5] (encoder 2's tail) is OR-ed in below
    wr1.flush();
  }
  // ---- 3. encoder 2 on the QPP-interleaved block, from its true start state.
  // The walk pi(k) = (f1 k + f2 k^2) mod K is formed 64 positions at a time,
  // lane l holding pi(k0 + l) = (pi(k0) + l d(k0) + f2 l (l - 1)) mod K, and
  // each gather takes its uniform row / shift by readlane: a per-bit scalar
  // recurrence would make the CU's one scalar unit the bottleneck.
  {
    uint32_t fall = 0u;   // every segment's end state from 0 (3 bits per segment)
#pragma unroll
    for (int p = 0; p < ENC_SEG; ++p) fall ^= xch[(2 * ENC_SEG + p) * 64 + lane];
    uint32_t st2 = 0u;
    for (int t = 0; t < q; ++t) {
      const int len = max(0, min(K, 32 * (t + 1) * SW) - 32 * t * SW);
      st2 = rsc_zero_steps(st2, len) ^ ((fall >> (3 * t)) & 7u);
    }
    s0 = st2 & 1u; s1 = (st2 >> 1) & 1u; s2 = (st2 >> 2) & 1u;
  }
  pq = 0;
  pnb = 0;
  {
    const int k0 = 32 * w0;
    int pi0 = (int)(((int64_t)ci.f1 * k0 + (int64_t)ci.f2 * k0 % K * k0) % K);
    int d0 = (int)(((int64_t)ci.f1 + (int64_t)ci.f2 * (2 * (int64_t)k0 + 1)) % K);   // pi(k+1) - pi(k)
    const float invK = 1.0f / (float)K;
    const int f2l = (int)(((int64_t)ci.f2 * lane * (lane - 1)) % K);
    const char* cwb = reinterpret_cast<const char*>(cwl) + 4 * lane;
    for (int w = w0; w < w1; w += 2) {
      int x = pi0 + (int)((lane * (int64_t)d0) % K) + f2l;   // < 3K
      x -= (int)((float)x * invK) * K;                      // float quotient: exact below 2^24, off by at most 1
      x += x < 0 ? K : 0;
      x -= x >= K ? K : 0;
      const int rowb = (x >> 5) << 8, shf = x & 31;
      uint32_t qw[2] = {0u, 0u};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (w + h >= w1) break;
        const int nb = min(32, K - 32 * (w + h));
        uint32_t u = 0u;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
          const int a = __builtin_amdgcn_readlane(rowb, 32 * h + j);
          const int sh = __builtin_amdgcn_readlane(shf, 32 * h + j);
          const uint32_t v = *reinterpret_cast<const uint32_t*>(cwb + a);
          u |= ((v << sh) >> 31) << (31 - j);   // positions past K: ignored by rsc_word (nb)
        }
        const uint32_t qq = rsc_word(u, nb, s0, s1, s2, &f);
        if (nb == 32) qw[h] = qq;
        else { pq = qq; pnb = nb; }
      }
      if (act) {   // the pair's whole words, back to back
        if (w < KWf) e[2 * EW + w] = qw[0];
        if (w + 1 < min(w1, KWf)) e[2 * EW + w + 1] = qw[1];
      }
      pi0 = (int)(((int64_t)pi0 + 64 * (int64_t)d0 + (int64_t)ci.f2 * 64 * 63) % K);
      d0 = (int)(((int64_t)d0 + 128 * (int64_t)ci.f2) % K);
    }
  }
  if (last && act) {
    BitWriter wr2{e + 2 * EW + KWf, 0, 0};
    if (pnb) wr2.put(pq >> (32 - pnb), pnb);
    for (int t = 0; t < 3; ++t) {
      const uint32_t v = rsc_tail(s0, s1, s2);
      const int pos = K + 3 + t;   // sys2 tail -> d0[K+3..K+5]
      if (v & 1u) e[pos >> 5] |= 1u << (31 - (pos & 31));
      wr2.put(v >> 1, 1);
    }
    wr2.flush();
  }
}

void encode_qmask(const CbInfo* cbs, int C, int qstride, uint16_t* out) {
  std::fill(out, out + (size_t)C * qstride, (uint16_t)0);
  for (int r = 0; r < C; ++r) {
    const int K = cbs[r].K, KW = (K + 31) / 32, SW = (KW + ENC_SEG - 1) / ENC_SEG;
    uint16_t v[7];
    uint32_t st = 1u;   // (s0, s1, s2) = (1, 0, 0): an input 1 from the zero state
    for (int m = 0; m < 7; ++m) {
      v[m] = (uint16_t)st;
      const uint32_t s0 = st & 1u, s1 = (st >> 1) & 1u, s2 = (st >> 2) & 1u;
      st = (s1 ^ s2) | (s0 << 1) | (s1 << 2);
    }
    for (int64_t k = 0; k < K; ++k) {
      const int p = (int)((cbs[r].f1 * k + (int64_t)cbs[r].f2 * k % K * k) % K);   // turbo_encoder.py:76-103
      const int t = (int)(k / (32 * SW)), end = std::min(32 * SW * (t + 1), K);
      out[(size_t)r * qstride + p] = (uint16_t)(v[(end - 1 - k) % 7] << (3 * t));
    }
  }
}

int launch_encode(hipStream_t s, const uint32_t* pw, int PW, int KWmax, uint32_t* enc, int EW,
                  const CbInfo* cbi_dev, int C, int B, const uint16_t* qmask, int qstride) {
  const int64_t blocks = (int64_t)C * ((B + 63) / 64);
  const size_t shm = ((size_t)KWmax * 64 + 3 * ENC_SEG * 64) * sizeof(uint32_t);
  if (blocks > 0x7FFFFFFF || KWmax > 4 * ENC_MAXSW + 1 || shm > 65536 || !qmask) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_encode, dim3((unsigned)blocks), dim3(64 * ENC_SEG), shm, s, pw, PW, KWmax, enc, EW, cbi_dev,
                     B, qmask, qstride);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// CRC-24A / desegmentation / bit-error count.  One lane per frame; lanes of a
// wave are 64 consecutive frames = one decoder group, so the decoded-word
// reads are coalesced rows; CRC_SEG waves split the frame's words.  Replaces desegment_code_blocks
// (segmentation.py:266-359), check_crc24a (crc.py:277-307) and the BER count
// (core/ofdm_core.py:1304-1311).

// 32 bits starting at bit position p of an MSB-first stream whose words are
// strided by `st` elements.
__device__ __forceinline__ uint32_t get32s(const uint32_t* w, int64_t st, int64_t p, int64_t nwords) {
  const int64_t i = p >> 5;
  const int o = (int)(p & 31);
  const uint32_t a = w[i * st];
  if (o == 0) return a;
  const uint32_t b = (i + 1 < nwords) ? w[(i + 1) * st] : 0u;
  return (a << o) | (b >> (32 - o));
}

// CRC_SEG waves per 64 frames: wave s walks TB words [s SW, (s+1) SW) of the
// 64 frames (lanes), so a frame's word chain is CRC_SEG times shorter and the
// chip holds CRC_SEG times more waves.  Each wave runs the CRC register from 0
// over its data bits (slice-by-4: one dependent step per word); the frame's
// CRC is sum_s crc_s * x^(data bits after segment s) mod P (lte_common.h CRC-24
// algebra, multipliers from the host), formed by wave 0 from the per-wave
// results parked in LDS.  The code-block layout (offsets, decoded-row bases)
// is read once into LDS: the word loop's address chain never waits on HBM.
constexpr int CRC_SEG = 8;
constexpr int CRC_MAXC = 32;   // code blocks per TB (LTE: at most 13)
struct CrcSeg { uint32_t x[CRC_SEG]; };

__global__ __launch_bounds__(64 * CRC_SEG) void k_crc_count(const CbInfo* __restrict__ cbi, int C,
                                                            uint32_t* const* __restrict__ dec,
                                                            const int* __restrict__ KW, int B,
                                                            const uint32_t* __restrict__ pw, int PW, int n_bits,
                                                            int SW, CrcSeg xs, uint32_t* __restrict__ frame_err,
                                                            uint32_t* __restrict__ frame_crc,
                                                            uint8_t* __restrict__ cap_bits, int b0,
                                                            const uint64_t* __restrict__ fid, uint64_t seed) {
  __shared__ uint32_t T[1024];
  __shared__ uint32_t part[3][CRC_SEG][64];
  __shared__ int s_off[CRC_MAXC], s_end[CRC_MAXC], s_F[CRC_MAXC], s_kw[CRC_MAXC];
  __shared__ const uint32_t* s_dec[CRC_MAXC];
  crc24_slice4_fill(T, (uint32_t)CRC24A_POLY);
  if (threadIdx.x < C) {
    const CbInfo ci = cbi[threadIdx.x];
    s_off[threadIdx.x] = ci.off;
    s_end[threadIdx.x] = ci.off + ci.info;
    s_F[threadIdx.x] = ci.F;
    s_kw[threadIdx.x] = KW[threadIdx.x];
    s_dec[threadIdx.x] = dec[threadIdx.x];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, seg = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // scalar
  const int b = b0 + blockIdx.x * 64 + lane;
  const bool act = b < B;
  const int bb = act ? b : b0;
  const int g = bb >> 6, gl = bb & 63;
  // the transmitted words: drawn again from their Philox counters (k_payload's
  // draws, a pure function of (seed, frame id, word)) when fid is given --
  // the frame-major payload rows would be fetched line by line per lane --
  // or read back from pw (injected payloads)
  const uint32_t* tx = pw + (size_t)bb * PW;
  const uint64_t fr = fid ? fid[bb] : 0ull;
  u32x4 rv{0u, 0u, 0u, 0u};
  int rvg = -1;
  const int Btb = n_bits + 24;
  const int nw = (Btb + 31) >> 5;
  const int w0 = seg * SW, w1 = min(nw, w0 + SW);
  uint32_t crc = 0, err = 0, rx_crc = 0;
  int r = 0, off = s_off[0], end = s_end[0], F = s_F[0], kw = s_kw[0];
  const uint32_t* base = s_dec[0] + (size_t)g * kw * 64 + gl;
  for (int w = w0; w < w1; ++w) {
    // assemble TB word w (bits 32w .. 32w+31) from the decoded code blocks
    uint32_t word = 0;
    int got = 0;
    const int want = min(32, Btb - 32 * w);
    while (got < want) {
      const int j = 32 * w + got;  // TB position
      while (j >= end) {
        ++r;
        off = s_off[r]; end = s_end[r]; F = s_F[r]; kw = s_kw[r];
        base = s_dec[r] + (size_t)g * kw * 64 + gl;
      }
      const int avail = min(want - got, end - j);
      const uint32_t v = get32s(base, 64, (int64_t)F + (j - off), kw);
      const uint32_t m = avail >= 32 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> avail);
      word |= (v & m) >> got;
      got += avail;
    }
    // CRC over data bits [0, n_bits), MSB-first
    const int dbits = min(32, max(0, n_bits - 32 * w));
    if (dbits == 32) {
      crc = crc24_slice4(T, crc, word);
    } else {
      int k = 0;
      for (; k + 8 <= dbits; k += 8) {
        const uint32_t byte = (word >> (24 - k)) & 0xFFu;
        crc = ((crc << 8) & 0xFFFFFFu) ^ T[((crc >> 16) ^ byte) & 0xFFu];
      }
      for (; k < dbits; ++k) {
        const uint32_t bit = (word >> (31 - k)) & 1u;
        const uint32_t msb = (crc >> 23) & 1u;
        crc = (crc << 1) & 0xFFFFFFu;
        if (msb ^ bit) crc ^= (uint32_t)CRC24A_POLY;
      }
      // received CRC bits [n_bits, n_bits+24), placed at their CRC bit position
      for (int q = max(0, n_bits - 32 * w); q < want; ++q)
        rx_crc |= ((word >> (31 - q)) & 1u) << (23 - (32 * w + q - n_bits));
    }
    if (dbits > 0) {
      const uint32_t m = dbits >= 32 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> dbits);
      uint32_t t;
      if (fid) {
        if ((w >> 2) != rvg) {
          rvg = w >> 2;
          rv = rng4(seed, fr, RNG_STREAM_BITS, (uint32_t)rvg);
        }
        t = (w & 3) == 0 ? rv.x : (w & 3) == 1 ? rv.y : (w & 3) == 2 ? rv.z : rv.w;
      } else {
        t = tx[w];
      }
      err += __popc((word ^ t) & m);
    }
    if (cap_bits && act) {
      for (int q = 0; q < dbits; ++q) cap_bits[(size_t)b * n_bits + 32 * w + q] = (word >> (31 - q)) & 1u;
    }
  }
  part[0][seg][lane] = gf24_mul(crc, xs.x[seg], (uint32_t)CRC24A_POLY);
  part[1][seg][lane] = err;
  part[2][seg][lane] = rx_crc;
  __syncthreads();
  if (seg == 0 && act) {
    uint32_t c = 0, e = 0, rc = 0;
#pragma unroll
    for (int s2 = 0; s2 < CRC_SEG; ++s2) {
      c ^= part[0][s2][lane];
      e += part[1][s2][lane];
      rc |= part[2][s2][lane];
    }
    frame_err[b] = e;
    frame_crc[b] = (c == rc) ? 1u : 0u;
  }
}

int launch_crc_count(hipStream_t s, const CbInfo* cbi_dev, int C, uint32_t* const* dec, const int* KW, int B,
                     const uint32_t* pw, int PW, int n_bits, uint32_t* frame_err, uint32_t* frame_crc,
                     uint8_t* cap_bits, int b0, const uint64_t* fid, uint64_t seed) {
  if (b0 < 0 || b0 >= B || n_bits < 0 || C < 1 || C > CRC_MAXC) return (int)hipErrorInvalidValue;
  const int nw = (n_bits + 24 + 31) >> 5;
  const int SW = (nw + CRC_SEG - 1) / CRC_SEG;
  CrcSeg xs{};
  for (int sg = 0; sg < CRC_SEG; ++sg) {
    const int end = std::min(32 * (sg + 1) * SW, n_bits);   // data bits up to the segment's end
    xs.x[sg] = gf24_xpow((uint64_t)(n_bits - std::max(end, 0)), (uint32_t)CRC24A_POLY);
  }
  hipLaunchKernelGGL(k_crc_count, dim3((B - b0 + 63) / 64), dim3(64 * CRC_SEG), 0, s, cbi_dev, C, dec, KW, B, pw, PW,
                     n_bits, SW, xs, frame_err, frame_crc, cap_bits, b0, fid, seed);
  return (int)hipGetLastError();
}

}  // namespace lte
