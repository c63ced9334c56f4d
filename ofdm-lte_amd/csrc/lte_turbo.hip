// Channel-coding kernels around the turbo decoder (lte_decoder.hip) for
// gfx950: RX rate dematch into the decoder's row layout (with the soft
// demapper fused in), TX code-block construction + turbo encoding, and the
// RX CRC-24A / desegmentation / bit-error count.
#include "lte_common.h"
#include "lte_internal.h"
#include "lte_dev.h"

namespace lte {

constexpr int RS = TURBO_RS;   // decoder row stride (elements): 64 lanes

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
template <class R>
__device__ __forceinline__ void dm_store(R* dst, R v, bool add) {
  if (add) *dst = *dst + (R)0.5 * v;
  else *dst = (R)0.5 * ((R)0 + v);
}

template <class R>
__global__ __launch_bounds__(256) void k_dematch(const R* __restrict__ llr, int T, int B,
                                                 const int32_t* __restrict__ rx_map, int add,
                                                 R* const* __restrict__ blk, const int64_t* __restrict__ rows,
                                                 int g0) {
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
    dm_store(&blk[r][((size_t)g * rows[r] + row) * RS + f], tile[f][c], add != 0);
  }
}

template <class R>
int launch_dematch(hipStream_t s, const R* llr, int T, int B, const int32_t* rx_map, int n_layers, R* const* blk,
                   const int64_t* rows, int g0) {
  const int G = (B + 63) / 64 - g0;   // groups g0 .. ceil(B/64)-1
  if (G < 1 || G > 65535 || n_layers < 1) return (int)hipErrorInvalidValue;
  for (int k = 0; k < n_layers; ++k) {
    hipLaunchKernelGGL(k_dematch<R>, dim3((T + DM_CH - 1) / DM_CH, G), dim3(256), 0, s, llr, T, B,
                       rx_map + (size_t)k * T, k > 0 ? 1 : 0, blk, rows, g0);
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
template <class R> constexpr int dz_re() { return sizeof(R) == 8 ? 8 : 16; }
template <class R, int BPS>
__global__ __launch_bounds__(256) void k_dematch_zn(const cx<R>* __restrict__ z, const R* __restrict__ nv, int n_re,
                                                    int nd, int n_nv, int B, const int32_t* __restrict__ rx_map,
                                                    int add,
                                                    R* const* __restrict__ blk, const int64_t* __restrict__ rows,
                                                    int g0) {
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
    zv[k] = ok ? z[i] : mkc((R)0, (R)0);
    nvv[k] = ok ? nv[(size_t)b * n_nv + (l / 14) * nd + j] : (R)1;
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
    dm_store(&blk[r][((size_t)g * rows[r] + row) * RS + f], tile[f][c], add != 0);
  }
}

template <class R>
int launch_dematch_zn(hipStream_t s, const cx<R>* z, const R* nv, int n_re, int nd, int bps, int B,
                      const int32_t* rx_map, int n_layers, R* const* blk, const int64_t* rows, int g0) {
  const int G = (B + 63) / 64 - g0;
  if (G < 1 || G > 65535 || (bps != 4 && bps != 6) || n_layers < 1 || nd < 1) return (int)hipErrorInvalidValue;
  const int n_nv = ((n_re / nd + 13) / 14) * nd;   // groups x data subcarriers per frame
  constexpr int DZ = dz_re<R>();
  const dim3 grid((n_re + DZ - 1) / DZ, G);
  const int T = n_re * bps;
  for (int k = 0; k < n_layers; ++k) {
    const int32_t* mp = rx_map + (size_t)k * T;
    if (bps == 4)
      hipLaunchKernelGGL((k_dematch_zn<R, 4>), grid, dim3(256), 0, s, z, nv, n_re, nd, n_nv, B, mp, k > 0 ? 1 : 0,
                         blk, rows, g0);
    else
      hipLaunchKernelGGL((k_dematch_zn<R, 6>), grid, dim3(256), 0, s, z, nv, n_re, nd, n_nv, B, mp, k > 0 ? 1 : 0,
                         blk, rows, g0);
    const int e = (int)hipGetLastError();
    if (e) return e;
  }
  return 0;
}

template int launch_dematch<float>(hipStream_t, const float*, int, int, const int32_t*, int, float* const*,
                                   const int64_t*, int);
template int launch_dematch<double>(hipStream_t, const double*, int, int, const int32_t*, int, double* const*,
                                    const int64_t*, int);
template int launch_dematch_zn<float>(hipStream_t, const float2*, const float*, int, int, int, int, const int32_t*,
                                      int, float* const*, const int64_t*, int);
template int launch_dematch_zn<double>(hipStream_t, const double2*, const double*, int, int, int, int,
                                       const int32_t*, int, double* const*, const int64_t*, int);

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

// TX coding in two kernels, one lane = one (CB slot, frame); lanes of a wave
// are 64 consecutive frames of one CB slot, so they share K and the QPP
// permutation.
//  k_encode   CB construction (segmentation.py:212-247 + CRC-24B crc.py:
//             162-184, a byte-table step per 8 bits) + encoder 1.  TB words
//             stream in through a two-word window (next word prefetched).  The
//             code block is written to a scratch as [wave][word][lane]
//             (coalesced rows).  No big LDS: occupancy is set by VGPRs.
//  k_encode2  encoder 2 on the QPP-interleaved block (turbo_encoder.py:
//             213-313): the wave copies its 64 code blocks into LDS (48 KB at
//             K = 6144, [word][lane]) and gathers from there -- pi(i) is
//             wave-uniform, so each gather is one conflict-free LDS read.
constexpr int ENC_WG = 256;
constexpr int ENC_CH = 16;   // output words per bunched store (k_encode)
constexpr int ENC2_CH = 8;   // (k_encode2)
__global__ __launch_bounds__(ENC_WG) void k_encode(const uint32_t* __restrict__ pw, int PW, int KWmax,
                                                   uint32_t* __restrict__ enc, int EW,
                                                   const CbInfo* __restrict__ cbi, int C, int B,
                                                   uint32_t* __restrict__ cw_scratch) {
  __shared__ uint32_t crc_t[256];
  for (int i = threadIdx.x; i < 256; i += ENC_WG) crc_t[i] = crc24_table_entry(i, 0x800063u);   // CRC-24B
  __syncthreads();
  // lanes = frames of ONE code-block slot: frame groups are padded to 64 per
  // slot (Bp), so K, F, f1, f2 are wave-uniform (scalar registers)
  const int Bp = (B + 63) & ~63;
  const int gid = blockIdx.x * ENC_WG + threadIdx.x;
  const int r = __builtin_amdgcn_readfirstlane(gid / Bp), b = gid % Bp;
  if (r >= C || b >= B) return;       // no barriers below: early exit is safe
  const CbInfo ci = cbi[r];
  const int K = ci.K, F = ci.F;
  const uint32_t* tb = pw + (size_t)b * PW;
  uint32_t* cw = cw_scratch + (size_t)(gid >> 6) * KWmax * 64 + (gid & 63);   // word w at cw[w * 64]
  uint32_t* e = enc + ((size_t)b * C + r) * 3 * EW;
  const int Kd = ci.crc ? K - 24 : K;   // every LTE K (and so Kd) is a multiple of 8
  const int KWf = K >> 5;               // whole 32-bit words of the code block
  uint32_t crc = 0, s0 = 0, s1 = 0, s2 = 0;
  // CB bit p in [F, Kd) is TB bit (off - F + p): the 32 bits of word w are a
  // fixed-offset window over TB words i00 + w, i00 + w + 1
  const int64_t base = (int64_t)ci.off - F;
  const int64_t i00 = base >> 5;      // arithmetic shift: floor for negative base
  const int o = (int)(base & 31);
  auto ldw = [&](int64_t i) -> uint32_t { return (i >= 0 && i < PW) ? tb[i] : 0u; };
  uint32_t wa = ldw(i00), wb = ldw(i00 + 1);
  // Whole output words are kept in registers and stored ENC_CH at a time: each
  // lane then completes its 64-B line pieces back to back instead of one word
  // per loop trip (lanes are 64 different frames, so a store instruction
  // touches 64 lines; spread over the loop, L2 evicted them half-written).
  uint32_t pf = 0, pq = 0;              // the last, partial word (K % 32 bits), if any
  int pnb = 0;
  for (int wc = 0; wc * 32 < K; wc += ENC_CH) {
    uint32_t fb[ENC_CH], qb[ENC_CH];
#pragma unroll
    for (int i = 0; i < ENC_CH; ++i) {
      const int w = wc + i;
      fb[i] = qb[i] = 0u;
      if (w * 32 >= K) continue;
      const uint32_t wn = ldw(i00 + w + 2);   // next window word, in flight during this one
      const int p0 = w * 32, nb = min(32, K - p0);
      uint32_t t = o ? ((wa << o) | (wb >> (32 - o))) : wa;
      if (p0 < F) t &= (F - p0 >= 32) ? 0u : (0xFFFFFFFFu >> (F - p0));   // filler bits are 0
      uint32_t u = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int p = p0 + 8 * k;
        if (8 * k < nb) {
          uint32_t byte;
          if (p < Kd) {
            byte = (t >> (24 - 8 * k)) & 0xFFu;
            if (ci.crc) crc = ((crc << 8) & 0xFFFFFFu) ^ crc_t[((crc >> 16) ^ byte) & 0xFFu];
          } else {
            byte = (crc >> (16 - (p - Kd))) & 0xFFu;   // CRC-24B bits after the data
          }
          u |= byte << (24 - 8 * k);
        }
      }
      cw[w * 64] = u;                      // left-aligned
      uint32_t f;
      const uint32_t q = rsc_word(u, nb, s0, s1, s2, &f);
      if (nb == 32) {
        fb[i] = f;
        qb[i] = q;
      } else {
        pf = f;
        pq = q;
        pnb = nb;
      }
      wa = wb;
      wb = wn;
    }
#pragma unroll
    for (int i = 0; i < ENC_CH; ++i)
      if (wc + i < KWf) e[wc + i] = fb[i];
#pragma unroll
    for (int i = 0; i < ENC_CH; ++i)
      if (wc + i < KWf) e[EW + wc + i] = qb[i];
  }
  BitWriter w0{e + KWf, 0, 0}, w1{e + EW + KWf, 0, 0};
  if (pnb) {
    w0.put(pf >> (32 - pnb), pnb);
    w1.put(pq >> (32 - pnb), pnb);
  }
  for (int t = 0; t < 3; ++t) {  // trellis termination, encoder 1
    const uint32_t v = rsc_tail(s0, s1, s2);
    w0.put(v & 1u, 1);
    w1.put(v >> 1, 1);
  }
  w0.flush();                    // d0[K+3..K+5] (encoder 2's tail) is OR-ed in by k_encode2
  w1.flush();
}

__global__ __launch_bounds__(64) void k_encode2(int KWmax, uint32_t* __restrict__ enc, int EW,
                                                const CbInfo* __restrict__ cbi, int C, int B,
                                                const uint32_t* __restrict__ cw_scratch) {
  extern __shared__ uint32_t cwl[];   // [KWmax][64]
  const int Bp = (B + 63) & ~63;     // frame groups padded per slot (see k_encode)
  const int gid = blockIdx.x * 64 + threadIdx.x;
  const int lane = threadIdx.x;
  const int r = __builtin_amdgcn_readfirstlane(gid / Bp), b = gid % Bp;
  if (r >= C || b >= B) return;       // no barriers: each lane reads back only its own column
  const CbInfo ci = cbi[r];
  const int K = ci.K, KW = (K + 31) >> 5;
  const uint32_t* cw = cw_scratch + (size_t)blockIdx.x * KWmax * 64 + lane;
  for (int w = 0; w < KW; ++w) cwl[w * 64 + lane] = cw[w * 64];
  uint32_t* e = enc + ((size_t)b * C + r) * 3 * EW;
  const int KWf = K >> 5;
  uint32_t s0 = 0, s1 = 0, s2 = 0;
  int pi = 0, d = (ci.f1 + ci.f2) % K;
  const int tf2 = (2 * ci.f2) % K;
  uint32_t pq = 0;                      // the last, partial parity word (K % 32 bits), if any
  int pnb = 0;
  for (int wc = 0; wc < KW; wc += ENC2_CH) {   // whole words stored ENC2_CH at a time (see k_encode)
    uint32_t qb[ENC2_CH];
#pragma unroll
    for (int j = 0; j < ENC2_CH; ++j) {
      const int w = wc + j;
      qb[j] = 0u;
      if (w >= KW) continue;
      const int nb = min(32, K - w * 32);
      uint32_t u = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {        // 16 gathers in flight together
        uint32_t v[16];
        int sh[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          v[i] = cwl[(pi >> 5) * 64 + lane];
          sh[i] = pi & 31;
          int pn = pi + d, dn = d + tf2;
          pn -= pn >= K ? K : 0;
          dn -= dn >= K ? K : 0;
          const bool adv = 16 * h + i < nb;
          pi = adv ? pn : pi;
          d = adv ? dn : d;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) u |= ((v[i] << sh[i]) >> 31) << (31 - 16 * h - i);
      }
      uint32_t f;
      const uint32_t q = rsc_word(u, nb, s0, s1, s2, &f);
      if (nb == 32) {
        qb[j] = q;
      } else {
        pq = q;
        pnb = nb;
      }
    }
#pragma unroll
    for (int j = 0; j < ENC2_CH; ++j)
      if (wc + j < KWf) e[2 * EW + wc + j] = qb[j];
  }
  BitWriter w2{e + 2 * EW + KWf, 0, 0};
  if (pnb) w2.put(pq >> (32 - pnb), pnb);
  for (int t = 0; t < 3; ++t) {
    const uint32_t v = rsc_tail(s0, s1, s2);
    const int pos = K + 3 + t;   // sys2 tail -> d0[K+3..K+5]
    if (v & 1u) e[pos >> 5] |= 1u << (31 - (pos & 31));
    w2.put(v >> 1, 1);
  }
  w2.flush();
}

size_t encode_scratch_words(int KWmax, int C, int B) { return (size_t)C * ((B + 63) / 64) * KWmax * 64; }

int launch_encode(hipStream_t s, const uint32_t* pw, int PW, int KWmax, uint32_t* enc, int EW,
                  const CbInfo* cbi_dev, int C, int B, uint32_t* cw_scratch) {
  const int64_t n = (int64_t)C * ((B + 63) & ~63);   // lanes: frames padded to 64 per CB slot
  if (n > 0x7FFFFFFF || !cw_scratch) return (int)hipErrorInvalidValue;
  const size_t shm = (size_t)KWmax * 64 * sizeof(uint32_t);
  if (shm > 65536) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_encode, dim3((unsigned)((n + ENC_WG - 1) / ENC_WG)), dim3(ENC_WG), 0, s, pw, PW, KWmax, enc,
                     EW, cbi_dev, C, B, cw_scratch);
  hipLaunchKernelGGL(k_encode2, dim3((unsigned)((n + 63) / 64)), dim3(64), shm, s, KWmax, enc, EW, cbi_dev, C, B,
                     cw_scratch);
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
// over its data bits; the frame's CRC is sum_s crc_s * x^(data bits after
// segment s) mod P (lte_common.h CRC-24 algebra, multipliers from the host),
// formed by wave 0 from the per-wave results parked in LDS.
constexpr int CRC_SEG = 8;
struct CrcSeg { uint32_t x[CRC_SEG]; };

__global__ __launch_bounds__(64 * CRC_SEG) void k_crc_count(const CbInfo* __restrict__ cbi, int C,
                                                            uint32_t* const* __restrict__ dec,
                                                            const int* __restrict__ KW, int B,
                                                            const uint32_t* __restrict__ pw, int PW, int n_bits,
                                                            int SW, CrcSeg xs, uint32_t* __restrict__ frame_err,
                                                            uint32_t* __restrict__ frame_crc,
                                                            uint8_t* __restrict__ cap_bits, int b0) {
  __shared__ uint32_t T[256];
  __shared__ uint32_t part[3][CRC_SEG][64];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) T[i] = crc24_table_entry(i, (uint32_t)CRC24A_POLY);
  __syncthreads();
  const int lane = threadIdx.x & 63, seg = threadIdx.x >> 6;
  const int b = b0 + blockIdx.x * 64 + lane;
  const bool act = b < B;
  const int bb = act ? b : b0;
  const int g = bb >> 6, gl = bb & 63;
  const uint32_t* tx = pw + (size_t)bb * PW;
  const int Btb = n_bits + 24;
  const int nw = (Btb + 31) >> 5;
  const int w0 = seg * SW, w1 = min(nw, w0 + SW);
  uint32_t crc = 0, err = 0, rx_crc = 0;
  int r = 0;
  for (int w = w0; w < w1; ++w) {
    // assemble TB word w (bits 32w .. 32w+31) from the decoded code blocks
    uint32_t word = 0;
    int got = 0;
    const int want = min(32, Btb - 32 * w);
    while (got < want) {
      const int j = 32 * w + got;  // TB position
      while (j >= cbi[r].off + cbi[r].info) ++r;
      const CbInfo ci = cbi[r];
      const int avail = min(want - got, ci.off + ci.info - j);
      const int64_t pcb = (int64_t)ci.F + (j - ci.off);
      const uint32_t* base = dec[r] + (size_t)g * KW[r] * 64 + gl;
      const uint32_t v = get32s(base, 64, pcb, KW[r]);
      const uint32_t m = avail >= 32 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> avail);
      word |= (v & m) >> got;
      got += avail;
    }
    // CRC over data bits [0, n_bits), byte-wise table (MSB-first)
    const int dbits = min(32, max(0, n_bits - 32 * w));
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
    if (dbits > 0) {
      const uint32_t m = dbits >= 32 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> dbits);
      err += __popc((word ^ tx[w]) & m);
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
                     uint8_t* cap_bits, int b0) {
  if (b0 < 0 || b0 >= B || n_bits < 0) return (int)hipErrorInvalidValue;
  const int nw = (n_bits + 24 + 31) >> 5;
  const int SW = (nw + CRC_SEG - 1) / CRC_SEG;
  CrcSeg xs{};
  for (int sg = 0; sg < CRC_SEG; ++sg) {
    const int end = std::min(32 * (sg + 1) * SW, n_bits);   // data bits up to the segment's end
    xs.x[sg] = gf24_xpow((uint64_t)(n_bits - std::max(end, 0)), (uint32_t)CRC24A_POLY);
  }
  hipLaunchKernelGGL(k_crc_count, dim3((B - b0 + 63) / 64), dim3(64 * CRC_SEG), 0, s, cbi_dev, C, dec, KW, B, pw, PW,
                     n_bits, SW, xs, frame_err, frame_crc, cap_bits, b0);
  return (int)hipGetLastError();
}

}  // namespace lte
