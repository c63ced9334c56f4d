// Front-end kernels of the LTE link chain for gfx950: payload/CRC, OFDM TX
// (QAM map + resource map + IFFT + CP), multipath Rayleigh + AWGN channel,
// RX (CP removal + FFT, CRS LS estimation + interpolation, ZF / MRC, hard
// decision or soft demap).  All HBM-bound: every kernel streams its frame
// data once, coalesced, with per-symbol FFTs staged in LDS.
#include "lte_common.h"
#include "lte_internal.h"
#include "lte_dev.h"
#include <cstdlib>

namespace lte {

constexpr int WG = 256;

// ---------------------------------------------------------------------------
// Payload bits (+ CRC-24, crc.py:89-134: CRC-24A attach crc.py:212-233, or
// CRC-24B for the stage entry, crc.py:162-184): one wave per frame.  The frame's
// PW words are cut into 128-bit groups (Philox counter g = group g, words
// 4g..4g+3: the draws of the one-lane-per-frame kernel this replaces), and lane
// l owns the KG consecutive groups [l KG, (l+1) KG): it draws and stores them
// and runs the CRC register over them (slice-by-4 tables, starting from 0).
// The 64 chunk CRCs are combined by the linearity of the CRC (lte_common.h): a
// 6-level tree with the multipliers x^(128 KG 2^s), then x^(-pad) for the zero
// bits the chunks hold past n_bits (products through per-block nibble tables).
// Waves loop over frames so the tables are built once per block.
// crc = the polynomial without its x^24 term (0: no CRC); CrcTree is formed on
// the host (crc_tree).
struct CrcTree {
  uint32_t poly, corr;   // corr = x^-(64 KG 128 - n_bits) mod P
  uint32_t xl[6];        // x^(128 KG 2^s) mod P
};

static CrcTree crc_tree(uint32_t poly, int KG, int n_bits) {
  CrcTree t{};
  t.poly = poly;
  if (!poly) return t;
  t.corr = gf24_xpow((uint64_t)64 * KG * 128 - (uint64_t)n_bits, poly, true);
  for (int s = 0; s < 6; ++s) t.xl[s] = gf24_xpow((uint64_t)128 * KG << s, poly);
  return t;
}

// c * X_k mod P through nibble tables NT[k][j][v] = (v x^(4j)) X_k mod P
__device__ __forceinline__ uint32_t gf24_mul_nt(const uint32_t* NT, int k, uint32_t c) {
  const uint32_t* t = NT + k * 96;
  uint32_t r = 0u;
#pragma unroll
  for (int j = 0; j < 6; ++j) r ^= t[j * 16 + ((c >> (4 * j)) & 15u)];
  return r;
}

__global__ __launch_bounds__(WG) void k_payload(uint32_t* __restrict__ pw, int PW, int n_bits, int KG, CrcTree ct,
                                                const uint64_t* __restrict__ fid, uint64_t seed, int B,
                                                const uint32_t* __restrict__ inj, int64_t inj_stride) {
  __shared__ uint32_t T[1024];      // slice-by-4 CRC tables
  __shared__ uint32_t NT[7 * 96];   // nibble tables of the 6 tree multipliers and x^-pad
  const uint32_t poly = ct.poly;
  if (poly) {
    crc24_slice4_fill(T, poly);
    for (int i = threadIdx.x; i < 7 * 96; i += blockDim.x) {
      const int k = i / 96, j = (i % 96) >> 4, v = i & 15;
      NT[i] = gf24_mul((uint32_t)v << (4 * j), k < 6 ? ct.xl[k] : ct.corr, poly);
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int nwd = (n_bits + 31) >> 5;
  // the (at most two) words holding the CRC bits [n_bits, n_bits + 24) are
  // stored after the CRC is known, by the lane that drew them
  const int c0 = n_bits >> 5, c1 = (n_bits + 23) >> 5;
  for (int b = blockIdx.x * (WG / 64) + (threadIdx.x >> 6); b < B; b += gridDim.x * (WG / 64)) {   // whole waves
    uint32_t* w = pw + (size_t)b * PW;
    uint32_t h0 = 0u, h1 = 0u;
    const uint64_t f = inj ? 0ull : fid[b];
    uint32_t c = 0u;
    if (!poly) {   // no CRC: lane l draws groups l, l + 64, ... (the same draws; each store instruction
                   // of the wave then covers one contiguous 1 KB span instead of 64 chunks KG x 16 B apart)
      for (int g = lane; 4 * g < nwd; g += 64) {
        u32x4 rv{0u, 0u, 0u, 0u};
        if (!inj) rv = rng4(seed, f, RNG_STREAM_BITS, (uint32_t)g);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = 4 * g + q;
          if (i >= nwd) break;
          uint32_t v = inj ? inj[(size_t)b * inj_stride + i] : (q == 0 ? rv.x : q == 1 ? rv.y : q == 2 ? rv.z : rv.w);
          const int rem = n_bits - 32 * i;
          if (rem < 32) v &= ~(0xFFFFFFFFu >> rem);
          w[i] = v;
        }
      }
      for (int i = nwd + lane; i < PW; i += 64) w[i] = 0u;   // words past the bits (the chunked loop stored zeros)
      continue;
    }
    for (int k = 0; k < KG; ++k) {
      const int g = lane * KG + k;
      u32x4 rv{0u, 0u, 0u, 0u};
      if (!inj && 4 * g < nwd) rv = rng4(seed, f, RNG_STREAM_BITS, (uint32_t)g);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = 4 * g + q;
        uint32_t v = 0u;
        if (i < nwd) {
          v = inj ? inj[(size_t)b * inj_stride + i] : (q == 0 ? rv.x : q == 1 ? rv.y : q == 2 ? rv.z : rv.w);
          const int rem = n_bits - 32 * i;
          if (rem < 32) v &= ~(0xFFFFFFFFu >> rem);
        }
        if (poly) {
          c = crc24_slice4(T, c, v);
          if (i == c0) { h0 = v; continue; }
          if (i == c1) { h1 = v; continue; }
        }
        if (i < PW) w[i] = v;
      }
    }
    if (poly) {
      // lane l's chunk sits 64 - 1 - l chunks before the end: merge neighbours,
      // the left one shifted past the right one's 128 KG 2^s bits
#pragma unroll
      for (int s = 0; s < 6; ++s) {
        const uint32_t r = __shfl_down(c, 1 << s);
        c = gf24_mul_nt(NT, s, c) ^ r;
      }
      const uint32_t crc = gf24_mul_nt(NT, 6, __shfl(c, 0));
      const uint32_t L = crc << 8, o = (uint32_t)(n_bits & 31);   // CRC left-aligned, MSB-first at bit n_bits
      if (lane == ((c0 >> 2) / KG) && c0 < PW) w[c0] = h0 | (L >> o);
      if (c1 != c0 && lane == ((c1 >> 2) / KG) && c1 < PW) w[c1] = h1 | (L << (32 - o));
    }
  }
}

int launch_payload(hipStream_t s, uint32_t* pw, int PW, int n_bits, int crc, const uint64_t* fid, uint64_t seed,
                   int B, const uint32_t* inj, int64_t inj_stride) {
  const uint32_t poly = (uint32_t)crc & 0xFFFFFFu;
  if (PW < 1 || n_bits < 0 || (poly && (!(poly & 1u) || PW * 32 < n_bits + 24))) return (int)hipErrorInvalidValue;
  const int KG = ((PW + 3) / 4 + 63) / 64;   // 128-bit groups per lane
  const int fpb = WG / 64;
  const int blocks = std::max(1, std::min((B + fpb - 1) / fpb, 1024));   // waves loop over frames (tables amortised)
  hipLaunchKernelGGL(k_payload, dim3(blocks), dim3(WG), 0, s, pw, PW, n_bits, KG,
                     crc_tree(poly, KG, n_bits), fid, seed, B, inj, inj_stride);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Every SISO / SIMO signal kernel below is templated on the arithmetic type R
// (double: the default, the reference's float64 / complex128; float: the
// opt-in fast mode) with V = cx<R> its complex type.  Dynamic LDS is declared
// once (16-B aligned) and viewed as V.
template <class V>
__device__ __forceinline__ V* dyn_lds() {
  extern __shared__ double2 lte_dyn_lds[];
  return reinterpret_cast<V*>(lte_dyn_lds);
}

// Fused static-tap channel for one OFDM symbol held in LDS (TxChannelT): y[m] =
// sum_p c_p x[m - d_p] over the CP-extended symbol, whose sample j is
// buf[j < cp ? N - cp + j : j - cp] (rayleighchannel.py:44-58; for m >=
// max_delay every delayed tap stays inside the symbol); stores m >= cp only
// and sums |y|^2 over m >= max_delay per slot in a fixed order.  Called by
// every thread of the block.  f32 folds the output scale into the taps; f64
// receives the symbol already scaled by the IFFT's last pass (x = ifft *
// sqrt(N) as the reference forms it) and applies the taps (gain * fading) * x
// in the reference's order.
//
// TV, time-varying taps (ch.tcoef, fD != 0): tap p at sample m of the symbol is
// the Horner value of the symbol's Taylor set at d = m - (S - 1) / 2
// (jakes_symbol_sets, as the multi-antenna links form it).  A wave belongs to
// one slot (T >= 64), so the set's address is wave-uniform (scalar loads);
// paths outer, the thread's samples (at most TXCH_MAXS) inner.
constexpr int TXCH_MAXS = 10;   // samples per thread per symbol: S <= 1.25 N (cp <= N / 4), T = N / 8
// NP > 0: the path count as a compile-time constant (static taps), so only NP
// taps are formed (with a runtime count the unrolled TXCH_MAXP taps were all
// computed and masked by selects).  float64 only: in float32 the compiler
// contracts the tap sums into FMAs differently once the selects are gone, and
// k_ofdm_txf must equal the per-symbol k_ofdm_tx<.., CH> bit for bit.
template <class R, bool TV, int NP = 0>
__device__ __forceinline__ void tx_channel(cx<R>* buf, const Grid& g, const TxChannelT<R>& ch, int b, int l, int slot,
                                           int tid, int T, bool active, R sc) {
  using V = cx<R>;
  __shared__ R red[2 * WG / 64];   // (k_ofdm_txf<.., SP = 2>: 512 threads)
  constexpr bool F64 = sizeof(R) == 8;
  const int N = g.N, cp = g.cp, S = N + cp, D = ch.max_delay;
  if (active && D > 0) {   // the TX samples x at both ends of the symbol (every RX's taps read them)
    V* xh = ch.xh + ((size_t)b * g.n_sym + l) * 2 * D;
    for (int i = tid; i < 2 * D; i += T) {
      const int j = i < D ? i : S - 2 * D + i;
      const V v = buf[(j - cp) & (N - 1)];
      xh[i] = F64 ? v : cscale(v, sc);
    }
  }
  if (active && ch.x_out) {   // the symbol for the receiver's taps (one stream instead of num_rx)
    V* xo = ch.x_out + ((size_t)b * g.n_sym + l) * N;
    for (int k = tid; k < N; k += T) xo[k] = buf[k];
  }
  // SIMO: each RX its own taps, stream and power partial (transmit_simo,
  // core/ofdm_core.py:361-412); the symbol in LDS is read once per RX
  for (int r = 0; r < ch.num_rx; ++r) {
    const size_t br = (size_t)b * ch.num_rx + r;
    R pw = (R)0;
    if (TV && active) {
      constexpr int NCF = mimo_ncf<R>();
      const int bu = __builtin_amdgcn_readfirstlane(b), lu = __builtin_amdgcn_readfirstlane(l);
      const V* tc = ch.tcoef + (((size_t)bu * ch.num_rx + r) * ch.n_paths * g.n_sym + lu) * NCF;
      const R dc = (R)0.5 * (R)(S - 1);
      V v[TXCH_MAXS];
#pragma unroll
      for (int i = 0; i < TXCH_MAXS; ++i) v[i] = mkc((R)0, (R)0);
      for (int p = 0; p < ch.n_paths; ++p) {
        const V* c = tc + (size_t)p * g.n_sym * NCF;
        V cc[NCF];
#pragma unroll
        for (int k = 0; k < NCF; ++k) cc[k] = F64 ? c[k] : cscale(c[k], sc);
        const int off = ch.delays[p] + cp;
#pragma unroll
        for (int i = 0; i < TXCH_MAXS; ++i) {
          const int m = D + tid + i * T;
          if (m < S) {
            const R d = (R)m - dc;
            V h = cc[NCF - 1];
#pragma unroll
            for (int k = NCF - 2; k >= 0; --k) h = mkc(h.x * d + cc[k].x, h.y * d + cc[k].y);
            v[i] = cadd(v[i], cmul(h, buf[(m - off) & (N - 1)]));
          }
        }
      }
      V* yo = ch.y + br * g.L + (size_t)l * S;
#pragma unroll
      for (int i = 0; i < TXCH_MAXS; ++i) {
        const int m = D + tid + i * T;
        if (m < S) {
          if (m >= cp) yo[m] = v[i];
          pw += v[i].x * v[i].x + v[i].y * v[i].y;
        }
      }
    } else if (!TV && active) {
      // sample j of the CP-extended symbol is buf[(j - cp) mod N] (N a power of 2)
      constexpr int PM = NP ? NP : TXCH_MAXP;
      const int np = NP ? NP : ch.n_paths;
      V cf[PM];
      int off[PM];
#pragma unroll
      for (int p = 0; p < PM; ++p) {
        const V c = p < np ? ch.coef[br * np + p] : mkc((R)0, (R)0);
        cf[p] = F64 ? c : cscale(c, sc);
        off[p] = ch.delays[p] + cp;
      }
      V* yo = ch.y + br * g.L + (size_t)l * S;
      for (int m = D + tid; m < S; m += T) {
        V v = mkc((R)0, (R)0);
#pragma unroll
        for (int p = 0; p < PM; ++p)
          if (p < np) v = cadd(v, cmul(cf[p], buf[(m - off[p]) & (N - 1)]));
        if (m >= cp && !ch.x_out) yo[m] = v;
        pw += v.x * v.x + v.y * v.y;
      }
    }
    // per-slot sum in a fixed order: T >= 64 threads = T / 64 whole waves per slot
    for (int o = 32; o > 0; o >>= 1) pw += __shfl_xor(pw, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = pw;
    __syncthreads();
    if (active && tid == 0) {
      const int wps = T >> 6;
      R t = (R)0;
      for (int w = 0; w < wps; ++w) t += red[slot * wps + w];
      ch.pow_part[br * g.n_sym + l] = t;
    }
    if (r + 1 < ch.num_rx) __syncthreads();   // red is rewritten by the next RX
  }
}

// OFDM TX: one slot = one OFDM symbol; 2048/N slots per 256-thread block.
// QAMModulator.bits_to_symbols (modulator.py:61-88) / coded RE mapping via
// tx_map (rate_match_turbo + T/F interleaver, rate_matching.py:193-297,
// ofdm_core.py:1040-1099), ResourceMapper.map_symbols (resource_mapper.py:
// 181-223), ifft*sqrt(N) + CP (modulator.py:242-248).
// SCF (SC-FDM, uncoded chains): the Nd QAM symbols of the OFDM symbol are
// DFT-precoded (M = Nd, core/modulator.py:232-236) in a second LDS buffer first.
// CH: the channel applied in place (tx_channel: 1 static taps, 2 time-varying);
// NC: compile-time N (fft_lds).
template <class R, int CODED, int BPS, bool SCF = false, int CH = 0, int NC = 0, int NP = 0>
__global__ __launch_bounds__(WG) void k_ofdm_tx(Grid g, const uint32_t* __restrict__ pw, int PW,
                                                const uint32_t* __restrict__ enc, int enc_words,
                                                const int32_t* __restrict__ tx_map, cx<R>* __restrict__ x, int B,
                                                cx<R>* __restrict__ cap_syms, int stage_enc, TxChannelT<R> ch) {
  using V = cx<R>;
  using G = GridT<R>;
  V* sm = dyn_lds<V>();
  const int N = NC ? NC : g.N, T = N >> 3, spw = WG / T;
  const int slot = threadIdx.x / T, tid = threadIdx.x % T;
  const int gs = blockIdx.x * spw + slot;
  const int b = gs / g.n_sym, l = gs - b * g.n_sym;
  const bool active = slot < spw && b < B;
  V* buf = sm + slot * N;
  V* pre = SCF ? sm + (spw + slot) * N : buf;   // SC-FDM: QAM symbols -> DFT buffer
  // coded: the frame's coded streams (~10 KB) are staged in LDS with coalesced
  // loads, so the 6 rate-match / interleaver bit gathers per RE hit LDS
  // instead of issuing scattered global loads
  const uint32_t* fe = enc + (size_t)b * enc_words;
  if (CODED && stage_enc) {
    uint32_t* es = reinterpret_cast<uint32_t*>(sm + spw * N) + slot * enc_words;
    if (active)
      for (int i = tid; i < enc_words; i += T) es[i] = fe[i];
    fe = es;
  }
  // coded: every tx_map entry and RE position of this thread's (at most QM)
  // data REs is loaded before the LDS zeroing and the barrier, so their
  // latency overlaps that instead of serialising with the per-RE gathers
  constexpr int QM = 4;   // Nd < N/2 = QM * T for every LTE profile
  int srcs[CODED ? QM : 1][CODED ? BPS : 1];
  int kpos[CODED ? QM : 1];
  if constexpr (CODED) {
#pragma unroll
    for (int q = 0; q < QM; ++q) {
      const int j = tid + q * T;
      const bool ok = active && j < g.Nd;
      const int64_t t0 = ((int64_t)l * g.Nd + j) * BPS;
#pragma unroll
      for (int m = 0; m < BPS; ++m) srcs[q][m] = ok ? tx_map[t0 + m] : -1;
      kpos[q] = ok ? g.data_idx[j] : 0;
    }
  }
  if (active) {
    for (int k = tid; k < N; k += T) buf[k] = mkc((R)0, (R)0);
    if constexpr (SCF)
      for (int k = g.Nd + tid; k < N; k += T) pre[k] = mkc((R)0, (R)0);
  }
  __syncthreads();
  if (CODED && active) {
#pragma unroll
    for (int q = 0; q < QM; ++q) {
      const int j = tid + q * T;
      if (j >= g.Nd) break;
      int idx = 0;
      bool zero = false;
#pragma unroll
      for (int m = 0; m < BPS; ++m) {
        zero |= srcs[q][m] == -2;
        const uint32_t bit = srcs[q][m] >= 0 ? getbit(fe, srcs[q][m]) : 0u;
        idx = (idx << 1) | (int)bit;
      }
      const V sym = zero ? mkc((R)0, (R)0) : qam_point<BPS, R>(idx);
      buf[kpos[q]] = sym;
      if (cap_syms) cap_syms[(size_t)b * g.n_sym * g.Nd + (size_t)l * g.Nd + j] = sym;
    }
  }
  if (active) {
    const uint32_t* fb = pw + (size_t)b * PW;
    for (int j = tid; j < (CODED ? 0 : g.Nd); j += T) {   // uncoded: payload bits in order
      const int64_t t0 = ((int64_t)l * g.Nd + j) * BPS;
      const int idx = (int)getbits<BPS>(fb, t0, INT64_MAX);
      const V sym = qam_point<BPS, R>(idx);
      if constexpr (SCF) pre[j] = sym;
      else buf[g.data_idx[j]] = sym;
      if (cap_syms) cap_syms[(size_t)b * g.n_sym * g.Nd + (size_t)l * g.Nd + j] = sym;
    }
    for (int p = tid; p < g.Np; p += T) buf[g.pilot_idx[p]] = G::pilots(g)[p];
  }
  if constexpr (SCF) {
    dft_bluestein(pre, g, tid, T, active);
    if (active)
      for (int j = tid; j < g.Nd; j += T) buf[g.data_idx[j]] = pre[j];
  }
  __syncthreads();
  const R sc = tx_scale<R>(N);
  // f64 + channel: the IFFT's last pass applies the output scale
  fft_lds<true, NC, CH != 0 && sizeof(R) == 8>(buf, N, g.log2N, G::tw(g), tid, active, sc);
  if constexpr (CH != 0) {
    tx_channel<R, CH == 2, NP>(buf, g, ch, b, l, slot, tid, T, active, sc);
  } else if (active) {
    V* xo = x + (size_t)b * g.L + (size_t)l * (N + g.cp);
    for (int k = tid; k < N; k += T) xo[g.cp + k] = cscale(buf[k], sc);
    for (int k = tid; k < g.cp; k += T) xo[k] = cscale(buf[N - g.cp + k], sc);
  }
}

// LDS bytes of the coded stream staged per slot (0: not staged).
// LTE_TX_STAGE=0 gathers the coded bits through L1 / L2 instead (A/B knob).
static size_t tx_enc_shm(int coded, int spw, int enc_words) {
  const size_t e = (size_t)spw * enc_words * sizeof(uint32_t);
  static const int on = [] {
    const char* v = std::getenv("LTE_TX_STAGE");
    return v ? std::atoi(v) : 1;
  }();
  return coded && on && e <= 32768 ? e : 0;
}

template <class R>
int launch_ofdm_tx(hipStream_t s, const Grid& g, int coded, const uint32_t* pw, int PW, const uint32_t* enc,
                   int enc_words, const int32_t* tx_map, cx<R>* x, int B, cx<R>* cap_syms, int sc_fdm) {
  const int spw = WG / (g.N >> 3);
  const int64_t total = (int64_t)B * g.n_sym;
  if (total > 0x7FFFFFFF - spw || (g.bps != 2 && g.bps != 4 && g.bps != 6)) return (int)hipErrorInvalidValue;
  if (sc_fdm && (coded || !GridT<R>::chirp(g) || !GridT<R>::bhat(g) || 2 * g.Nd > g.N))
    return (int)hipErrorInvalidValue;
  const int blocks = (int)((total + spw - 1) / spw);
  const size_t enc_shm = tx_enc_shm(coded, spw, enc_words);
  const int stage_enc = enc_shm > 0;
  const size_t shm = (sc_fdm ? 2 : 1) * spw * g.N * sizeof(cx<R>) + enc_shm;
#define LTE_TX(C_, B_, S_)                                                                                      \
  hipLaunchKernelGGL((k_ofdm_tx<R, C_, B_, S_>), dim3(blocks), dim3(WG), shm, s, g, pw, PW, enc, enc_words, tx_map, \
                     x, B, cap_syms, stage_enc, TxChannelT<R>{})
  if (coded) {
    if (g.bps == 2) LTE_TX(1, 2, false); else if (g.bps == 4) LTE_TX(1, 4, false); else LTE_TX(1, 6, false);
  } else if (sc_fdm) {
    if (g.bps == 2) LTE_TX(0, 2, true); else if (g.bps == 4) LTE_TX(0, 4, true); else LTE_TX(0, 6, true);
  } else {
    if (g.bps == 2) LTE_TX(0, 2, false); else if (g.bps == 4) LTE_TX(0, 4, false); else LTE_TX(0, 6, false);
  }
#undef LTE_TX
  return (int)hipGetLastError();
}

bool txch_supported(const Grid& g, int n_paths, int max_delay) {
  return g.N >= 512 && n_paths >= 1 && n_paths <= TXCH_MAXP && max_delay >= 0 && max_delay <= g.cp &&
         2 * max_delay < g.N + g.cp;
}

// one k_ofdm_tx<.., CH> launch; float64 static taps (CH 1) of the ITU path
// counts 4 and 6 with the count at compile time (tx_channel NP)
template <class R, int C_, int B_, bool S_, int CH_, int NC_>
static void ofdm_tx_ch_np(hipStream_t s, int blocks, size_t shm, const Grid& g, const uint32_t* pw, int PW,
                          const uint32_t* enc, int enc_words, const int32_t* tx_map, int B, cx<R>* cap_syms,
                          int stage_enc, const TxChannelT<R>& ch) {
  if constexpr (CH_ == 1 && !S_ && sizeof(R) == 8) {
    if (ch.n_paths == 4) {
      hipLaunchKernelGGL((k_ofdm_tx<R, C_, B_, S_, CH_, NC_, 4>), dim3(blocks), dim3(WG), shm, s, g, pw, PW, enc,
                         enc_words, tx_map, (cx<R>*)nullptr, B, cap_syms, stage_enc, ch);
      return;
    }
    if (ch.n_paths == 6) {
      hipLaunchKernelGGL((k_ofdm_tx<R, C_, B_, S_, CH_, NC_, 6>), dim3(blocks), dim3(WG), shm, s, g, pw, PW, enc,
                         enc_words, tx_map, (cx<R>*)nullptr, B, cap_syms, stage_enc, ch);
      return;
    }
  }
  hipLaunchKernelGGL((k_ofdm_tx<R, C_, B_, S_, CH_, NC_>), dim3(blocks), dim3(WG), shm, s, g, pw, PW, enc, enc_words,
                     tx_map, (cx<R>*)nullptr, B, cap_syms, stage_enc, ch);
}
// compile-time N: 2048 (20 MHz), and 1024 (10 MHz, config 3) for the uncoded
// OFDM transmitters with static taps
template <class R, int C_, int B_, bool S_, int CH_>
static void ofdm_tx_ch_go(hipStream_t s, int blocks, size_t shm, const Grid& g, const uint32_t* pw, int PW,
                          const uint32_t* enc, int enc_words, const int32_t* tx_map, int B, cx<R>* cap_syms,
                          int stage_enc, const TxChannelT<R>& ch) {
  if (g.N == 2048) {
    ofdm_tx_ch_np<R, C_, B_, S_, CH_, 2048>(s, blocks, shm, g, pw, PW, enc, enc_words, tx_map, B, cap_syms, stage_enc, ch);
    return;
  }
  if constexpr (CH_ == 1 && !S_ && !C_) {
    if (g.N == 1024) {
      ofdm_tx_ch_np<R, C_, B_, S_, CH_, 1024>(s, blocks, shm, g, pw, PW, enc, enc_words, tx_map, B, cap_syms, stage_enc,
                                              ch);
      return;
    }
  }
  ofdm_tx_ch_np<R, C_, B_, S_, CH_, 0>(s, blocks, shm, g, pw, PW, enc, enc_words, tx_map, B, cap_syms, stage_enc, ch);
}

template <class R>
int launch_ofdm_tx_ch(hipStream_t s, const Grid& g, int coded, const uint32_t* pw, int PW, const uint32_t* enc,
                      int enc_words, const int32_t* tx_map, int B, cx<R>* cap_syms, const TxChannelT<R>& ch,
                      int sc_fdm) {
  const int spw = WG / (g.N >> 3);
  const int64_t total = (int64_t)B * g.n_sym;
  if (sc_fdm && (coded || !GridT<R>::chirp(g) || !GridT<R>::bhat(g) || 2 * g.Nd > g.N))
    return (int)hipErrorInvalidValue;
  if (!txch_supported(g, ch.n_paths, ch.max_delay) || total > 0x7FFFFFFF - spw ||
      (g.bps != 2 && g.bps != 4 && g.bps != 6))
    return (int)hipErrorInvalidValue;
  if constexpr (sizeof(R) == 8) {   // config 3: the wave-private TX (lte_wave.hip; LTE_SIMO_TX_WAVE=0: this kernel)
    if (simo_tx_wave_enabled() && tx_simo_w_supported(g, 1, coded, sc_fdm, ch))
      return launch_ofdm_tx_simo_w(s, g, pw, PW, B, cap_syms, ch);
  }
  const int blocks = (int)((total + spw - 1) / spw);
  const size_t enc_shm = tx_enc_shm(coded, spw, enc_words);
  const int stage_enc = enc_shm > 0;
  const size_t shm = (sc_fdm ? 2 : 1) * (size_t)spw * g.N * sizeof(cx<R>) + enc_shm;
#define LTE_TXC2(C_, B_, S_, CH_) \
  ofdm_tx_ch_go<R, C_, B_, S_, CH_>(s, blocks, shm, g, pw, PW, enc, enc_words, tx_map, B, cap_syms, stage_enc, ch)
#define LTE_TXC(C_, B_, S_)                                                                                      \
  do {                                                                                                             \
    if (ch.tcoef) { LTE_TXC2(C_, B_, S_, 2); } else { LTE_TXC2(C_, B_, S_, 1); }                                   \
  } while (0)
  if (coded) {
    if (g.bps == 2) LTE_TXC(1, 2, false); else if (g.bps == 4) LTE_TXC(1, 4, false); else LTE_TXC(1, 6, false);
  } else if (sc_fdm) {   // SC-FDM (uncoded SISO / SIMO transmitters): DFT precoding, then the same channel
    if (g.bps == 2) LTE_TXC(0, 2, true); else if (g.bps == 4) LTE_TXC(0, 4, true); else LTE_TXC(0, 6, true);
  } else {
    if (g.bps == 2) LTE_TXC(0, 2, false); else if (g.bps == 4) LTE_TXC(0, 4, false); else LTE_TXC(0, 6, false);
  }
#undef LTE_TXC
#undef LTE_TXC2
  return (int)hipGetLastError();
}

// Coded OFDM TX + static-tap channel, one slot per frame walking its OFDM
// symbols in order: the frame's coded streams are staged in LDS once (instead
// of once per symbol), then per symbol the same work as k_ofdm_tx<.., CH>: RE
// mapping through tx_map, pilots, IFFT (f64: output scale in the last pass),
// taps, received stream and per-symbol power.  Identical arithmetic per
// sample (test_frame_tx_matches_symbol_tx).
#ifndef TXF_WAVES
#define TXF_WAVES 1
#endif
#ifndef LTE_LDS_PROBE   // timing probes of the per-RE LDS accesses (A/B builds only)
#define LTE_LDS_PROBE 0
#endif
#ifndef TXF_STAGE   // 1: the frame's coded streams staged in LDS; 0: bit gathers through L1 / L2
#define TXF_STAGE 1
#endif
// Lane order (txf_re, plan_txf_lane_order): slot s = tid + q T of symbol l
// carries RE txf_re[l][s] and reads its coded-bit sources from the slot-ordered
// copy of tx_map (txf_map[l][s][m]), chosen on the host so that the 32 lanes of
// each ds_read_b32 gather hit distinct LDS banks; null: slot s = RE s.
// SP = 2 (N = 2048): a 512-thread block per frame whose halves transform
// symbols 2s and 2s + 1 side by side, sharing one LDS copy of the coded
// streams (the symbols of a frame are independent here: the taps' reach into
// the previous symbol is k_chan_fix's).
template <class R, int BPS, int NC = 0, bool TV = false, int NP = 0, int SP = 1>
__global__ __launch_bounds__(WG * SP, TXF_WAVES) void k_ofdm_txf(Grid g, const uint32_t* __restrict__ enc, int enc_words,
                                                          const int32_t* __restrict__ tx_map,
                                                          const int32_t* __restrict__ txf_map,
                                                          const int32_t* __restrict__ txf_re, int B,
                                                          cx<R>* __restrict__ cap_syms, TxChannelT<R> ch) {
  using V = cx<R>;
  using G = GridT<R>;
  V* sm = dyn_lds<V>();
  static_assert(SP == 1 || NC == 2048, "symbol pairs: one frame per block");
  const int N = NC ? NC : g.N, T = N >> 3, spw = SP == 1 ? WG / T : 1;
  const int slot = threadIdx.x / T, tid0 = threadIdx.x % T;   // SP = 2: slot = the half
  const int b = SP == 1 ? blockIdx.x * spw + slot : blockIdx.x;
  const bool fa = SP == 1 ? slot < spw && b < B : b < B;
  V* buf = sm + slot * N;
#if TXF_STAGE
  uint32_t* es = reinterpret_cast<uint32_t*>(sm + (SP == 1 ? spw : 2) * N) + (SP == 1 ? slot * enc_words : 0);
  if (fa) {
    const uint32_t* fe = enc + (size_t)b * enc_words;
    for (int i = SP == 1 ? tid0 : (int)threadIdx.x; i < enc_words; i += SP == 1 ? T : 2 * T) es[i] = fe[i];
  }
#else
  const uint32_t* es = enc + (size_t)(fa ? b : 0) * enc_words;
#endif
  const R sc = tx_scale<R>(N);
  constexpr int QM = 4;   // Nd < N/2 = QM * T for every LTE profile
  for (int l0 = 0; l0 < g.n_sym; l0 += SP) {
    const int l = l0 + (SP == 1 ? 0 : slot);
    const bool active = fa && l < g.n_sym;
    int tid = tid0;   // opaque per symbol: address arithmetic is not hoisted out of the loop
    asm volatile("" : "+v"(tid));
    int srcs[QM][BPS];
    int kpos[QM], jre[QM];
#pragma unroll
    for (int q = 0; q < QM; ++q) {
      const int sl = tid + q * T;
      const bool ok = active && sl < g.Nd;
      const int j = txf_re ? (ok ? txf_re[(size_t)l * QM * T + sl] : 0) : sl;
      const int64_t t0 = txf_re ? ((int64_t)l * QM * T + sl) * BPS : ((int64_t)l * g.Nd + j) * BPS;
      const int32_t* map = txf_re ? txf_map : tx_map;
      // the RE's BPS entries as 8-B loads (t0 even; BPS 4: 16 B)
      if (ok) {
        if constexpr (BPS == 4) {
          const int4 v = *reinterpret_cast<const int4*>(map + t0);
          srcs[q][0] = v.x; srcs[q][1] = v.y; srcs[q][2] = v.z; srcs[q][3] = v.w;
        } else {
#pragma unroll
          for (int m = 0; m < BPS; m += 2) {
            const int2 v = *reinterpret_cast<const int2*>(map + t0 + m);
            srcs[q][m] = v.x;
            srcs[q][m + 1] = v.y;
          }
        }
      } else {
#pragma unroll
        for (int m = 0; m < BPS; ++m) srcs[q][m] = -1;
      }
      kpos[q] = ok ? g.data_idx[j] : 0;
      jre[q] = j;
#if LTE_LDS_PROBE & 1   // timing probe only (wrong outputs): conflict-free RE positions
      kpos[q] = ok ? N / 2 - 512 + j : 0;
#endif
#if LTE_LDS_PROBE & 2   // timing probe only (wrong outputs): conflict-free bit gathers
#pragma unroll
      for (int m = 0; m < BPS; ++m) srcs[q][m] = ok ? 32 * ((j + 41 * m) % 300) + 5 : -1;
#endif
    }
    if (active)
      for (int k = tid; k < N; k += T) buf[k] = mkc((R)0, (R)0);
    __syncthreads();   // (first symbol: also the staged streams)
    if (active) {
#pragma unroll
      for (int q = 0; q < QM; ++q) {
        if (tid + q * T >= g.Nd) break;
        int idx = 0;
        bool zero = false;
#pragma unroll
        for (int m = 0; m < BPS; ++m) {
          zero |= srcs[q][m] == -2;
          const uint32_t bit = srcs[q][m] >= 0 ? getbit(es, srcs[q][m]) : 0u;
          idx = (idx << 1) | (int)bit;
        }
        const V sym = zero ? mkc((R)0, (R)0) : qam_point<BPS, R>(idx);
        buf[kpos[q]] = sym;
        if (cap_syms) cap_syms[(size_t)b * g.n_sym * g.Nd + (size_t)l * g.Nd + jre[q]] = sym;
      }
      for (int p = tid; p < g.Np; p += T) buf[g.pilot_idx[p]] = G::pilots(g)[p];
    }
    __syncthreads();
    fft_lds<true, NC, sizeof(R) == 8>(buf, N, g.log2N, G::tw(g), tid, active, sc);
    // every read of buf in tx_channel precedes its reduction barrier, so the
    // next symbol may overwrite buf after it
    tx_channel<R, TV, NP>(buf, g, ch, b, l, slot, tid, T, active, sc);
  }
}

#ifndef LTE_TXF_SP   // symbols per pass of k_ofdm_txf's float64 PedA instance (1 or 2)
#define LTE_TXF_SP 2
#endif
// k_ofdm_txf's compile-time-path-count instance (N = 2048): SP = 2 takes one
// 512-thread block per frame and 64 KB + the staged streams of LDS
template <class R, int BPS, int SP>
static void txf_peda_launch(hipStream_t s, const Grid& g, const uint32_t* enc, int enc_words, const int32_t* tx_map,
                            const int32_t* txf_map, const int32_t* txf_re, int B, cx<R>* cap_syms,
                            const TxChannelT<R>& ch, int blocks, size_t shm, size_t shm2) {
  auto k = k_ofdm_txf<R, BPS, 2048, false, 4, SP>;
  if (SP == 2) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm2);
  hipLaunchKernelGGL(k, dim3(SP == 2 ? B : blocks), dim3(WG * SP), SP == 2 ? shm2 : shm, s, g, enc, enc_words, tx_map,
                     txf_map, txf_re, B, cap_syms, ch);
}
template <class R>
int launch_ofdm_txf(hipStream_t s, const Grid& g, const uint32_t* enc, int enc_words, const int32_t* tx_map,
                    const int32_t* txf_map, const int32_t* txf_re, int B, cx<R>* cap_syms,
                    const TxChannelT<R>& ch) {
  const int spw = WG / (g.N >> 3);
  if (!txch_supported(g, ch.n_paths, ch.max_delay) || (g.bps != 2 && g.bps != 4 && g.bps != 6)) return (int)hipErrorInvalidValue;
  if constexpr (sizeof(R) == 8)
    if (!txf_map && txf_w_supported(g, 1, ch.n_paths, ch.max_delay, ch.num_rx, ch.tcoef != nullptr) &&
        tx_wave_enabled())
      return launch_ofdm_txf_w(s, g, enc, enc_words, tx_map, B, cap_syms, ch);
  const size_t shm = (size_t)spw * g.N * sizeof(cx<R>) + (TXF_STAGE ? (size_t)spw * enc_words * sizeof(uint32_t) : 0);
  if (shm > 65536) return (int)hipErrorInvalidValue;
  // symbol pairs (LTE_TXF_SP = 2): two grids and one staged copy per frame
  const size_t shm2 = 2 * (size_t)g.N * sizeof(cx<R>) + (TXF_STAGE ? (size_t)enc_words * sizeof(uint32_t) : 0);
  const int blocks = (B + spw - 1) / spw;
#define LTE_TXF(BPS_, NC_)                                                                                      \
  do {                                                                                                          \
    if (ch.tcoef)                                                                                               \
      hipLaunchKernelGGL((k_ofdm_txf<R, BPS_, NC_, true>), dim3(blocks), dim3(WG), shm, s, g, enc, enc_words,   \
                         tx_map, txf_map, txf_re, B, cap_syms, ch);                              \
    else if (NC_ == 2048 && ch.n_paths == 4 && sizeof(R) == 8)                                                  \
      txf_peda_launch<R, BPS_, NC_ == 2048 ? LTE_TXF_SP : 1>(s, g, enc, enc_words, tx_map, txf_map, txf_re, B,     \
                                                            cap_syms, ch, blocks, shm, shm2);                   \
    else                                                                                                        \
      hipLaunchKernelGGL((k_ofdm_txf<R, BPS_, NC_>), dim3(blocks), dim3(WG), shm, s, g, enc, enc_words, tx_map, \
                         txf_map, txf_re, B, cap_syms, ch);                                      \
  } while (0)
  if (g.N == 2048) {
    if (g.bps == 2) LTE_TXF(2, 2048); else if (g.bps == 4) LTE_TXF(4, 2048); else LTE_TXF(6, 2048);
  } else {
    if (g.bps == 2) LTE_TXF(2, 0); else if (g.bps == 4) LTE_TXF(4, 0); else LTE_TXF(6, 0);
  }
#undef LTE_TXF
  return (int)hipGetLastError();
}

// Power of each symbol's first max_delay channel-output samples (their delayed
// taps reach into the previous symbol's tail, or the zero prefix of symbol 0),
// added to the symbol's partial.  16 lanes per (frame, symbol), one sample
// each (coalesced head / tail reads), summed by a fixed xor butterfly.
constexpr int CHF_LANES = 16;
template <class R>
__global__ __launch_bounds__(WG) void k_chan_fix(Grid g, int B, TxChannelT<R> ch) {
  using V = cx<R>;
  const int64_t i = ((int64_t)blockIdx.x * WG + threadIdx.x) / CHF_LANES;   // (frame, RX, symbol)
  const int lane = threadIdx.x % CHF_LANES;
  const bool ok = i < (int64_t)B * ch.num_rx * g.n_sym;
  R pw = (R)0;
  if (ok) {
    const int l = (int)(i % g.n_sym);
    const int64_t br = i / g.n_sym;
    const int b = (int)(br / ch.num_rx);
    const int D = ch.max_delay;
    const V* hd = ch.xh + ((size_t)b * g.n_sym + l) * 2 * D;   // this symbol's head; hd[-D..-1] = previous symbol's tail
    const V* cb = ch.coef + (size_t)br * ch.n_paths;
    constexpr int NCF = mimo_ncf<R>();
    const R dc = (R)0.5 * (R)(g.N + g.cp - 1);
    for (int m = lane; m < D; m += CHF_LANES) {
      V v = mkc((R)0, (R)0);
      for (int p = 0; p < ch.n_paths; ++p) {
        const int j = m - ch.delays[p];
        const V xv = (j >= 0 || l > 0) ? hd[j] : mkc((R)0, (R)0);
        V h;
        if (ch.tcoef) {   // the symbol's Taylor set at d = m - (S - 1) / 2 (tx_channel)
          const V* c = ch.tcoef + (((size_t)br * ch.n_paths + p) * g.n_sym + l) * NCF;
          const R d = (R)m - dc;
          h = c[NCF - 1];
#pragma unroll
          for (int k = NCF - 2; k >= 0; --k) h = mkc(h.x * d + c[k].x, h.y * d + c[k].y);
        } else {
          h = cb[p];
        }
        v = cadd(v, cmul(h, xv));
      }
      pw += v.x * v.x + v.y * v.y;
    }
  }
#pragma unroll
  for (int o = CHF_LANES / 2; o > 0; o >>= 1) pw += __shfl_xor(pw, o);
  if (ok && lane == 0) ch.pow_part[i] += pw;
}

template <class R>
int launch_chan_fix(hipStream_t s, const Grid& g, int B, const TxChannelT<R>& ch) {
  const int64_t n = (int64_t)B * ch.num_rx * g.n_sym * CHF_LANES;
  if (ch.max_delay == 0 || n == 0) return 0;
  hipLaunchKernelGGL(k_chan_fix<R>, dim3((unsigned)((n + WG - 1) / WG)), dim3(WG), 0, s, g, B, ch);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Fading taps: RayleighChannel.jakes_fading phases (rayleighchannel.py:20-42).
// One thread per (frame, rx, path): 16 phases phi_m (Philox or injected) and
// the static coefficient used when fD = 0.  f64 forms it as the reference
// does: h = (sum_m exp(j phi_m)) * sqrt(2/16), then gain * h; f32 folds
// sqrt(2/16) * gain into one factor.
template <class R>
__global__ __launch_bounds__(WG) void k_fading(int B, int num_rx, int n_paths, const R* __restrict__ gains,
                                               const uint64_t* __restrict__ fid, uint64_t seed,
                                               const R* __restrict__ inj, int64_t inj_stride,
                                               R* __restrict__ phases, cx<R>* __restrict__ coef) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int per = num_rx * n_paths;
  if (i >= B * per) return;
  const int b = i / per, rp = i % per, rx = rp / n_paths, p = rp % n_paths;
  R* ph = phases + (size_t)i * 16;
  R sr = (R)0, si = (R)0;
  for (int m = 0; m < 16; ++m) {
    R v;
    if (inj) {
      v = inj[(size_t)b * inj_stride + (size_t)rp * 16 + m];
    } else {
      const u32x4 r = rng4(seed, fid[b], RNG_STREAM_FADE + (uint32_t)rx * 64u + (uint32_t)p, (uint32_t)(m >> 2));
      const int q = m & 3;
      const uint32_t u = q == 0 ? r.x : q == 1 ? r.y : q == 2 ? r.z : r.w;
      if constexpr (sizeof(R) == 8) v = 6.283185307179586 * (((double)u + 0.5) * 2.3283064365386962890625e-10);
      else v = 6.2831853071795864f * ((u >> 8) * (1.0f / 16777216.0f));
    }
    ph[m] = v;
    R s, c;
    if constexpr (sizeof(R) == 8) sincos(v, &s, &c);
    else sincosf(v, &s, &c);
    sr += c;
    si += s;
  }
  if constexpr (sizeof(R) == 8) {
    const double k = sqrt(2.0 / 16.0), gn = gains[p];
    coef[i] = make_double2(gn * (sr * k), gn * (si * k));
  } else {
    const float k = sqrtf(2.0f / 16.0f) * gains[p];
    coef[i] = make_float2(sr * k, si * k);
  }
}

template <class R>
int launch_fading(hipStream_t s, int B, int num_rx, int n_paths, const R* gains_dev, const uint64_t* fid,
                  uint64_t seed, const R* inj_ph, int64_t inj_stride, R* phases, cx<R>* coef) {
  const int n = B * num_rx * n_paths;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_fading<R>, dim3((n + WG - 1) / WG), dim3(WG), 0, s, B, num_rx, n_paths, gains_dev, fid, seed,
                     inj_ph, inj_stride, phases, coef);
  return (int)hipGetLastError();
}

// Host payload injection: the caller's uint8 bits (copied to the device as
// they are) packed MSB-first into 32-bit words, one word per thread (the
// lanes of a wave read 64 consecutive 32-byte runs: coalesced).
__global__ __launch_bounds__(WG) void k_pack_bits(const uint8_t* __restrict__ bits, int64_t stride, int n_bits,
                                                  int nwd, int nf, uint32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * WG + threadIdx.x;
  if (i >= (int64_t)nf * nwd) return;
  const int f = (int)(i / nwd), w = (int)(i - (int64_t)f * nwd);
  const uint8_t* src = bits + f * stride + (int64_t)w * 32;
  const int n = min(32, n_bits - w * 32);
  uint32_t v = 0;
  for (int k = 0; k < n; ++k) v |= (uint32_t)(src[k] & 1) << (31 - k);
  out[i] = v;
}

int launch_pack_bits(hipStream_t s, const uint8_t* bits, int64_t stride, int n_bits, int nwd, int nf, uint32_t* out) {
  const int64_t n = (int64_t)nf * nwd;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_pack_bits, dim3((unsigned)((n + WG - 1) / WG)), dim3(WG), 0, s, bits, stride, n_bits, nwd, nf,
                     out);
  return (int)hipGetLastError();
}

// The Philox mode's raw streams (lte_philox_host): one thread per (frame,
// counter) -- the four 32-bit outputs of rng4 and the unit normal pairs every
// noise loader forms from them, (x, y) and (z, w): gauss2<double>
// (box_muller64t) and gauss2<float> (box_muller).
__global__ __launch_bounds__(WG) void k_philox_draws(uint64_t seed, const uint64_t* __restrict__ fid, int nf,
                                                     uint32_t stream, int64_t n_ctr, uint32_t* __restrict__ u,
                                                     double* __restrict__ g64, float* __restrict__ g32) {
  const int64_t i = (int64_t)blockIdx.x * WG + threadIdx.x;
  if (i >= (int64_t)nf * n_ctr) return;
  const int f = (int)(i / n_ctr);
  const uint32_t c = (uint32_t)(i - (int64_t)f * n_ctr);
  const u32x4 r = rng4(seed, fid[f], stream, c);
  if (u) {
    u[4 * i] = r.x;
    u[4 * i + 1] = r.y;
    u[4 * i + 2] = r.z;
    u[4 * i + 3] = r.w;
  }
  if (g64) {
    const double2 a = gauss2<double>(r.x, r.y), b = gauss2<double>(r.z, r.w);
    g64[4 * i] = a.x;
    g64[4 * i + 1] = a.y;
    g64[4 * i + 2] = b.x;
    g64[4 * i + 3] = b.y;
  }
  if (g32) {
    const float2 a = gauss2<float>(r.x, r.y), b = gauss2<float>(r.z, r.w);
    g32[4 * i] = a.x;
    g32[4 * i + 1] = a.y;
    g32[4 * i + 2] = b.x;
    g32[4 * i + 3] = b.y;
  }
}

int launch_philox_draws(hipStream_t s, uint64_t seed, const uint64_t* fid, int nf, uint32_t stream, int64_t n_ctr,
                        uint32_t* u, double* g64, float* g32) {
  const int64_t n = (int64_t)nf * n_ctr;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_philox_draws, dim3((unsigned)((n + WG - 1) / WG)), dim3(WG), 0, s, seed, fid, nf, stream, n_ctr,
                     u, g64, g32);
  return (int)hipGetLastError();
}

// Per-symbol Taylor sets of the SISO paths (fD != 0, the fused TX channel):
// one thread per (frame, path) from k_fading's 16 phases (jakes_symbol_sets).
template <class R>
__global__ __launch_bounds__(WG) void k_jakes_sets(int B, int n_paths, int n_sym, int sym_len,
                                                   const R* __restrict__ phases, const R* __restrict__ gains,
                                                   double fD, double fs, cx<R>* __restrict__ tcoef) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * n_paths) return;
  const int p = i % n_paths;
  double ph[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) ph[m] = phases[(size_t)i * 16 + m];
  jakes_symbol_sets<R>(ph, (double)gains[p], fD, fs, sym_len, n_sym, tcoef + (size_t)i * n_sym * mimo_ncf<R>());
}

template <class R>
int launch_jakes_sets(hipStream_t s, int B, int n_paths, int n_sym, int sym_len, const R* phases, const R* gains,
                      double fD, double fs, cx<R>* tcoef) {
  const int n = B * n_paths;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_jakes_sets<R>, dim3((n + WG - 1) / WG), dim3(WG), 0, s, B, n_paths, n_sym, sym_len, phases,
                     gains, fD, fs, tcoef);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Channel: y[n] = sum_p g_p h_p[n] x[n - d_p] (RayleighChannel.filter,
// rayleighchannel.py:44-58: stream-level delay with zero prefix, Q4) and the
// per-block partial sums of |y|^2 for the measured-power SNR (channel.py:
// 217-224, Q5).  AWGN: only the power of x.  grid (nblk, num_rx, B); a block
// streams CH_CHUNK samples, CH_PER per thread with a 256-sample stride (every
// load / store instruction is one coalesced row), then one block reduction of
// the power.
constexpr int CH_PER = 8, CH_CHUNK = WG * CH_PER;

// jakes_fading at t = n / fs: h = sqrt(2/16) sum_m exp(j (2 pi fD cos(alpha_m) t
// + phi_m)), alpha_m = 2 pi (m+1) / 16, times the path gain
template <class R>
__device__ __forceinline__ cx<R> jakes_coef(const R* __restrict__ ph, R gain, R fD, R t) {
  R sr = (R)0, si = (R)0;
  for (int m = 0; m < 16; ++m) {
    if constexpr (sizeof(R) == 8) {
      const double al = 6.283185307179586 * (double)(m + 1) / 16.0;
      const double arg = 6.283185307179586 * fD * cos(al) * t + ph[m];
      double sv, cv;
      sincos(arg, &sv, &cv);
      sr += cv;
      si += sv;
    } else {
      const float al = 6.2831853071795864f * (float)(m + 1) / 16.0f;
      const float arg = 6.2831853071795864f * fD * cosf(al) * t + ph[m];
      float sv, cv;
      sincosf(arg, &sv, &cv);
      sr += cv;
      si += sv;
    }
  }
  if constexpr (sizeof(R) == 8) {
    const double k = sqrt(2.0 / 16.0);
    return make_double2(gain * (sr * k), gain * (si * k));
  } else {
    const float k = sqrtf(2.0f / 16.0f) * gain;
    return make_float2(sr * k, si * k);
  }
}

// Time-varying taps (fD != 0) by a Taylor expansion of the Jakes sum: over a
// sub-interval of SL samples centred at t_c the sum is
//   sum_m a_m exp(j w_m tau) = sum_k c_k tau^k,  a_m = exp(j (w_m t_c + phi_m)),
//   c_k = sum_m a_m (j w_m)^k / k!,  tau = t - t_c,
// with a_m formed exactly as jakes_coef forms one sample (the reference's
// argument order).  The host picks SL (a power of two, >= 64) so that
// |w tau| <= 2.7e-3 on it: the degree-5 remainder is below 16 (2.7e-3)^6 / 720
// ~ 9e-18, under float64 rounding, and the per-sample cost drops from 16 sincos
// to 5 complex Horner steps per path (3 km/h at 20 MHz: one interval per 2048
// samples; SL = 64 covers fD <= ~420 Hz).  Larger fD, or more than CH_MAXP
// paths, keep the per-sample sum (SL = 0).
constexpr int JK_DEG = 5;
constexpr int JK_MINSL = 64;

// Rayleigh with every delay <= CH_HALO: the chunk plus its delay halo is staged
// in LDS once, so the n_paths delayed taps read LDS instead of re-fetching x
// through L1/L2 (the kernel was latency bound at ~2.2 TB/s); otherwise the
// taps load from global memory.
constexpr int CH_HALO = 256;
constexpr int CH_MAXP = 8;   // taps held in registers (ITU profiles have <= 6)

template <class R>
__global__ __launch_bounds__(WG) void k_channel(int L, int num_rx, int rayleigh, int n_paths,
                                                const int32_t* __restrict__ delays, const R* __restrict__ gains,
                                                R fD, R fs, const R* __restrict__ phases,
                                                const cx<R>* __restrict__ coef, const cx<R>* __restrict__ x,
                                                cx<R>* __restrict__ y, R* __restrict__ pow_part, int nblk,
                                                int staged, int SL) {
  using V = cx<R>;
  __shared__ R red[WG / 64];
  __shared__ V xs[CH_CHUNK + CH_HALO];
  V* jc = dyn_lds<V>();   // Taylor coefficients [sub-interval][path][degree] (SL > 0; sized by the launch)
  const int blk = blockIdx.x % nblk, b = blockIdx.x / nblk;
  const int rx = blockIdx.y;
  const V* xf = x + (size_t)b * L;
  V* yf = y + ((size_t)b * num_rx + rx) * L;
  const size_t cb = ((size_t)b * num_rx + rx) * n_paths;
  const int n0 = blk * CH_CHUNK;
  R pw = (R)0;
  if (rayleigh && SL > 0) {
    // time-varying taps: the Taylor coefficients first, overlapping the staging
    // loads below (one barrier for both): one lane per (sub-interval, path,
    // m), the 16 m of a (sub-interval, path) on 16 consecutive lanes, summed
    // by an xor butterfly
    const int nsub = CH_CHUNK / SL, items = nsub * n_paths * 16;
    for (int e0 = 0; e0 < items; e0 += WG) {   // uniform trip count: every lane reaches the shuffles
      const int e = e0 + threadIdx.x, grp = e >> 4, m = e & 15;
      const bool ok = e < items;
      const int sb = ok ? grp / n_paths : 0, p = ok ? grp - sb * n_paths : 0;
      V t = mkc((R)0, (R)0);
      R w = (R)0;
      if (ok) {
        const R tc = (R)(n0 + sb * SL + SL / 2) / fs;
        R arg;
        if constexpr (sizeof(R) == 8) {
          const double al = 6.283185307179586 * (double)(m + 1) / 16.0;
          w = 6.283185307179586 * fD * cos(al);
          arg = w * tc + phases[(cb + p) * 16 + m];
        } else {
          const float al = 6.2831853071795864f * (float)(m + 1) / 16.0f;
          w = 6.2831853071795864f * fD * cosf(al);
          arg = w * tc + phases[(cb + p) * 16 + m];
        }
        R sv, cv;
        if constexpr (sizeof(R) == 8) sincos(arg, &sv, &cv);
        else sincosf(arg, &sv, &cv);
        t = mkc(cv, sv);   // a_m, then a_m (j w_m)^k / k!
      }
#pragma unroll
      for (int k = 0; k <= JK_DEG; ++k) {
        V c = t;
        t = mkc(-t.y * (w / (R)(k + 1)), t.x * (w / (R)(k + 1)));
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          c.x += __shfl_xor(c.x, o);
          c.y += __shfl_xor(c.y, o);
        }
        if (ok && m == 0) jc[(sb * CH_MAXP + p) * (JK_DEG + 1) + k] = c;
      }
    }
  }
  if (rayleigh && staged) {
    if constexpr (sizeof(R) == 4) {   // 16-B pairs of samples (L even)
      const float4* x4 = reinterpret_cast<const float4*>(xf);
      for (int e = threadIdx.x; e < (CH_CHUNK + CH_HALO) / 2; e += WG) {
        const int n = n0 - CH_HALO + 2 * e;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (n >= 0 && n + 1 < L) v = x4[n >> 1];
        else if (n >= 0 && n < L) v.x = xf[n].x, v.y = xf[n].y;
        xs[2 * e] = make_float2(v.x, v.y);
        xs[2 * e + 1] = make_float2(v.z, v.w);
      }
    } else {   // one 16-B sample per lane
      for (int e = threadIdx.x; e < CH_CHUNK + CH_HALO; e += WG) {
        const int n = n0 - CH_HALO + e;
        xs[e] = (n >= 0 && n < L) ? xf[n] : make_double2(0.0, 0.0);
      }
    }
    __syncthreads();
  } else if (rayleigh && SL > 0) {
    __syncthreads();
  }
  if (rayleigh && staged && fD == (R)0 && n_paths <= CH_MAXP) {
    // static taps (fD = 0, the OFDMSimulator default): coefficients and delays
    // in registers, the halo (zero before the frame start) makes every tap an
    // unconditional LDS read
    V cf[CH_MAXP];
    int dl[CH_MAXP];
#pragma unroll
    for (int p = 0; p < CH_MAXP; ++p) {
      cf[p] = p < n_paths ? coef[cb + p] : mkc((R)0, (R)0);
      dl[p] = p < n_paths ? delays[p] : 0;
    }
#pragma unroll
    for (int i = 0; i < CH_PER; ++i) {
      const int n = n0 + i * WG + threadIdx.x;
      if (n >= L) break;
      V v = mkc((R)0, (R)0);
#pragma unroll
      for (int p = 0; p < CH_MAXP; ++p)
        if (p < n_paths) v = cadd(v, cmul(cf[p], xs[n - dl[p] - n0 + CH_HALO]));
      yf[n] = v;
      pw += v.x * v.x + v.y * v.y;
    }
    const R t = block_sum(pw, red);
    if (threadIdx.x == 0) pow_part[((size_t)b * num_rx + rx) * nblk + blk] = t;
    return;
  }
  if (rayleigh && SL > 0) {
    const R k2 = sizeof(R) == 8 ? (R)sqrt(2.0 / 16.0) : sqrtf(2.0f / 16.0f);
#pragma unroll
    for (int i = 0; i < CH_PER; ++i) {
      const int n = n0 + i * WG + threadIdx.x;
      if (n >= L) break;
      const int sb = (n - n0) / SL;
      const R tau = (R)(n - (n0 + sb * SL + SL / 2)) / fs;
      V v = mkc((R)0, (R)0);
      for (int p = 0; p < n_paths; ++p) {
        const int src = n - delays[p];
        if (src < 0) continue;
        const V* cc = jc + (sb * CH_MAXP + p) * (JK_DEG + 1);
        V H = cc[JK_DEG];
#pragma unroll
        for (int k = JK_DEG - 1; k >= 0; --k) H = mkc(H.x * tau + cc[k].x, H.y * tau + cc[k].y);
        const R gn = gains[p];
        const V hc = sizeof(R) == 8 ? mkc(gn * (H.x * k2), gn * (H.y * k2)) : mkc(H.x * (k2 * gn), H.y * (k2 * gn));
        v = cadd(v, cmul(hc, staged ? xs[src - n0 + CH_HALO] : xf[src]));
      }
      yf[n] = v;
      pw += v.x * v.x + v.y * v.y;
    }
    const R t = block_sum(pw, red);
    if (threadIdx.x == 0) pow_part[((size_t)b * num_rx + rx) * nblk + blk] = t;
    return;
  }
#pragma unroll
  for (int i = 0; i < CH_PER; ++i) {
    const int n = n0 + i * WG + threadIdx.x;
    if (n >= L) break;
    V v = mkc((R)0, (R)0);
    if (!rayleigh) {
      v = xf[n];
    } else {
      for (int p = 0; p < n_paths; ++p) {
        const int src = n - delays[p];
        if (src < 0) continue;
        const V c = fD == (R)0 ? coef[cb + p] : jakes_coef<R>(phases + (cb + p) * 16, gains[p], fD, (R)n / fs);
        v = cadd(v, cmul(c, staged ? xs[src - n0 + CH_HALO] : xf[src]));
      }
      yf[n] = v;
    }
    pw += v.x * v.x + v.y * v.y;
  }
  const R t = block_sum(pw, red);
  if (threadIdx.x == 0) pow_part[((size_t)b * num_rx + rx) * nblk + blk] = t;
}

int channel_nblk(int L) { return (L + CH_CHUNK - 1) / CH_CHUNK; }

template <class R>
int launch_channel(hipStream_t s, const Grid& g, int B, int num_rx, int rayleigh, int n_paths,
                   const int32_t* delays_dev, const R* gains_dev, R fD, R fs, const R* phases, const cx<R>* coef,
                   const cx<R>* x, cx<R>* y, R* pow_part, int nblk, int max_delay) {
  if (nblk != channel_nblk(g.L)) return (int)hipErrorInvalidValue;
  // f32 staging uses 16-B pairs: every frame's stream must start 16-B aligned (L even)
  const int staged = rayleigh && max_delay >= 0 && max_delay <= CH_HALO && (sizeof(R) == 8 || (g.L & 1) == 0);
  int SL = 0;   // Taylor sub-interval of the time-varying taps (0: the per-sample sum)
  if (rayleigh && fD != (R)0 && n_paths <= CH_MAXP && phases) {
    SL = CH_CHUNK;
    while (SL >= JK_MINSL && 6.283185307179586 * std::fabs((double)fD) * (SL / 2) / (double)fs > 2.7e-3) SL /= 2;
    if (SL < JK_MINSL) SL = 0;
  }
  const size_t shm = SL ? (size_t)(CH_CHUNK / SL) * CH_MAXP * (JK_DEG + 1) * sizeof(cx<R>) : 0;
  hipLaunchKernelGGL(k_channel<R>, dim3(nblk * B, num_rx), dim3(WG), shm, s, g.L, num_rx, rayleigh, n_paths,
                     delays_dev, gains_dev, fD, fs, phases, coef, x, y, pow_part, nblk, staged, SL);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// RX helpers
template <class R>
__device__ __forceinline__ R frame_power(const R* pp, int nblk, int L) {
  R t = (R)0;
  for (int i = 0; i < nblk; ++i) t += pp[i];
  return t / (R)L;
}

// ---------------------------------------------------------------------------
// Channel estimation: one slot per (frame, rx, 14-symbol group) on the group's
// first symbol (LTEReceiver._estimate_channel_periodic lte_receiver.py:360-411,
// LTEChannelEstimator.estimate_channel :40-96, _interpolate_channel :98-133:
// np.linspace between pilots = j * ((v1 - v0) * (1/gap)) + v0, NumPy's complex
// / real divide being a multiply by the reciprocal).
template <class R, int NC = 0>
__global__ __launch_bounds__(WG) void k_rx_chest(Grid g, int B, int num_rx, const cx<R>* __restrict__ y,
                                                 int64_t y_rx_stride, int64_t y_frame_stride,
                                                 const R* __restrict__ npow_in, const uint64_t* __restrict__ fid,
                                                 uint64_t seed, const R* __restrict__ inj_z, int64_t inj_stride,
                                                 cx<R>* __restrict__ H, R* __restrict__ pstats) {
  using V = cx<R>;
  using G = GridT<R>;
  V* sm = dyn_lds<V>();
  const int N = NC ? NC : g.N, T = N >> 3, spw = WG / T;
  const int slot = threadIdx.x / T, tid = threadIdx.x % T;
  const int64_t gs = (int64_t)blockIdx.x * spw + slot;
  const int per = num_rx * g.n_grp;
  const int b = (int)(gs / per), rr = (int)(gs % per), rx = rr / g.n_grp, grp = rr % g.n_grp;
  const bool active = slot < spw && b < B;
  V* buf = sm + slot * N;
  V* hp = sm + spw * N + slot * g.Np;
  if (active) {
    const R sigma = sqrt(npow_in[(size_t)b * num_rx + rx] / (R)2);
    const R* zf = inj_z ? inj_z + (size_t)b * inj_stride + (size_t)rx * 2 * g.L : nullptr;
    load_symbol_noisy(buf, y + b * y_frame_stride + rx * y_rx_stride, N, g.cp, grp * 14, sigma, seed, fid[b], rx,
                      zf, g.L, tid, T);
  }
  __syncthreads();
  fft_lds<false, NC>(buf, N, g.log2N, G::tw(g), tid, active);
  if (active) {
    const R sc = rx_scale<R>(N);
    for (int p = tid; p < g.Np; p += T) {
      const V Y = cscale(buf[g.pilot_idx[p]], sc);
      hp[p] = cdiv(Y, G::pilots(g)[p]);
      buf[g.pilot_idx[p]] = Y;  // keep scaled pilots for the SNR stats
    }
  }
  __syncthreads();
  if (active) {
    V* Hf = H + (((size_t)b * num_rx + rx) * g.n_grp + grp) * N;
    for (int k = tid; k < N; k += T) {
      const int sidx = g.seg[k];
      V h;
      if (sidx < 0) h = hp[0];
      else if (sidx >= g.Np - 1) h = hp[g.Np - 1];
      else {
        const V v0 = hp[sidx], v1 = hp[sidx + 1];
        const R fk = (R)(k - g.pilot_idx[sidx]);
        const R ig = G::inv_gap(g)[sidx];
        h = mkc(fk * ((v1.x - v0.x) * ig) + v0.x, fk * ((v1.y - v0.y) * ig) + v0.y);
      }
      Hf[k] = h;
    }
    if (tid == 0) {
      R pp = (R)0, en = (R)0;
      for (int p = 0; p < g.Np; ++p) {
        const V Y = buf[g.pilot_idx[p]], X = G::pilots(g)[p];
        pp += Y.x * Y.x + Y.y * Y.y;
        const V d = csub(Y, X);
        en += d.x * d.x + d.y * d.y;
      }
      R* st = pstats + (((size_t)b * num_rx + rx) * g.n_grp + grp) * 2;
      st[0] = pp / (R)g.Np;
      st[1] = en / (R)g.Np;
    }
  }
}

// per (frame, rx): P = mean |y|^2 over the stream, noise power = P / SNR (channel.py:44-53, 217-224)
template <class R>
__global__ void k_npow(int B, int num_rx, const R* __restrict__ pow_part, int nblk, int L,
                       const R* __restrict__ snr_lin, R* __restrict__ npow) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * num_rx) return;
  npow[i] = frame_power(pow_part + (size_t)i * nblk, nblk, L) / snr_lin[i / num_rx];
}

template <class R>
int launch_npow(hipStream_t s, int B, int num_rx, const R* pow_part, int nblk, int L, const R* snr_lin, R* npow) {
  hipLaunchKernelGGL(k_npow<R>, dim3((B * num_rx + WG - 1) / WG), dim3(WG), 0, s, B, num_rx, pow_part, nblk, L,
                     snr_lin, npow);
  return (int)hipGetLastError();
}

template <class R>
int launch_rx_chest(hipStream_t s, const Grid& g, int B, int num_rx, const cx<R>* y, int64_t y_rx_stride,
                    int64_t y_frame_stride, const R* npow, const uint64_t* fid, uint64_t seed, const R* inj_z,
                    int64_t inj_stride, cx<R>* H, R* pstats) {
  const int spw = WG / (g.N >> 3);
  const int64_t total = (int64_t)B * num_rx * g.n_grp;
  const int blocks = (int)((total + spw - 1) / spw);
  const size_t shm = (size_t)spw * (g.N + g.Np) * sizeof(cx<R>);
  if (g.N == 2048)
    hipLaunchKernelGGL((k_rx_chest<R, 2048>), dim3(blocks), dim3(WG), shm, s, g, B, num_rx, y, y_rx_stride,
                       y_frame_stride, npow, fid, seed, inj_z, inj_stride, H, pstats);
  else
    hipLaunchKernelGGL((k_rx_chest<R, 0>), dim3(blocks), dim3(WG), shm, s, g, B, num_rx, y, y_rx_stride,
                       y_frame_stride, npow, fid, seed, inj_z, inj_stride, H, pstats);
  return (int)hipGetLastError();
}

// float32 |h|^2 never contracted: rounded products, then their sum, in every
// instance (left to the compiler, one receiver instance formed it as an FMA and
// another not, and their f32 sigma^2_eff -- hence LLRs -- parted by an ulp)
__device__ __forceinline__ float abs2_nc(float2 h) {
#pragma clang fp contract(off)
  return h.x * h.x + h.y * h.y;
}
// |h|^2 as the reference forms it: f64 np.abs(h) ** 2 (hypot, then squared);
// f32 h.x^2 + h.y^2
template <class V>
__device__ __forceinline__ re_t<V> abs2_ref(V h) {
  if constexpr (sizeof(re_t<V>) == 8) {
    const double a = hypot(h.x, h.y);
    return a * a;
  } else {
    return abs2_nc(h);
  }
}

// ---------------------------------------------------------------------------
// Hard decision / soft demap.  Natural-binary QAM, I-level-major index
// (modulator.py:28-59, Q9): bits = [I-level bits | Q-level bits], MSB first.
// ---------------------------------------------------------------------------
// Data path: one slot per (frame, OFDM symbol).  Per RX: CP-remove + noise +
// FFT/sqrt(N) (lte_receiver.py:444-491); then
//  UNCODED: ZF Y/(H+1e-6) (lte_receiver.py:154-180) -> hard bits -> bit errors
//  CODED:   ZF -> sigma2_eff (ofdm_core.py:1224-1243) -> LLRs (RE order)
//  SIMO:    MRC sum conj(H_i)Y_i / (sum|H_i|^2 + 1e-10) (ofdm_core.py:1405-1534)
// Templated on chain and bits/symbol so every per-RE array stays in VGPRs.
//  SCF (SC-FDM, UNCODED): the ZF outputs of the symbol's Nd data REs go
//       through the M = Nd IDFT (core/lte_receiver.py:318-333) before slicing.
template <class R, int CHAIN, int BPS, bool SCF = false, int NC = 0>
__global__ __launch_bounds__(WG) void k_rx_data(Grid g, int rayleigh, int B, int num_rx,
                                                const cx<R>* __restrict__ y, int64_t y_rx_stride,
                                                int64_t y_frame_stride, const cx<R>* __restrict__ H,
                                                const R* __restrict__ npow, const R* __restrict__ snr_lin,
                                                const uint64_t* __restrict__ fid, uint64_t seed,
                                                const R* __restrict__ inj_z, int64_t inj_stride,
                                                const uint32_t* __restrict__ pw, int PW, int n_bits,
                                                uint32_t* __restrict__ frame_err, R* __restrict__ llr,
                                                cx<R>* __restrict__ cap_syms, uint8_t* __restrict__ cap_bits,
                                                R* __restrict__ nvo) {
  using V = cx<R>;
  using G = GridT<R>;
  V* sm = dyn_lds<V>();
  const int N = NC ? NC : g.N, T = N >> 3, spw = WG / T;
  const int slot = threadIdx.x / T, tid = threadIdx.x % T;
  const int gs = blockIdx.x * spw + slot;
  const int b = gs / g.n_sym, l = gs - b * g.n_sym;
  const bool active = slot < spw && b < B;
  V* buf = sm + slot * N;
  const int grp = l / 14;
  const R sc = rx_scale<R>(N);
  constexpr R QS = (R)qam_norm<BPS>();
  constexpr int QM = 4;  // data REs per thread (Nd < N/2 for every LTE profile)
  constexpr int NRX = CHAIN == LTE_CHAIN_SIMO ? 8 : 1;
  V num[QM];
  R den[QM];
#pragma unroll
  for (int q = 0; q < QM; ++q) { num[q] = mkc((R)0, (R)0); den[q] = (R)0; }
  for (int rx = 0; rx < (NRX == 1 ? 1 : num_rx); ++rx) {
    if (active) {
      const R sigma = sqrt(npow[(size_t)b * num_rx + rx] / (R)2);
      const R* zf = inj_z ? inj_z + (size_t)b * inj_stride + (size_t)rx * 2 * g.L : nullptr;
      load_symbol_noisy2<true>(buf, y + b * y_frame_stride + rx * y_rx_stride, N, g.cp, l, sigma, seed, fid[b], rx,
                               zf, g.L, tid, T);
    }
    __syncthreads();
    fft_lds<false, NC, false, (NC > 0), true>(buf, N, g.log2N, G::tw(g), tid, active);
    if (active) {
      const V* Hf = H + (((size_t)b * num_rx + rx) * g.n_grp + grp) * N;
#pragma unroll
      for (int q = 0; q < QM; ++q) {
        const int j = tid + q * T;
        if (j < g.Nd) {
          const int k = g.data_idx[j];
          const V Y = cscale(buf[k], sc), h = Hf[k];
          if constexpr (CHAIN == LTE_CHAIN_SIMO) {
            num[q] = cadd(num[q], cmulc(Y, h));
            den[q] += abs2_ref(h);
          } else {
            num[q] = (CHAIN == LTE_CHAIN_UNCODED && g.no_eq) ? Y : zf_eq(Y, h);
            den[q] = abs2_ref(h);
          }
        }
      }
    }
    if constexpr (NRX > 1) __syncthreads();
  }
  if constexpr (SCF) {   // IDFT(z) = conj(DFT(conj(z))) over the Nd data REs, in the (consumed) FFT buffer
    __syncthreads();
    if (active) {
#pragma unroll
      for (int q = 0; q < QM; ++q) {
        const int j = tid + q * T;
        if (j < g.Nd) buf[j] = mkc(num[q].x, -num[q].y);
      }
      for (int k = g.Nd + tid; k < N; k += T) buf[k] = mkc((R)0, (R)0);
    }
    dft_bluestein(buf, g, tid, T, active);
    if (active) {
#pragma unroll
      for (int q = 0; q < QM; ++q) {
        const int j = tid + q * T;
        if (j < g.Nd) num[q] = mkc(buf[j].x, -buf[j].y);
      }
    }
  }
  uint32_t errs = 0;
  const uint32_t* fb = pw + (size_t)b * PW;
  const size_t fre = (size_t)b * g.n_sym * g.Nd;
#pragma unroll
  for (int q = 0; q < QM; ++q) {
    const int j = tid + q * T;
    if (!active || j >= g.Nd) continue;
    const int re = l * g.Nd + j;
    V z = num[q];
    if constexpr (CHAIN == LTE_CHAIN_SIMO) {
      const R r = (R)1 / (den[q] + (R)1e-10);
      z = mkc(z.x * r, z.y * r);
    }
    if (cap_syms) cap_syms[fre + re] = z;
    if constexpr (CHAIN == LTE_CHAIN_CODED) {
      const R s2 = (R)1 / snr_lin[b];
      R nv = s2;
      if (rayleigh) nv = fmax(s2 / fmin(fmax(den[q], (R)1e-6), (R)1e6), s2 / (R)4);
      if (nvo) {   // demap in k_dematch_zn: the equalised symbol and sigma^2_eff per (group, subcarrier)
        reinterpret_cast<V*>(llr)[fre + re] = z;
        nvo[((size_t)b * g.n_grp + grp) * g.Nd + j] = nv;
        continue;
      }
      R o[BPS];
      soft_demap<BPS>(z, nv, o);
      R* lo = llr + (fre + re) * BPS;
      if constexpr (BPS == 4 && sizeof(R) == 4) {
        *reinterpret_cast<float4*>(lo) = make_float4(o[0], o[1], o[2], o[3]);
      } else {
#pragma unroll
        for (int m = 0; m < BPS; m += 2) *reinterpret_cast<V*>(lo + m) = mkc(o[m], o[m + 1]);
      }
    } else {
      const int idx = hard_index(z, BPS, QS);
      const int64_t pb0 = (int64_t)re * BPS;
      errs += __popc(((uint32_t)idx ^ getbits<BPS>(fb, pb0, n_bits)) & bits_valid<BPS>(pb0, n_bits));
      if (cap_bits) {
#pragma unroll
        for (int m = 0; m < BPS; ++m)
          if (pb0 + m < n_bits) cap_bits[(size_t)b * n_bits + pb0 + m] = (uint8_t)((idx >> (BPS - 1 - m)) & 1);
      }
    }
  }
  // one atomic per frame per wave (all lanes reach this point; inactive lanes carry 0)
  if constexpr (CHAIN != LTE_CHAIN_CODED) frame_err_add(frame_err, b, errs);
}

// ---------------------------------------------------------------------------
// Fused SISO receiver: one slot per frame walks its OFDM symbols in order; the
// first symbol of each 14-symbol group also yields the group's LS estimate
// (k_rx_chest's work on the FFT the data path needs anyway), and the per-
// subcarrier equaliser terms -- NumPy's complex division by H + 1e-6 reduced
// to its per-subcarrier ratio / scale (ZfCoef), and sigma^2_eff -- are formed
// once per group in registers for the thread's data subcarriers instead of per
// RE.  H is never re-read from HBM (written only for a capture).  Same
// arithmetic per RE as k_rx_chest + k_rx_data (parity test
// test_fused_receiver_matches_separate_kernels).
template <class R> struct ZfCoef;
template <> struct ZfCoef<double> {   // cdiv(y, h) (Smith, lte_common.h) with the h-only terms precomputed
  double rat, sre, sim;
  bool swp;
  __device__ __forceinline__ void set(double2 h) {
    swp = !(fabs(h.x) >= fabs(h.y));
    if (!swp) {
      rat = (h.x == 0.0 && h.y == 0.0) ? 0.0 : h.y / h.x;   // h = 0: a / 0 as cdiv
      sre = sim = (h.x == 0.0 && h.y == 0.0) ? 1.0 / h.x : 1.0 / (h.x + h.y * rat);
    } else {
      rat = h.x / h.y;
      sre = 1.0 / (h.y + h.x * rat);
      sim = -sre;
    }
  }
  // !swp: ((a.x + a.y rat) s, (a.y - a.x rat) s); swp: ((a.x rat + a.y) s, (a.y rat - a.x) s)
  __device__ __forceinline__ double2 apply(double2 a) const {
    const double u = swp ? a.x : a.y, v = swp ? a.y : a.x;
    return make_double2((v + u * rat) * sre, (u - v * rat) * sim);
  }
};
template <> struct ZfCoef<float> {    // zf_div(y, h): y conj(h) / |h|^2
  float2 h;
  float r;
  __device__ __forceinline__ void set(float2 hh) {
    h = hh;
    r = 1.0f / (hh.x * hh.x + hh.y * hh.y);
  }
  __device__ __forceinline__ float2 apply(float2 y) const {
    return make_float2((y.x * h.x + y.y * h.y) * r, (y.y * h.x - y.x * h.y) * r);
  }
};

// linear interpolation of the pilot LS estimates hp at subcarrier k with edge
// hold (lte_receiver.py:114-133), as k_rx_chest forms it
template <class R>
__device__ __forceinline__ cx<R> chest_interp(const Grid& g, const cx<R>* hp, int k) {
  using V = cx<R>;
  const int sidx = g.seg[k];
  if (sidx < 0) return hp[0];
  if (sidx >= g.Np - 1) return hp[g.Np - 1];
  const V v0 = hp[sidx], v1 = hp[sidx + 1];
  const R fk = (R)(k - g.pilot_idx[sidx]);
  const R ig = GridT<R>::inv_gap(g)[sidx];
  return mkc(fk * ((v1.x - v0.x) * ig) + v0.x, fk * ((v1.y - v0.y) * ig) + v0.y);
}

#ifndef RXF_EXP
#define RXF_EXP 0
#endif
#ifndef RXF_WAVES
#define RXF_WAVES 3
#endif
// ZN (coded, the default): the equalised symbols go to k_dematch_zn and the
// per-subcarrier sigma^2_eff to nvo at each estimate, so no per-RE noise
// variance stays live across the symbol loop (8 VGPRs of the f64 instance)
template <class R, int CHAIN, int BPS, int NC = 0, bool ZN = false>
__global__ __launch_bounds__(WG, RXF_WAVES) void k_rx_frame(Grid g, int rayleigh, int B, const cx<R>* __restrict__ y,
                                                 int64_t y_frame_stride, const R* __restrict__ npow,
                                                 const R* __restrict__ snr_lin, const uint64_t* __restrict__ fid,
                                                 uint64_t seed, const R* __restrict__ inj_z, int64_t inj_stride,
                                                 const uint32_t* __restrict__ pw, int PW, int n_bits,
                                                 uint32_t* __restrict__ frame_err, R* __restrict__ llr,
                                                 cx<R>* __restrict__ cap_syms, uint8_t* __restrict__ cap_bits,
                                                 R* __restrict__ nvo, cx<R>* __restrict__ H, R* __restrict__ pstats) {
  using V = cx<R>;
  using G = GridT<R>;
  V* sm = dyn_lds<V>();
  const int N = NC ? NC : g.N, T = N >> 3, spw = WG / T;
  const int slot = threadIdx.x / T, tid0 = threadIdx.x % T;
  const int b = blockIdx.x * spw + slot;
  const bool active = slot < spw && b < B;
  V* buf = sm + slot * (N + g.Np);
  V* hp = buf + N;
  const R sc = rx_scale<R>(N);
  constexpr R QS = (R)qam_norm<BPS>();
  constexpr int QM = 4;   // data REs per thread (Nd < N/2 for every LTE profile)
  const R sigma = active ? sqrt(npow[b] / (R)2) : (R)0;
  const R s2 = active ? (R)1 / snr_lin[b] : (R)1;
  const uint64_t fr = active ? fid[b] : 0ull;
  const R* zf = (inj_z && active) ? inj_z + (size_t)b * inj_stride : nullptr;
  const V* yf = y + (size_t)(active ? b : 0) * y_frame_stride;
  const uint32_t* fb = pw + (size_t)(active ? b : 0) * PW;
  const size_t fre = (size_t)(active ? b : 0) * g.n_sym * g.Nd;
  int kpos[QM];
#pragma unroll
  for (int q = 0; q < QM; ++q) {
    const int j = tid0 + q * T;
    kpos[q] = (active && j < g.Nd) ? g.data_idx[j] : 0;
#if LTE_LDS_PROBE & 1   // timing probe only (wrong outputs): conflict-free RE positions
    kpos[q] = (active && j < g.Nd) ? N / 2 - 512 + j : 0;
#endif
  }
  ZfCoef<R> zc[QM];
  R nvq[QM];
  uint32_t errs = 0;
  LTE_BM_LDS_DECL(R);
  const auto bmt = bm_stage<R>(lte_bmt);
  __syncthreads();
  for (int l = 0; l < g.n_sym; ++l) {
    // tid made opaque per symbol: the FFT / loader address arithmetic derived
    // from it is recomputed each symbol instead of hoisted and held live
    // across the loop (which took the kernel to 255 VGPRs)
    int tid = tid0;
    asm volatile("" : "+v"(tid));
    if (active) load_symbol_noisy2<true>(buf, yf, N, g.cp, l, sigma, seed, fr, 0, zf, g.L, tid, T, bmt);
    __syncthreads();
    fft_lds<false, NC, false, (NC > 0), true>(buf, N, g.log2N, G::tw(g), tid, active);
    if (l % 14 == 0) {   // group estimate from its first symbol (lte_receiver.py:360-411)
      const int grp = l / 14;
      if (active)
        for (int p = tid; p < g.Np; p += T) {
          const V Y = cscale(buf[g.pilot_idx[p]], sc);
          hp[p] = cdiv(Y, G::pilots(g)[p]);
          buf[g.pilot_idx[p]] = Y;   // scaled pilots for the SNR stats
        }
      __syncthreads();
      if (active) {
        if (RXF_EXP != 1 && H) {
          V* Hf = H + ((size_t)b * g.n_grp + grp) * N;
          for (int k = tid; k < N; k += T) Hf[k] = chest_interp<R>(g, hp, k);
        }
#pragma unroll
        for (int q = 0; q < QM; ++q) {
          const int j = tid + q * T;
          if (j < g.Nd) {
            const V h = chest_interp<R>(g, hp, kpos[q]);
            zc[q].set(mkc(h.x + (R)1e-6, h.y));
            const R den = abs2_ref(h);
            const R nv = rayleigh ? fmax(s2 / fmin(fmax(den, (R)1e-6), (R)1e6), s2 / (R)4) : s2;
            if constexpr (ZN) nvo[((size_t)b * g.n_grp + grp) * g.Nd + j] = nv;
            else nvq[q] = nv;
          }
        }
        if (RXF_EXP != 1 && pstats && tid == 0) {
          R pp = (R)0, en = (R)0;
          for (int p = 0; p < g.Np; ++p) {
            const V Yp = buf[g.pilot_idx[p]], X = G::pilots(g)[p];
            pp += Yp.x * Yp.x + Yp.y * Yp.y;
            const V d = csub(Yp, X);
            en += d.x * d.x + d.y * d.y;
          }
          R* st = pstats + ((size_t)b * g.n_grp + grp) * 2;
          st[0] = pp / (R)g.Np;
          st[1] = en / (R)g.Np;
        }
      }
    }
    if (active) {
#pragma unroll
      for (int q = 0; q < QM; ++q) {
        const int j = tid + q * T;
        if (j >= g.Nd) continue;
        const int re = l * g.Nd + j;
        const V Y = cscale(buf[kpos[q]], sc);
        const V z = (CHAIN == LTE_CHAIN_UNCODED && g.no_eq) ? Y : zc[q].apply(Y);
        if (cap_syms) cap_syms[fre + re] = z;
        if constexpr (CHAIN == LTE_CHAIN_CODED && ZN) {
          // demap in k_dematch_zn: the equalised symbol (sigma^2_eff per subcarrier in nvo)
          reinterpret_cast<V*>(llr)[fre + re] = z;
        } else if constexpr (CHAIN == LTE_CHAIN_CODED) {
          R o[BPS];
          soft_demap<BPS>(z, nvq[q], o);
          R* lo = llr + (fre + re) * BPS;
          if constexpr (BPS == 4 && sizeof(R) == 4) {
            *reinterpret_cast<float4*>(lo) = make_float4(o[0], o[1], o[2], o[3]);
          } else {
#pragma unroll
            for (int m = 0; m < BPS; m += 2) *reinterpret_cast<V*>(lo + m) = mkc(o[m], o[m + 1]);
          }
        } else {
          const int idx = hard_index(z, BPS, QS);
          const int64_t pb0 = (int64_t)re * BPS;
          errs += __popc(((uint32_t)idx ^ getbits<BPS>(fb, pb0, n_bits)) & bits_valid<BPS>(pb0, n_bits));
          if (cap_bits) {
#pragma unroll
            for (int m = 0; m < BPS; ++m)
              if (pb0 + m < n_bits) cap_bits[(size_t)b * n_bits + pb0 + m] = (uint8_t)((idx >> (BPS - 1 - m)) & 1);
          }
        }
      }
    }
    __syncthreads();   // every read of buf done before the next symbol lands in it
  }
  if constexpr (CHAIN != LTE_CHAIN_CODED) frame_err_add(frame_err, b, errs);
}

bool rx_frame_supported(const Grid& g, int chain, int num_rx, int sc_fdm) {
  return num_rx == 1 && !sc_fdm && (chain == LTE_CHAIN_CODED || chain == LTE_CHAIN_UNCODED) &&
         (g.bps == 2 || g.bps == 4 || g.bps == 6) && 2 * g.Nd < g.N;
}

template <class R>
int launch_rx_frame(hipStream_t s, const Grid& g, int chain, int rayleigh, int B, const cx<R>* y,
                    int64_t y_frame_stride, const R* npow, const R* snr_lin, const uint64_t* fid, uint64_t seed,
                    const R* inj_z, int64_t inj_stride, const uint32_t* pw, int PW, int n_bits, uint32_t* frame_err,
                    R* llr, cx<R>* cap_syms, uint8_t* cap_bits, R* nv_out, cx<R>* H, R* pstats) {
  if (!rx_frame_supported(g, chain, 1, 0) || (nv_out && chain != LTE_CHAIN_CODED)) return (int)hipErrorInvalidValue;
  if constexpr (sizeof(R) == 8)
    if (nv_out && rx_frame_w_supported(g, chain, 1) && rx_wave_enabled())
      return launch_rx_frame_w(s, g, rayleigh, B, y, y_frame_stride, npow, snr_lin, fid, seed, inj_z, inj_stride,
                               llr, nv_out, cap_syms, H, pstats);
  const int spw = WG / (g.N >> 3);
  const int blocks = (B + spw - 1) / spw;
  const size_t shm = (size_t)spw * (g.N + g.Np) * sizeof(cx<R>);
#define LTE_RXF(CH_, BPS_, NC_)                                                                                      \
  do {                                                                                                               \
    if (CH_ == LTE_CHAIN_CODED && nv_out)                                                                            \
      hipLaunchKernelGGL((k_rx_frame<R, CH_, BPS_, NC_, CH_ == LTE_CHAIN_CODED>), dim3(blocks), dim3(WG), shm, s, g, rayleigh, B, y,   \
                         y_frame_stride, npow, snr_lin, fid, seed, inj_z, inj_stride, pw, PW, n_bits, frame_err,    \
                         llr, cap_syms, cap_bits, nv_out, H, pstats);                                                \
    else                                                                                                             \
      hipLaunchKernelGGL((k_rx_frame<R, CH_, BPS_, NC_>), dim3(blocks), dim3(WG), shm, s, g, rayleigh, B, y,         \
                         y_frame_stride, npow, snr_lin, fid, seed, inj_z, inj_stride, pw, PW, n_bits, frame_err,    \
                         llr, cap_syms, cap_bits, nv_out, H, pstats);                                                \
  } while (0)
#define LTE_RXF_BPS(CH_, NC_)                                                                                        \
  do {                                                                                                               \
    if (g.bps == 2) LTE_RXF(CH_, 2, NC_);                                                                            \
    else if (g.bps == 4) LTE_RXF(CH_, 4, NC_);                                                                       \
    else LTE_RXF(CH_, 6, NC_);                                                                                       \
  } while (0)
  if (chain == LTE_CHAIN_CODED) {
    if (g.N == 2048) LTE_RXF_BPS(LTE_CHAIN_CODED, 2048);   // the headline chain
    else LTE_RXF_BPS(LTE_CHAIN_CODED, 0);
  } else {
    if (g.N == 2048) LTE_RXF_BPS(LTE_CHAIN_UNCODED, 2048);
    else LTE_RXF_BPS(LTE_CHAIN_UNCODED, 0);
  }
#undef LTE_RXF_BPS
#undef LTE_RXF
  return (int)hipGetLastError();
}

// Fused SIMO MRC receiver (simulate_simo, core/ofdm_core.py:1405-1534): one
// slot per frame walks its OFDM symbols; per symbol every RX in turn is loaded
// with its noise, FFT'd and folded into the MRC sums sum_r conj(H_r) Y_r /
// (sum_r |H_r|^2 + 1e-10), RX 0 first as k_rx_data sums them.  The first symbol
// of each 14-symbol group also yields every RX's LS pilot estimates, kept in
// LDS per RX (k_rx_chest's work on the FFT the data path needs anyway); each
// RE's estimate is interpolated from them per symbol with the thread's
// per-subcarrier segment / offset / 1-over-gap held in registers (chest_interp's
// expression), so no per-RX estimate occupies registers.  Same arithmetic per
// RE as k_rx_chest + k_rx_data<SIMO> (test_fused_simo_receiver_matches_separate_kernels).
template <class R>
__device__ __forceinline__ cx<R> interp_seg(const cx<R>* hp, int np, int sidx, R fk, R ig) {
  if (sidx < 0) return hp[0];
  if (sidx >= np - 1) return hp[np - 1];
  const cx<R> v0 = hp[sidx], v1 = hp[sidx + 1];
  return mkc(fk * ((v1.x - v0.x) * ig) + v0.x, fk * ((v1.y - v0.y) * ig) + v0.y);
}

template <class R, int BPS, int NC = 0>
__global__ __launch_bounds__(WG, RXF_WAVES) void k_rx_frame_simo(
    Grid g, int B, int num_rx, const cx<R>* __restrict__ y, int64_t y_rx_stride, int64_t y_frame_stride,
    const R* __restrict__ npow, const uint64_t* __restrict__ fid, uint64_t seed, const R* __restrict__ inj_z,
    int64_t inj_stride, const uint32_t* __restrict__ pw, int PW, int n_bits, uint32_t* __restrict__ frame_err,
    cx<R>* __restrict__ cap_syms, uint8_t* __restrict__ cap_bits, cx<R>* __restrict__ H, R* __restrict__ pstats) {
  using V = cx<R>;
  using G = GridT<R>;
  V* sm = dyn_lds<V>();
  const int N = NC ? NC : g.N, T = N >> 3, spw = WG / T;
  const int slot = threadIdx.x / T, tid0 = threadIdx.x % T;
  const int b = blockIdx.x * spw + slot;
  const bool active = slot < spw && b < B;
  V* buf = sm + slot * (N + RXS_MAXRX * g.Np);
  V* hpa = buf + N;   // [RXS_MAXRX][Np] pilot LS estimates of the current group
  const R sc = rx_scale<R>(N);
  constexpr R QS = (R)qam_norm<BPS>();
  constexpr int QM = 4;   // data REs per thread (Nd < N/2 for every LTE profile)
  const uint64_t fr = active ? fid[b] : 0ull;
  const V* yf = y + (size_t)(active ? b : 0) * y_frame_stride;
  const uint32_t* fb = pw + (size_t)(active ? b : 0) * PW;
  const size_t fre = (size_t)(active ? b : 0) * g.n_sym * g.Nd;
  int kpos[QM], sg[QM];
  R fk[QM], ig[QM];
#pragma unroll
  for (int q = 0; q < QM; ++q) {   // chest_interp's per-subcarrier terms
    const int j = tid0 + q * T;
    kpos[q] = (active && j < g.Nd) ? g.data_idx[j] : 0;
    sg[q] = g.seg[kpos[q]];
    const int sc_ = sg[q] < 0 ? 0 : (sg[q] >= g.Np - 1 ? g.Np - 1 : sg[q]);
    fk[q] = (R)(kpos[q] - g.pilot_idx[sc_]);
    ig[q] = GridT<R>::inv_gap(g)[sc_];
  }
  R den[QM];
#pragma unroll
  for (int q = 0; q < QM; ++q) den[q] = (R)0;
  uint32_t errs = 0;
  LTE_BM_LDS_DECL(R);
  const auto bmt = bm_stage<R>(lte_bmt);
  __syncthreads();
  for (int l = 0; l < g.n_sym; ++l) {
    const bool est = l % 14 == 0;
    const int grp = l / 14;
    V num[QM];
#pragma unroll
    for (int q = 0; q < QM; ++q) num[q] = mkc((R)0, (R)0);
    if (est) {
#pragma unroll
      for (int q = 0; q < QM; ++q) den[q] = (R)0;
    }
    for (int rx = 0; rx < num_rx; ++rx) {
      int tid = tid0;   // opaque per pass (see k_rx_frame)
      asm volatile("" : "+v"(tid));
      if (active) {
        const R sigma = sqrt(npow[(size_t)b * num_rx + rx] / (R)2);
        const R* zf = inj_z ? inj_z + (size_t)b * inj_stride + (size_t)rx * 2 * g.L : nullptr;
        load_symbol_noisy2<true>(buf, yf + rx * y_rx_stride, N, g.cp, l, sigma, seed, fr, rx, zf, g.L, tid, T, bmt);
      }
      __syncthreads();
      fft_lds<false, NC, false, (NC > 0), true>(buf, N, g.log2N, G::tw(g), tid, active);
      V* hp = hpa + rx * g.Np;
      if (est) {   // this RX's group estimate from the group's first symbol (lte_receiver.py:360-411)
        if (active)
          for (int p = tid; p < g.Np; p += T) {
            const V Y = cscale(buf[g.pilot_idx[p]], sc);
            hp[p] = cdiv(Y, G::pilots(g)[p]);
            buf[g.pilot_idx[p]] = Y;   // scaled pilots for the SNR stats
          }
        __syncthreads();
        if (active) {
          const size_t hr = ((size_t)b * num_rx + rx) * g.n_grp + grp;
          if (H) {
            V* Hf = H + hr * N;
            for (int k = tid; k < N; k += T) Hf[k] = chest_interp<R>(g, hp, k);
          }
#pragma unroll
          for (int q = 0; q < QM; ++q) {
            const int j = tid + q * T;
            if (j < g.Nd) den[q] += abs2_ref(interp_seg<R>(hp, g.Np, sg[q], fk[q], ig[q]));
          }
          if (pstats && tid == 0) {
            R pp = (R)0, en = (R)0;
            for (int p = 0; p < g.Np; ++p) {
              const V Yp = buf[g.pilot_idx[p]], X = G::pilots(g)[p];
              pp += Yp.x * Yp.x + Yp.y * Yp.y;
              const V d = csub(Yp, X);
              en += d.x * d.x + d.y * d.y;
            }
            pstats[hr * 2] = pp / (R)g.Np;
            pstats[hr * 2 + 1] = en / (R)g.Np;
          }
        }
      }
      if (active) {
#pragma unroll
        for (int q = 0; q < QM; ++q) {
          const int j = tid + q * T;
          if (j < g.Nd)
            num[q] = cadd(num[q], cmulc(cscale(buf[kpos[q]], sc), interp_seg<R>(hp, g.Np, sg[q], fk[q], ig[q])));
        }
      }
      __syncthreads();   // every read of buf done before the next RX / symbol lands in it
    }
    if (active) {
#pragma unroll
      for (int q = 0; q < QM; ++q) {
        const int j = tid0 + q * T;
        if (j >= g.Nd) continue;
        const int re = l * g.Nd + j;
        const R rr = (R)1 / (den[q] + (R)1e-10);
        const V z = mkc(num[q].x * rr, num[q].y * rr);
        if (cap_syms) cap_syms[fre + re] = z;
        const int idx = hard_index(z, BPS, QS);
        const int64_t pb0 = (int64_t)re * BPS;
        errs += __popc(((uint32_t)idx ^ getbits<BPS>(fb, pb0, n_bits)) & bits_valid<BPS>(pb0, n_bits));
        if (cap_bits) {
#pragma unroll
          for (int m = 0; m < BPS; ++m)
            if (pb0 + m < n_bits) cap_bits[(size_t)b * n_bits + pb0 + m] = (uint8_t)((idx >> (BPS - 1 - m)) & 1);
        }
      }
    }
  }
  frame_err_add(frame_err, b, errs);
}

// k_rx_frame_simo2<.., XIN>'s loader: RX rx's N samples of symbol l formed
// from the TX symbol xs (LDS, natural order) with tx_channel's taps in its
// order -- y[n] = sum_p c_rp x[(n - d_p) mod N]: every delay is within the CP,
// so the received samples past the CP are a cyclic convolution of the symbol
// -- plus the noise exactly as load_symbol_noisy2 draws it (one Philox per
// sample pair), stored swizzled for fft_lds<.., ISW = true>.
template <class V, class TB>
__device__ __forceinline__ void tap_symbol_noisy2(V* buf, const V* xs, const V (&cf)[TXCH_MAXP],
                                                  const int (&dl)[TXCH_MAXP], int np, int N, int cp, int l,
                                                  re_t<V> sigma, uint64_t seed, uint64_t frame, int rx,
                                                  const re_t<V>* __restrict__ zf, int L, int tid, int T, const TB& tb) {
  using R = re_t<V>;
  const int off = l * (N + cp) + cp;
  auto tap = [&](int n) {
    V v = mkc((R)0, (R)0);
#pragma unroll
    for (int p = 0; p < TXCH_MAXP; ++p)
      if (p < np) v = cadd(v, cmul(cf[p], xs[(n - dl[p]) & (N - 1)]));
    return v;
  };
  if (zf) {
    for (int k = tid; k < N; k += T) {
      const int n = off + k;
      const V v = tap(k);
      buf[fft_sw<V>(k)] = mkc(v.x + sigma * zf[n], v.y + sigma * zf[L + n]);
    }
    return;
  }
  const int p0 = off >> 1, p1 = (off + N - 1) >> 1;
  constexpr int MAXR = 5;
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int p = p0 + tid + i * T, n0 = 2 * p;
    if (p > p1) break;
    const u32x4 r = rng4(seed, frame, RNG_STREAM_NOISE + (uint32_t)rx, (uint32_t)p);
    if (n0 >= off) {
      const V v = tap(n0 - off);
      const V z = gauss2t<R>(r.x, r.y, tb);
      buf[fft_sw<V>(n0 - off)] = mkc(v.x + sigma * z.x, v.y + sigma * z.y);
    }
    if (n0 + 1 < off + N) {
      const V v = tap(n0 + 1 - off);
      const V z = gauss2t<R>(r.z, r.w, tb);
      buf[fft_sw<V>(n0 + 1 - off)] = mkc(v.x + sigma * z.x, v.y + sigma * z.y);
    }
  }
}

// k_rx_frame_simo with the receive antennas in pairs (N = 1024, an even
// number of RX, no capture of H / pilot statistics): one frame per 256-thread
// block; each half loads and transforms one RX of the pair (RX 2p + h) into
// its own buffer, then every thread folds both into its REs' MRC sums in RX
// order -- the same operations per RE as k_rx_frame_simo, with half the
// passes (and barriers) per symbol.
// XIN: the TX handed over its symbols instead of the received streams
// (TxChannelT::x_out): each symbol is staged in LDS once and every RX forms its
// samples with its own taps (tap_symbol_noisy2) -- one stream through HBM
// instead of num_rx, both ways.
template <class R, int BPS, int NC, bool XIN = false>
__global__ __launch_bounds__(WG, RXF_WAVES) void k_rx_frame_simo2(
    Grid g, int B, int num_rx, const cx<R>* __restrict__ y, int64_t y_rx_stride, int64_t y_frame_stride,
    const R* __restrict__ npow, const uint64_t* __restrict__ fid, uint64_t seed, const R* __restrict__ inj_z,
    int64_t inj_stride, const uint32_t* __restrict__ pw, int PW, int n_bits, uint32_t* __restrict__ frame_err,
    cx<R>* __restrict__ cap_syms, uint8_t* __restrict__ cap_bits, TxChannelT<R> xc) {
  using V = cx<R>;
  using G = GridT<R>;
  constexpr int N = NC, T = N >> 3;
  static_assert(2 * T == WG, "one frame per block, one RX per half");
  V* sm = dyn_lds<V>();
  const int half = threadIdx.x / T, th = threadIdx.x % T, tid0 = threadIdx.x;
  const int b = blockIdx.x;
  V* bufs = sm;                  // [2][N]
  V* hpa = sm + 2 * N;           // [RXS_MAXRX][Np] pilot LS estimates of the current group
  V* xs = hpa + RXS_MAXRX * g.Np;   // XIN: [N] the TX symbol
  const R sc = rx_scale<R>(N);
  constexpr R QS = (R)qam_norm<BPS>();
  constexpr int QM = 2;   // data REs per thread (Nd < N/2 = QM WG)
  const uint64_t fr = fid[b];
  const V* yf = y + (size_t)b * y_frame_stride;
  const uint32_t* fb = pw + (size_t)b * PW;
  const size_t fre = (size_t)b * g.n_sym * g.Nd;
  int kpos[QM], sg[QM];
  R fk[QM], ig[QM];
#pragma unroll
  for (int q = 0; q < QM; ++q) {   // chest_interp's per-subcarrier terms
    const int j = tid0 + q * WG;
    kpos[q] = j < g.Nd ? g.data_idx[j] : 0;
    sg[q] = g.seg[kpos[q]];
    const int sc_ = sg[q] < 0 ? 0 : (sg[q] >= g.Np - 1 ? g.Np - 1 : sg[q]);
    fk[q] = (R)(kpos[q] - g.pilot_idx[sc_]);
    ig[q] = GridT<R>::inv_gap(g)[sc_];
  }
  R den[QM];
#pragma unroll
  for (int q = 0; q < QM; ++q) den[q] = (R)0;
  uint32_t errs = 0;
  LTE_BM_LDS_DECL(R);
  const auto bmt = bm_stage<R>(lte_bmt);
  __syncthreads();
  for (int l = 0; l < g.n_sym; ++l) {
    const bool est = l % 14 == 0;
    V num[QM];
#pragma unroll
    for (int q = 0; q < QM; ++q) num[q] = mkc((R)0, (R)0);
    if (est) {
#pragma unroll
      for (int q = 0; q < QM; ++q) den[q] = (R)0;
    }
    if constexpr (XIN) {   // (the previous symbol's last barrier precedes this)
      const V* xo = xc.x_out + ((size_t)b * g.n_sym + l) * N;
      for (int k = tid0; k < N; k += WG) xs[k] = xo[k];
      __syncthreads();
    }
    for (int r0 = 0; r0 < num_rx; r0 += 2) {
      int tid = th;   // opaque per pass (see k_rx_frame)
      asm volatile("" : "+v"(tid));
      const int rx = r0 + half;
      V* buf = bufs + half * N;
      {
        const R sigma = sqrt(npow[(size_t)b * num_rx + rx] / (R)2);
        const R* zf = inj_z ? inj_z + (size_t)b * inj_stride + (size_t)rx * 2 * g.L : nullptr;
        if constexpr (XIN) {   // tx_channel's taps for this RX (f32: the output scale folded in)
          const int np = xc.n_paths;
          V cf[TXCH_MAXP];
          int dl[TXCH_MAXP];
#pragma unroll
          for (int p = 0; p < TXCH_MAXP; ++p) {
            const V c = p < np ? xc.coef[((size_t)b * num_rx + rx) * np + p] : mkc((R)0, (R)0);
            cf[p] = sizeof(R) == 8 ? c : cscale(c, tx_scale<R>(N));
            dl[p] = xc.delays[p];
          }
          tap_symbol_noisy2(buf, xs, cf, dl, np, N, g.cp, l, sigma, seed, fr, rx, zf, g.L, tid, T, bmt);
        } else {
          load_symbol_noisy2<true>(buf, yf + rx * y_rx_stride, N, g.cp, l, sigma, seed, fr, rx, zf, g.L, tid, T, bmt);
        }
      }
      __syncthreads();
      fft_lds<false, NC, false, true, true>(buf, N, g.log2N, G::tw(g), tid, true);
      if (est) {   // this RX's group estimate from the group's first symbol (lte_receiver.py:360-411)
        V* hp = hpa + rx * g.Np;
        for (int p = tid; p < g.Np; p += T) hp[p] = cdiv(cscale(buf[g.pilot_idx[p]], sc), G::pilots(g)[p]);
        __syncthreads();
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {   // the pair's RX in order
        const V* bu = bufs + u * N;
        const V* hp = hpa + (r0 + u) * g.Np;
#pragma unroll
        for (int q = 0; q < QM; ++q) {
          const int j = tid0 + q * WG;
          if (j < g.Nd) {
            const V h = interp_seg<R>(hp, g.Np, sg[q], fk[q], ig[q]);
            if (est) den[q] += abs2_ref(h);
            num[q] = cadd(num[q], cmulc(cscale(bu[kpos[q]], sc), h));
          }
        }
      }
      __syncthreads();   // every read of both buffers done before the next pair / symbol lands in them
    }
#pragma unroll
    for (int q = 0; q < QM; ++q) {
      const int j = tid0 + q * WG;
      if (j >= g.Nd) continue;
      const int re = l * g.Nd + j;
      const R rr = (R)1 / (den[q] + (R)1e-10);
      const V z = mkc(num[q].x * rr, num[q].y * rr);
      if (cap_syms) cap_syms[fre + re] = z;
      const int idx = hard_index(z, BPS, QS);
      const int64_t pb0 = (int64_t)re * BPS;
      errs += __popc(((uint32_t)idx ^ getbits<BPS>(fb, pb0, n_bits)) & bits_valid<BPS>(pb0, n_bits));
      if (cap_bits) {
#pragma unroll
        for (int m = 0; m < BPS; ++m)
          if (pb0 + m < n_bits) cap_bits[(size_t)b * n_bits + pb0 + m] = (uint8_t)((idx >> (BPS - 1 - m)) & 1);
      }
    }
  }
  frame_err_add(frame_err, b, errs);
}

bool rx_frame_simo_supported(const Grid& g, int num_rx) {
  return num_rx >= 2 && num_rx <= RXS_MAXRX && (g.bps == 2 || g.bps == 4 || g.bps == 6) && 2 * g.Nd < g.N;
}

bool rx_simo2_ok(const Grid& g, int num_rx, bool H, bool pstats) {
  return g.N == 1024 && (num_rx & 1) == 0 && num_rx <= RXS_MAXRX && !H && !pstats && g.Nd <= 2 * WG;
}

template <class R>
int launch_rx_frame_simo(hipStream_t s, const Grid& g, int B, int num_rx, const cx<R>* y, int64_t y_rx_stride,
                         int64_t y_frame_stride, const R* npow, const uint64_t* fid, uint64_t seed, const R* inj_z,
                         int64_t inj_stride, const uint32_t* pw, int PW, int n_bits, uint32_t* frame_err,
                         cx<R>* cap_syms, uint8_t* cap_bits, cx<R>* H, R* pstats, const TxChannelT<R>* xc) {
  if (!rx_frame_simo_supported(g, num_rx)) return (int)hipErrorInvalidValue;
  if constexpr (sizeof(R) == 8) {   // config 3: the wave-private receiver (lte_wave.hip)
    if (simo_rx_wave_enabled() &&
        rx_simo_w_supported(g, num_rx, 1, H != nullptr, pstats != nullptr, xc && xc->x_out))
      return launch_rx_frame_simo_w(s, g, B, num_rx, y, y_rx_stride, y_frame_stride, npow, fid, seed, inj_z, inj_stride,
                                    pw, PW, n_bits, frame_err, cap_syms, cap_bits);
  }
  const char* pe = std::getenv("LTE_RXS_PAIRS");   // 0: one slot per frame with T threads, the RX in sequence (A/B)
  if (rx_simo2_ok(g, num_rx, H != nullptr, pstats != nullptr) && (!pe || std::atoi(pe) != 0)) {
    const bool xin = xc && xc->x_out;
    const size_t shm2 = (2 * (size_t)g.N + RXS_MAXRX * g.Np + (xin ? g.N : 0)) * sizeof(cx<R>);
    const TxChannelT<R> xcv = xin ? *xc : TxChannelT<R>{};
#define LTE_RXS2(BPS_)                                                                                               \
  do {                                                                                                               \
    if (xin)                                                                                                         \
      hipLaunchKernelGGL((k_rx_frame_simo2<R, BPS_, 1024, true>), dim3(B), dim3(WG), shm2, s, g, B, num_rx, y,       \
                         y_rx_stride, y_frame_stride, npow, fid, seed, inj_z, inj_stride, pw, PW, n_bits, frame_err, \
                         cap_syms, cap_bits, xcv);                                                                   \
    else                                                                                                             \
      hipLaunchKernelGGL((k_rx_frame_simo2<R, BPS_, 1024>), dim3(B), dim3(WG), shm2, s, g, B, num_rx, y, y_rx_stride, \
                         y_frame_stride, npow, fid, seed, inj_z, inj_stride, pw, PW, n_bits, frame_err, cap_syms,    \
                         cap_bits, xcv);                                                                             \
  } while (0)
    if (g.bps == 2) LTE_RXS2(2); else if (g.bps == 4) LTE_RXS2(4); else LTE_RXS2(6);
#undef LTE_RXS2
    return (int)hipGetLastError();
  }
  if (xc && xc->x_out) return (int)hipErrorInvalidValue;   // the symbol handoff needs the paired receiver
  const int spw = WG / (g.N >> 3);
  const int blocks = (B + spw - 1) / spw;
  const size_t shm = (size_t)spw * (g.N + RXS_MAXRX * g.Np) * sizeof(cx<R>);
#define LTE_RXS(BPS_, NC_)                                                                                           \
  hipLaunchKernelGGL((k_rx_frame_simo<R, BPS_, NC_>), dim3(blocks), dim3(WG), shm, s, g, B, num_rx, y, y_rx_stride,  \
                     y_frame_stride, npow, fid, seed, inj_z, inj_stride, pw, PW, n_bits, frame_err, cap_syms,        \
                     cap_bits, H, pstats)
#define LTE_RXS_BPS(NC_)                                                                                             \
  do {                                                                                                               \
    if (g.bps == 2) LTE_RXS(2, NC_);                                                                                 \
    else if (g.bps == 4) LTE_RXS(4, NC_);                                                                            \
    else LTE_RXS(6, NC_);                                                                                            \
  } while (0)
  if (g.N == 1024) LTE_RXS_BPS(1024);   // config 3 (10 MHz)
  else LTE_RXS_BPS(0);
#undef LTE_RXS_BPS
#undef LTE_RXS
  return (int)hipGetLastError();
}

template <class R, int CHAIN, bool SCF = false, int NC = 0>
static void rx_data_bps(int bps, hipStream_t s, int blocks, size_t shm, const Grid& g, int rayleigh, int B,
                        int num_rx, const cx<R>* y, int64_t y_rx_stride, int64_t y_frame_stride, const cx<R>* H,
                        const R* npow, const R* snr_lin, const uint64_t* fid, uint64_t seed, const R* inj_z,
                        int64_t inj_stride, const uint32_t* pw, int PW, int n_bits, uint32_t* frame_err, R* llr,
                        cx<R>* cap_syms, uint8_t* cap_bits, R* nvo) {
#define LTE_RXD(BPS_)                                                                                             \
  hipLaunchKernelGGL((k_rx_data<R, CHAIN, BPS_, SCF, NC>), dim3(blocks), dim3(WG), shm, s, g, rayleigh, B, num_rx, y, \
                     y_rx_stride, y_frame_stride, H, npow, snr_lin, fid, seed, inj_z, inj_stride, pw, PW, n_bits,   \
                     frame_err, llr, cap_syms, cap_bits, nvo)
  if (bps == 2) LTE_RXD(2);
  else if (bps == 4) LTE_RXD(4);
  else LTE_RXD(6);
#undef LTE_RXD
}

template <class R>
int launch_rx_data(hipStream_t s, const Grid& g, int chain, int rayleigh, int B, int num_rx, const cx<R>* y,
                   int64_t y_rx_stride, int64_t y_frame_stride, const cx<R>* H, const R* npow, const R* snr_lin,
                   const uint64_t* fid, uint64_t seed, const R* inj_z, int64_t inj_stride, const uint32_t* pw, int PW,
                   int n_bits, uint32_t* frame_err, R* llr, cx<R>* cap_syms, uint8_t* cap_bits, int sc_fdm,
                   R* nv_out) {
  if (g.bps != 2 && g.bps != 4 && g.bps != 6) return (int)hipErrorInvalidValue;
  if (nv_out && chain != LTE_CHAIN_CODED) return (int)hipErrorInvalidValue;
  if (sc_fdm && (chain != LTE_CHAIN_UNCODED || !GridT<R>::chirp(g) || !GridT<R>::bhat(g)))
    return (int)hipErrorInvalidValue;
  if (chain == LTE_CHAIN_SIMO && num_rx > 8) return (int)hipErrorInvalidValue;
  const int spw = WG / (g.N >> 3);
  const int64_t total = (int64_t)B * g.n_sym;
  if (total > 0x7FFFFFFF - spw) return (int)hipErrorInvalidValue;
  const int blocks = (int)((total + spw - 1) / spw);
  const size_t shm = spw * g.N * sizeof(cx<R>);
#define LTE_RXA(CH_, SCF_, NC_)                                                                                   \
  rx_data_bps<R, CH_, SCF_, NC_>(g.bps, s, blocks, shm, g, rayleigh, B, num_rx, y, y_rx_stride, y_frame_stride, H, \
                                 npow, snr_lin, fid, seed, inj_z, inj_stride, pw, PW, n_bits, frame_err, llr,      \
                                 cap_syms, cap_bits, nv_out)
  if (chain == LTE_CHAIN_CODED && g.N == 2048) LTE_RXA(LTE_CHAIN_CODED, false, 2048);   // the headline chain
  else if (chain == LTE_CHAIN_CODED) LTE_RXA(LTE_CHAIN_CODED, false, 0);
  else if (chain == LTE_CHAIN_SIMO) LTE_RXA(LTE_CHAIN_SIMO, false, 0);
  else if (sc_fdm) LTE_RXA(LTE_CHAIN_UNCODED, true, 0);
  else LTE_RXA(LTE_CHAIN_UNCODED, false, 0);
#undef LTE_RXA
  return (int)hipGetLastError();
}

// explicit instances of the precision-templated launchers (lte_capi.hip)
#define LTE_INST(R)                                                                                                   \
  template int launch_ofdm_tx<R>(hipStream_t, const Grid&, int, const uint32_t*, int, const uint32_t*, int,          \
                                 const int32_t*, cx<R>*, int, cx<R>*, int);                                         \
  template int launch_ofdm_tx_ch<R>(hipStream_t, const Grid&, int, const uint32_t*, int, const uint32_t*, int,       \
                                    const int32_t*, int, cx<R>*, const TxChannelT<R>&, int);                        \
  template int launch_chan_fix<R>(hipStream_t, const Grid&, int, const TxChannelT<R>&);                             \
  template int launch_ofdm_txf<R>(hipStream_t, const Grid&, const uint32_t*, int, const int32_t*, const int32_t*,   \
                                  const int32_t*, int, cx<R>*, const TxChannelT<R>&);                                \
  template int launch_fading<R>(hipStream_t, int, int, int, const R*, const uint64_t*, uint64_t, const R*, int64_t, \
                                R*, cx<R>*);                                                                         \
  template int launch_jakes_sets<R>(hipStream_t, int, int, int, int, const R*, const R*, double, double, cx<R>*);     \
  template int launch_channel<R>(hipStream_t, const Grid&, int, int, int, int, const int32_t*, const R*, R, R,       \
                                 const R*, const cx<R>*, const cx<R>*, cx<R>*, R*, int, int);                       \
  template int launch_npow<R>(hipStream_t, int, int, const R*, int, int, const R*, R*);                             \
  template int launch_rx_chest<R>(hipStream_t, const Grid&, int, int, const cx<R>*, int64_t, int64_t, const R*,      \
                                  const uint64_t*, uint64_t, const R*, int64_t, cx<R>*, R*);                        \
  template int launch_rx_data<R>(hipStream_t, const Grid&, int, int, int, int, const cx<R>*, int64_t, int64_t,       \
                                 const cx<R>*, const R*, const R*, const uint64_t*, uint64_t, const R*, int64_t,    \
                                 const uint32_t*, int, int, uint32_t*, R*, cx<R>*, uint8_t*, int, R*);              \
  template int launch_rx_frame_simo<R>(hipStream_t, const Grid&, int, int, const cx<R>*, int64_t, int64_t, const R*,  \
                                       const uint64_t*, uint64_t, const R*, int64_t, const uint32_t*, int, int,       \
                                       uint32_t*, cx<R>*, uint8_t*, cx<R>*, R*, const TxChannelT<R>*);               \
  template int launch_rx_frame<R>(hipStream_t, const Grid&, int, int, int, const cx<R>*, int64_t, const R*, const R*, \
                                  const uint64_t*, uint64_t, const R*, int64_t, const uint32_t*, int, int, uint32_t*, \
                                  R*, cx<R>*, uint8_t*, R*, cx<R>*, R*);
LTE_INST(float)
LTE_INST(double)
#undef LTE_INST

// ---------------------------------------------------------------------------
// Per-SNR counters {bit errors, bits, block errors, blocks}.  Each block sums
// its frames (grid-stride) into LDS counters, then adds them to the global
// counters once: 4 * n_snr global atomics per block instead of 4 per frame
// (262 144 u64 atomics onto 64 addresses at 65 536 frames).  n_snr too large
// for LDS (> ACC_LDS_SNR): direct global atomics.
constexpr int ACC_LDS_SNR = 1024;
__global__ __launch_bounds__(WG) void k_accumulate(int B, int coded, int n_bits, int n_snr,
                                                   const int32_t* __restrict__ snr_idx,
                                                   const uint32_t* __restrict__ frame_err,
                                                   const uint32_t* __restrict__ frame_crc,
                                                   unsigned long long* __restrict__ counts) {
  extern __shared__ unsigned long long acc[];   // [n_snr][4] when n_snr <= ACC_LDS_SNR
  const bool lds = n_snr <= ACC_LDS_SNR;
  unsigned long long* dst = lds ? acc : counts;
  if (lds) {
    for (int i = threadIdx.x; i < 4 * n_snr; i += WG) acc[i] = 0ull;
    __syncthreads();
  }
  for (int b = blockIdx.x * WG + threadIdx.x; b < B; b += gridDim.x * WG) {
    const int s = snr_idx[b];
    const uint32_t e = frame_err[b];
    const uint32_t blk = coded ? (frame_crc[b] ? 0u : 1u) : (e ? 1u : 0u);
    atomicAdd(dst + 4 * s + 0, (unsigned long long)e);
    atomicAdd(dst + 4 * s + 1, (unsigned long long)n_bits);
    atomicAdd(dst + 4 * s + 2, (unsigned long long)blk);
    atomicAdd(dst + 4 * s + 3, 1ull);
  }
  if (lds) {
    __syncthreads();
    for (int i = threadIdx.x; i < 4 * n_snr; i += WG)
      if (acc[i]) atomicAdd(counts + i, acc[i]);
  }
}

int launch_accumulate(hipStream_t s, int B, int coded, int n_bits, int n_snr, const int32_t* snr_idx,
                      const uint32_t* frame_err, const uint32_t* frame_crc, unsigned long long* counts) {
  const int blocks = std::min((B + WG - 1) / WG, 512);
  const size_t shm = n_snr <= ACC_LDS_SNR ? (size_t)4 * n_snr * sizeof(unsigned long long) : 0;
  hipLaunchKernelGGL(k_accumulate, dim3(blocks), dim3(WG), shm, s, B, coded, n_bits, n_snr, snr_idx, frame_err,
                     frame_crc, counts);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Stage kernels for the parity entry points (both precisions).
template <class R>
__global__ __launch_bounds__(WG) void k_fft_batch(Grid g, int inverse, int64_t batch, const cx<R>* __restrict__ in,
                                                  cx<R>* __restrict__ out) {
  using V = cx<R>;
  V* sm = dyn_lds<V>();
  const int N = g.N, T = N >> 3, spw = WG / T;
  const int slot = threadIdx.x / T, tid = threadIdx.x % T;
  const int64_t i = (int64_t)blockIdx.x * spw + slot;
  const bool active = slot < spw && i < batch;
  V* buf = sm + slot * N;
  if (active)
    for (int k = tid; k < N; k += T) buf[k] = in[i * N + k];
  __syncthreads();
  if (inverse) fft_lds<true>(buf, N, g.log2N, GridT<R>::tw(g), tid, active);
  else fft_lds<false>(buf, N, g.log2N, GridT<R>::tw(g), tid, active);
  if (active) {
    const R sc = inverse ? tx_scale<R>(N) : rx_scale<R>(N);
    for (int k = tid; k < N; k += T) out[i * N + k] = cscale(buf[k], sc);
  }
}

template <class R>
int launch_fft(hipStream_t s, const Grid& g, int inverse, int64_t batch, const cx<R>* in, cx<R>* out) {
  const int spw = WG / (g.N >> 3);
  const int blocks = (int)((batch + spw - 1) / spw);
  hipLaunchKernelGGL(k_fft_batch<R>, dim3(blocks), dim3(WG), spw * g.N * sizeof(cx<R>), s, g, inverse, batch, in,
                     out);
  return (int)hipGetLastError();
}

template <class R, int BPS>
__global__ void k_llr(int64_t n, const cx<R>* __restrict__ syms, const R* __restrict__ nv, R* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  R o[BPS];
  soft_demap<BPS>(syms[i], nv[i], o);
#pragma unroll
  for (int m = 0; m < BPS; ++m) out[i * BPS + m] = o[m];
}

template <class R>
int launch_llr(hipStream_t s, int bps, int64_t n, const cx<R>* syms, const R* nv, R* llr) {
  const dim3 grid((unsigned)((n + WG - 1) / WG));
  if (bps == 2) hipLaunchKernelGGL((k_llr<R, 2>), grid, dim3(WG), 0, s, n, syms, nv, llr);
  else if (bps == 4) hipLaunchKernelGGL((k_llr<R, 4>), grid, dim3(WG), 0, s, n, syms, nv, llr);
  else if (bps == 6) hipLaunchKernelGGL((k_llr<R, 6>), grid, dim3(WG), 0, s, n, syms, nv, llr);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

template <class R, int BPS>
__global__ void k_hard(int64_t n, const cx<R>* __restrict__ syms, uint8_t* __restrict__ bits) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int idx = hard_index(syms[i], BPS, (R)qam_norm<BPS>());
#pragma unroll
  for (int m = 0; m < BPS; ++m) bits[i * BPS + m] = (idx >> (BPS - 1 - m)) & 1;
}

template <class R>
int launch_hard(hipStream_t s, int bps, int64_t n, const cx<R>* syms, uint8_t* bits) {
  const dim3 grid((unsigned)((n + WG - 1) / WG));
  if (bps == 2) hipLaunchKernelGGL((k_hard<R, 2>), grid, dim3(WG), 0, s, n, syms, bits);
  else if (bps == 4) hipLaunchKernelGGL((k_hard<R, 4>), grid, dim3(WG), 0, s, n, syms, bits);
  else if (bps == 6) hipLaunchKernelGGL((k_hard<R, 6>), grid, dim3(WG), 0, s, n, syms, bits);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Stage entry: batched SC-FDM DFT / IDFT of size M = g.Nd (DFTPrecodifier.
// precoding / IDFTDecodifier.decoding, core/dft_precoding.py:66-118, 199-226)
// on host-supplied vectors; one slot per vector, the same dft_bluestein the
// chains run in-line.
template <class R>
__global__ __launch_bounds__(WG) void k_dft_stage(Grid g, int inverse, int64_t batch, const cx<R>* __restrict__ in,
                                                  cx<R>* __restrict__ out) {
  using V = cx<R>;
  V* sm = dyn_lds<V>();
  const int N = g.N, T = N >> 3, spw = WG / T;
  const int slot = threadIdx.x / T, tid = threadIdx.x % T;
  const int64_t v = (int64_t)blockIdx.x * spw + slot;
  const bool active = slot < spw && v < batch;
  V* buf = sm + slot * N;
  if (active) {
    for (int k = tid; k < N; k += T) {
      V x = k < g.Nd ? in[v * g.Nd + k] : mkc((R)0, (R)0);
      if (inverse) x.y = -x.y;
      buf[k] = x;
    }
  }
  dft_bluestein(buf, g, tid, T, active);
  if (active)
    for (int k = tid; k < g.Nd; k += T) {
      V x = buf[k];
      if (inverse) x.y = -x.y;
      out[v * g.Nd + k] = x;
    }
}

template <class R>
int launch_dft(hipStream_t s, const Grid& g, int inverse, int64_t batch, const cx<R>* in, cx<R>* out) {
  const int spw = WG / (g.N >> 3);
  const int64_t blocks = (batch + spw - 1) / spw;
  if (blocks > 0x7FFFFFFF || !GridT<R>::chirp(g) || !GridT<R>::bhat(g) || 2 * g.Nd - 1 > g.N)
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_dft_stage<R>, dim3((unsigned)blocks), dim3(WG), spw * g.N * sizeof(cx<R>), s, g, inverse,
                     batch, in, out);
  return (int)hipGetLastError();
}

#define LTE_INST_STAGE(R)                                                                                      \
  template int launch_fft<R>(hipStream_t, const Grid&, int, int64_t, const cx<R>*, cx<R>*);                   \
  template int launch_dft<R>(hipStream_t, const Grid&, int, int64_t, const cx<R>*, cx<R>*);                   \
  template int launch_llr<R>(hipStream_t, int, int64_t, const cx<R>*, const R*, R*);                          \
  template int launch_hard<R>(hipStream_t, int, int64_t, const cx<R>*, uint8_t*);
LTE_INST_STAGE(float)
LTE_INST_STAGE(double)
#undef LTE_INST_STAGE

}  // namespace lte
