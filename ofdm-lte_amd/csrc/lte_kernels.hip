// Front-end kernels of the LTE link chain for gfx950: payload/CRC, OFDM TX
// (QAM map + resource map + IFFT + CP), multipath Rayleigh + AWGN channel,
// RX (CP removal + FFT, CRS LS estimation + interpolation, ZF / MRC, hard
// decision or soft demap).  All HBM-bound: every kernel streams its frame
// data once, coalesced, with per-symbol FFTs staged in LDS.
#include "lte_common.h"
#include "lte_internal.h"
#include "lte_dev.h"

namespace lte {

constexpr int WG = 256;

// ---------------------------------------------------------------------------
// Payload bits (+ CRC-24A, crc.py:212-233) : one lane per frame.
__device__ __forceinline__ uint32_t crc24_entry(uint32_t i, uint32_t poly) {
  uint32_t r = i << 16;
  for (int k = 0; k < 8; ++k) r = (r & 0x800000u) ? ((r << 1) ^ poly) : (r << 1);
  return r & 0xFFFFFFu;
}

__global__ __launch_bounds__(WG) void k_payload(uint32_t* __restrict__ pw, int PW, int n_bits, int crc,
                                                const uint64_t* __restrict__ fid, uint64_t seed, int B,
                                                const uint32_t* __restrict__ inj, int64_t inj_stride) {
  __shared__ uint32_t T[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) T[i] = crc24_entry(i, 0x864CFBu);
  __syncthreads();
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  uint32_t* w = pw + (size_t)b * PW;
  const int nwd = (n_bits + 31) >> 5;
  u32x4 rv{0, 0, 0, 0};
  uint32_t c = 0;
  for (int i = 0; i < PW; ++i) {
    uint32_t v = 0;
    if (i < nwd) {
      if (inj) {
        v = inj[(size_t)b * inj_stride + i];
      } else {
        if ((i & 3) == 0) rv = rng4(seed, fid[b], RNG_STREAM_BITS, (uint32_t)(i >> 2));
        const int q = i & 3;
        v = q == 0 ? rv.x : q == 1 ? rv.y : q == 2 ? rv.z : rv.w;
      }
      const int rem = n_bits - 32 * i;
      if (rem < 32) v &= ~(0xFFFFFFFFu >> rem);
      if (crc) {
        const int dbits = min(32, rem);
        int k = 0;
        for (; k + 8 <= dbits; k += 8) c = ((c << 8) & 0xFFFFFFu) ^ T[((c >> 16) ^ (v >> (24 - k))) & 0xFFu];
        for (; k < dbits; ++k) {
          const uint32_t msb = (c >> 23) & 1u;
          c = (c << 1) & 0xFFFFFFu;
          if (msb ^ ((v >> (31 - k)) & 1u)) c ^= 0x864CFBu;
        }
      }
    }
    w[i] = v;
  }
  if (crc) {  // append the 24 CRC bits MSB-first at [n_bits, n_bits+24)
    for (int t = 0; t < 24; ++t) {
      const int p = n_bits + t;
      if ((c >> (23 - t)) & 1u) w[p >> 5] |= 1u << (31 - (p & 31));
    }
  }
}

int launch_payload(hipStream_t s, uint32_t* pw, int PW, int n_bits, int crc, const uint64_t* fid, uint64_t seed,
                   int B, const uint32_t* inj, int64_t inj_stride) {
  hipLaunchKernelGGL(k_payload, dim3((B + WG - 1) / WG), dim3(WG), 0, s, pw, PW, n_bits, crc, fid, seed, B, inj,
                     inj_stride);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Fused static-tap channel for one OFDM symbol held in LDS (TxChannel): y[m] =
// sum_p c_p x[m - d_p] over the CP-extended symbol, whose sample j is
// buf[j < cp ? N - cp + j : j - cp] (rayleighchannel.py:44-58; for m >=
// max_delay every delayed tap stays inside the symbol); stores m >= cp only
// and sums |y|^2 over m >= max_delay per slot in a fixed order.  Called by
// every thread of the block.
__device__ __forceinline__ void tx_channel(float2* buf, const Grid& g, const TxChannel& ch, int b, int l, int slot,
                                           int tid, int T, bool active, float sc) {
  __shared__ float red[WG / 64];
  const int N = g.N, cp = g.cp, S = N + cp, D = ch.max_delay;
  float pw = 0.f;
  if (active) {
    if (D > 0) {   // the TX samples x = buf / sqrt(N) at both ends of the symbol
      float2* xh = ch.xh + ((size_t)b * g.n_sym + l) * 2 * D;
      for (int i = tid; i < 2 * D; i += T) {
        const int j = i < D ? i : S - 2 * D + i;
        xh[i] = cscale(buf[(j - cp) & (N - 1)], sc);
      }
    }
    // 1/sqrt(N) folded into the taps; sample j of the CP-extended symbol is
    // buf[(j - cp) mod N] (N a power of 2)
    float2 cf[TXCH_MAXP];
    int off[TXCH_MAXP];
#pragma unroll
    for (int p = 0; p < TXCH_MAXP; ++p) {
      cf[p] = p < ch.n_paths ? cscale(ch.coef[(size_t)b * ch.n_paths + p], sc) : make_float2(0.f, 0.f);
      off[p] = ch.delays[p] + cp;
    }
    float2* yo = ch.y + (size_t)b * g.L + (size_t)l * S;
    for (int m = D + tid; m < S; m += T) {
      float2 v = make_float2(0.f, 0.f);
#pragma unroll
      for (int p = 0; p < TXCH_MAXP; ++p)
        if (p < ch.n_paths) v = cadd(v, cmul(cf[p], buf[(m - off[p]) & (N - 1)]));
      if (m >= cp) yo[m] = v;
      pw += v.x * v.x + v.y * v.y;
    }
  }
  // per-slot sum in a fixed order: T >= 64 threads = T / 64 whole waves per slot
  for (int o = 32; o > 0; o >>= 1) pw += __shfl_xor(pw, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = pw;
  __syncthreads();
  if (active && tid == 0) {
    const int wps = T >> 6;
    float t = 0.f;
    for (int w = 0; w < wps; ++w) t += red[slot * wps + w];
    ch.pow_part[(size_t)b * g.n_sym + l] = t;
  }
}

// OFDM TX: one slot = one OFDM symbol; 2048/N slots per 256-thread block.
// QAMModulator.bits_to_symbols (modulator.py:61-88) / coded RE mapping via
// tx_map (rate_match_turbo + T/F interleaver, rate_matching.py:193-297,
// ofdm_core.py:1040-1099), ResourceMapper.map_symbols (resource_mapper.py:
// 181-223), ifft*sqrt(N) + CP (modulator.py:242-248).
// SCF (SC-FDM, uncoded chains): the Nd QAM symbols of the OFDM symbol are
// DFT-precoded (M = Nd, core/modulator.py:232-236) in a second LDS buffer first.
// CH: the channel applied in place (tx_channel); NC: compile-time N (fft_lds).
template <int CODED, int BPS, bool SCF = false, bool CH = false, int NC = 0>
__global__ __launch_bounds__(WG) void k_ofdm_tx(Grid g, const uint32_t* __restrict__ pw, int PW,
                                                const uint32_t* __restrict__ enc, int enc_words,
                                                const int32_t* __restrict__ tx_map, float2* __restrict__ x, int B,
                                                float2* __restrict__ cap_syms, int stage_enc, TxChannel ch) {
  extern __shared__ float2 sm[];
  const int N = NC ? NC : g.N, T = N >> 3, spw = WG / T;
  const int slot = threadIdx.x / T, tid = threadIdx.x % T;
  const int gs = blockIdx.x * spw + slot;
  const int b = gs / g.n_sym, l = gs - b * g.n_sym;
  const bool active = slot < spw && b < B;
  float2* buf = sm + slot * N;
  float2* pre = SCF ? sm + (spw + slot) * N : buf;   // SC-FDM: QAM symbols -> DFT buffer
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
    for (int k = tid; k < N; k += T) buf[k] = make_float2(0.f, 0.f);
    if constexpr (SCF)
      for (int k = g.Nd + tid; k < N; k += T) pre[k] = make_float2(0.f, 0.f);
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
      const float2 sym = zero ? make_float2(0.f, 0.f) : qam_point<BPS>(idx);
      buf[kpos[q]] = sym;
      if (cap_syms) cap_syms[(size_t)b * g.n_sym * g.Nd + (size_t)l * g.Nd + j] = sym;
    }
  }
  if (active) {
    const uint32_t* fb = pw + (size_t)b * PW;
    for (int j = tid; j < (CODED ? 0 : g.Nd); j += T) {   // uncoded: payload bits in order
      const int64_t t0 = ((int64_t)l * g.Nd + j) * BPS;
      int idx = 0;
#pragma unroll
      for (int m = 0; m < BPS; ++m) idx = (idx << 1) | (int)getbit(fb, t0 + m);
      const float2 sym = qam_point<BPS>(idx);
      if constexpr (SCF) pre[j] = sym;
      else buf[g.data_idx[j]] = sym;
      if (cap_syms) cap_syms[(size_t)b * g.n_sym * g.Nd + (size_t)l * g.Nd + j] = sym;
    }
    for (int p = tid; p < g.Np; p += T) buf[g.pilot_idx[p]] = g.pilots[p];
  }
  if constexpr (SCF) {
    dft_bluestein(pre, g, tid, T, active);
    if (active)
      for (int j = tid; j < g.Nd; j += T) buf[g.data_idx[j]] = pre[j];
  }
  __syncthreads();
  fft_lds<true, NC>(buf, N, g.log2N, g.tw, tid, active);
  if constexpr (CH) {
    tx_channel(buf, g, ch, b, l, slot, tid, T, active, rsqrtf((float)N));
  } else if (active) {
    const float sc = rsqrtf((float)N);
    float2* xo = x + (size_t)b * g.L + (size_t)l * (N + g.cp);
    for (int k = tid; k < N; k += T) xo[g.cp + k] = cscale(buf[k], sc);
    for (int k = tid; k < g.cp; k += T) xo[k] = cscale(buf[N - g.cp + k], sc);
  }
}

int launch_ofdm_tx(hipStream_t s, const Grid& g, int coded, const uint32_t* pw, int PW, const uint32_t* enc,
                   int enc_words, const int32_t* tx_map, float2* x, int B, float2* cap_syms, int sc_fdm) {
  const int spw = WG / (g.N >> 3);
  const int64_t total = (int64_t)B * g.n_sym;
  if (total > 0x7FFFFFFF - spw || (g.bps != 2 && g.bps != 4 && g.bps != 6)) return (int)hipErrorInvalidValue;
  if (sc_fdm && (coded || !g.chirp || !g.bhat || 2 * g.Nd > g.N)) return (int)hipErrorInvalidValue;
  const int blocks = (int)((total + spw - 1) / spw);
  const size_t enc_shm = (size_t)spw * enc_words * sizeof(uint32_t);
  const int stage_enc = coded && enc_shm <= 32768;
  const size_t shm = (sc_fdm ? 2 : 1) * spw * g.N * sizeof(float2) + (stage_enc ? enc_shm : 0);
#define LTE_TX(C_, B_, S_)                                                                                         \
  hipLaunchKernelGGL((k_ofdm_tx<C_, B_, S_>), dim3(blocks), dim3(WG), shm, s, g, pw, PW, enc, enc_words, tx_map, x, \
                     B, cap_syms, stage_enc, TxChannel{})
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

int launch_ofdm_tx_ch(hipStream_t s, const Grid& g, int coded, const uint32_t* pw, int PW, const uint32_t* enc,
                      int enc_words, const int32_t* tx_map, int B, float2* cap_syms, const TxChannel& ch) {
  const int spw = WG / (g.N >> 3);
  const int64_t total = (int64_t)B * g.n_sym;
  if (!txch_supported(g, ch.n_paths, ch.max_delay) || total > 0x7FFFFFFF - spw ||
      (g.bps != 2 && g.bps != 4 && g.bps != 6))
    return (int)hipErrorInvalidValue;
  const int blocks = (int)((total + spw - 1) / spw);
  const size_t enc_shm = (size_t)spw * enc_words * sizeof(uint32_t);
  const int stage_enc = coded && enc_shm <= 32768;
  const size_t shm = (size_t)spw * g.N * sizeof(float2) + (stage_enc ? enc_shm : 0);
#define LTE_TXC(C_, B_)                                                                                      \
  if (g.N == 2048)                                                                                             \
    hipLaunchKernelGGL((k_ofdm_tx<C_, B_, false, true, 2048>), dim3(blocks), dim3(WG), shm, s, g, pw, PW, enc, \
                       enc_words, tx_map, (float2*)nullptr, B, cap_syms, stage_enc, ch);                         \
  else                                                                                                         \
    hipLaunchKernelGGL((k_ofdm_tx<C_, B_, false, true>), dim3(blocks), dim3(WG), shm, s, g, pw, PW, enc,        \
                       enc_words, tx_map, (float2*)nullptr, B, cap_syms, stage_enc, ch)
  if (coded) {
    if (g.bps == 2) LTE_TXC(1, 2); else if (g.bps == 4) LTE_TXC(1, 4); else LTE_TXC(1, 6);
  } else {
    if (g.bps == 2) LTE_TXC(0, 2); else if (g.bps == 4) LTE_TXC(0, 4); else LTE_TXC(0, 6);
  }
#undef LTE_TXC
  return (int)hipGetLastError();
}

// Power of each symbol's first max_delay channel-output samples (their delayed
// taps reach into the previous symbol's tail, or the zero prefix of symbol 0),
// added to the symbol's partial.  16 lanes per (frame, symbol), one sample
// each (coalesced head / tail reads), summed by a fixed xor butterfly.
constexpr int CHF_LANES = 16;
__global__ __launch_bounds__(WG) void k_chan_fix(Grid g, int B, TxChannel ch) {
  const int64_t i = ((int64_t)blockIdx.x * WG + threadIdx.x) / CHF_LANES;
  const int lane = threadIdx.x % CHF_LANES;
  const bool ok = i < (int64_t)B * g.n_sym;
  float pw = 0.f;
  if (ok) {
    const int l = (int)(i % g.n_sym), b = (int)(i / g.n_sym);
    const int D = ch.max_delay;
    const float2* hd = ch.xh + (size_t)i * 2 * D;   // this symbol's head; hd[-D..-1] = previous symbol's tail
    const float2* cb = ch.coef + (size_t)b * ch.n_paths;
    for (int m = lane; m < D; m += CHF_LANES) {
      float2 v = make_float2(0.f, 0.f);
      for (int p = 0; p < ch.n_paths; ++p) {
        const int j = m - ch.delays[p];
        const float2 xv = (j >= 0 || l > 0) ? hd[j] : make_float2(0.f, 0.f);
        v = cadd(v, cmul(cb[p], xv));
      }
      pw += v.x * v.x + v.y * v.y;
    }
  }
#pragma unroll
  for (int o = CHF_LANES / 2; o > 0; o >>= 1) pw += __shfl_xor(pw, o);
  if (ok && lane == 0) ch.pow_part[i] += pw;
}

int launch_chan_fix(hipStream_t s, const Grid& g, int B, const TxChannel& ch) {
  const int64_t n = (int64_t)B * g.n_sym * CHF_LANES;
  if (ch.max_delay == 0 || n == 0) return 0;
  hipLaunchKernelGGL(k_chan_fix, dim3((unsigned)((n + WG - 1) / WG)), dim3(WG), 0, s, g, B, ch);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Fading taps: RayleighChannel.jakes_fading phases (rayleighchannel.py:20-42).
// One thread per (frame, rx, path): 16 phases phi_m (Philox or injected) and
// the static coefficient g_p * sqrt(2/16) * sum_m exp(j phi_m) used when fD=0.
__global__ __launch_bounds__(WG) void k_fading(int B, int num_rx, int n_paths, const float* __restrict__ gains,
                                               const uint64_t* __restrict__ fid, uint64_t seed,
                                               const float* __restrict__ inj, int64_t inj_stride,
                                               float* __restrict__ phases, float2* __restrict__ coef) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int per = num_rx * n_paths;
  if (i >= B * per) return;
  const int b = i / per, rp = i % per, rx = rp / n_paths, p = rp % n_paths;
  float* ph = phases + (size_t)i * 16;
  float sr = 0.f, si = 0.f;
  for (int m = 0; m < 16; ++m) {
    float v;
    if (inj) {
      v = inj[(size_t)b * inj_stride + (size_t)rp * 16 + m];
    } else {
      const u32x4 r = rng4(seed, fid[b], RNG_STREAM_FADE + (uint32_t)rx * 64u + (uint32_t)p, (uint32_t)(m >> 2));
      const int q = m & 3;
      const uint32_t u = q == 0 ? r.x : q == 1 ? r.y : q == 2 ? r.z : r.w;
      v = 6.2831853071795864f * ((u >> 8) * (1.0f / 16777216.0f));
    }
    ph[m] = v;
    float s, c;
    sincosf(v, &s, &c);
    sr += c;
    si += s;
  }
  const float k = sqrtf(2.0f / 16.0f) * gains[p];
  coef[i] = make_float2(sr * k, si * k);
}

int launch_fading(hipStream_t s, int B, int num_rx, int n_paths, const float* gains_dev, const uint64_t* fid,
                  uint64_t seed, const float* inj_ph, int64_t inj_stride, float* phases, float2* coef) {
  const int n = B * num_rx * n_paths;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_fading, dim3((n + WG - 1) / WG), dim3(WG), 0, s, B, num_rx, n_paths, gains_dev, fid, seed,
                     inj_ph, inj_stride, phases, coef);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Channel: y[n] = sum_p g_p h_p[n] x[n - d_p] (RayleighChannel.filter,
// rayleighchannel.py:44-58: stream-level delay with zero prefix, Q4) and the
// per-block partial sums of |y|^2 for the measured-power SNR (channel.py:
// 217-224, Q5).  AWGN: only the power of x.  grid (nblk, num_rx, B); a block
// streams CH_CHUNK samples, CH_PER per thread with a 256-sample stride (every
// load / store instruction is one coalesced 2-KB row), then one block
// reduction of the power.
constexpr int CH_PER = 8, CH_CHUNK = WG * CH_PER;

__device__ __forceinline__ float2 jakes_coef(const float* __restrict__ ph, float gain, float fD, float t) {
  float sr = 0.f, si = 0.f;
  for (int m = 0; m < 16; ++m) {   // jakes_fading with t = n / fs
    const float al = 6.2831853071795864f * (float)(m + 1) / 16.0f;
    const float arg = 6.2831853071795864f * fD * cosf(al) * t + ph[m];
    float sv, cv;
    sincosf(arg, &sv, &cv);
    sr += cv;
    si += sv;
  }
  const float k = sqrtf(2.0f / 16.0f) * gain;
  return make_float2(sr * k, si * k);
}

// Rayleigh with every delay <= CH_HALO: the chunk plus its delay halo is staged
// in LDS once with 16-B loads (2 samples per lane), so the n_paths delayed taps
// read LDS instead of re-fetching x through L1/L2 (the kernel was latency
// bound at ~2.2 TB/s); otherwise the taps load from global memory.
constexpr int CH_HALO = 256;
constexpr int CH_MAXP = 8;   // taps held in registers (ITU profiles have <= 6)

__global__ __launch_bounds__(WG) void k_channel(int L, int num_rx, int rayleigh, int n_paths,
                                                const int32_t* __restrict__ delays, const float* __restrict__ gains,
                                                float fD, float fs, const float* __restrict__ phases,
                                                const float2* __restrict__ coef, const float2* __restrict__ x,
                                                float2* __restrict__ y, float* __restrict__ pow_part, int nblk,
                                                int staged) {
  __shared__ float red[WG / 64];
  __shared__ float2 xs[CH_CHUNK + CH_HALO];
  const int blk = blockIdx.x % nblk, b = blockIdx.x / nblk;
  const int rx = blockIdx.y;
  const float2* xf = x + (size_t)b * L;
  float2* yf = y + ((size_t)b * num_rx + rx) * L;
  const size_t cb = ((size_t)b * num_rx + rx) * n_paths;
  const int n0 = blk * CH_CHUNK;
  float pw = 0.f;
  if (rayleigh && staged) {
    const float4* x4 = reinterpret_cast<const float4*>(xf);
    for (int e = threadIdx.x; e < (CH_CHUNK + CH_HALO) / 2; e += WG) {
      const int n = n0 - CH_HALO + 2 * e;   // even: 16-B aligned pair (L is even)
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (n >= 0 && n + 1 < L) v = x4[n >> 1];
      else if (n >= 0 && n < L) v.x = xf[n].x, v.y = xf[n].y;
      xs[2 * e] = make_float2(v.x, v.y);
      xs[2 * e + 1] = make_float2(v.z, v.w);
    }
    __syncthreads();
  }
  if (rayleigh && staged && fD == 0.0f && n_paths <= CH_MAXP) {
    // static taps (fD = 0, the OFDMSimulator default): coefficients and delays
    // in registers, the halo (zero before the frame start) makes every tap an
    // unconditional LDS read
    float2 cf[CH_MAXP];
    int dl[CH_MAXP];
#pragma unroll
    for (int p = 0; p < CH_MAXP; ++p) {
      cf[p] = p < n_paths ? coef[cb + p] : make_float2(0.f, 0.f);
      dl[p] = p < n_paths ? delays[p] : 0;
    }
#pragma unroll
    for (int i = 0; i < CH_PER; ++i) {
      const int n = n0 + i * WG + threadIdx.x;
      if (n >= L) break;
      float2 v = make_float2(0.f, 0.f);
#pragma unroll
      for (int p = 0; p < CH_MAXP; ++p)
        if (p < n_paths) v = cadd(v, cmul(cf[p], xs[n - dl[p] - n0 + CH_HALO]));
      yf[n] = v;
      pw += v.x * v.x + v.y * v.y;
    }
    const float t = block_sum(pw, red);
    if (threadIdx.x == 0) pow_part[((size_t)b * num_rx + rx) * nblk + blk] = t;
    return;
  }
#pragma unroll
  for (int i = 0; i < CH_PER; ++i) {
    const int n = n0 + i * WG + threadIdx.x;
    if (n >= L) break;
    float2 v = make_float2(0.f, 0.f);
    if (!rayleigh) {
      v = xf[n];
    } else {
      for (int p = 0; p < n_paths; ++p) {
        const int src = n - delays[p];
        if (src < 0) continue;
        const float2 c = fD == 0.0f ? coef[cb + p] : jakes_coef(phases + (cb + p) * 16, gains[p], fD, (float)n / fs);
        v = cadd(v, cmul(c, staged ? xs[src - n0 + CH_HALO] : xf[src]));
      }
      yf[n] = v;
    }
    pw += v.x * v.x + v.y * v.y;
  }
  const float t = block_sum(pw, red);
  if (threadIdx.x == 0) pow_part[((size_t)b * num_rx + rx) * nblk + blk] = t;
}

int channel_nblk(int L) { return (L + CH_CHUNK - 1) / CH_CHUNK; }

int launch_channel(hipStream_t s, const Grid& g, int B, int num_rx, int rayleigh, int n_paths,
                   const int32_t* delays_dev, const float* gains_dev, float fD, float fs, const float* phases,
                   const float2* coef, const float2* x, float2* y, float* pow_part, int nblk, int max_delay) {
  if (nblk != channel_nblk(g.L)) return (int)hipErrorInvalidValue;
  // staging uses 16-B pairs: every frame's stream must start 16-B aligned (L even)
  const int staged = rayleigh && max_delay >= 0 && max_delay <= CH_HALO && (g.L & 1) == 0;
  hipLaunchKernelGGL(k_channel, dim3(nblk * B, num_rx), dim3(WG), 0, s, g.L, num_rx, rayleigh, n_paths, delays_dev,
                     gains_dev, fD, fs, phases, coef, x, y, pow_part, nblk, staged);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// RX helpers
__device__ __forceinline__ float frame_power(const float* pp, int nblk, int L) {
  float t = 0.f;
  for (int i = 0; i < nblk; ++i) t += pp[i];
  return t / (float)L;
}

// Load one OFDM symbol (CP removed) of (frame, rx) into LDS adding AWGN:
// noise = sigma * z, sigma = sqrt(P/SNR/2) (channel.py:52-60).
// ---------------------------------------------------------------------------
// Channel estimation: one slot per (frame, rx, 14-symbol group) on the group's
// first symbol (LTEReceiver._estimate_channel_periodic lte_receiver.py:360-411,
// LTEChannelEstimator.estimate_channel :40-96, _interpolate_channel :98-133).
template <int NC = 0>
__global__ __launch_bounds__(WG) void k_rx_chest(Grid g, int B, int num_rx, const float2* __restrict__ y,
                                                 int64_t y_rx_stride, int64_t y_frame_stride,
                                                 const float* __restrict__ npow_in, const uint64_t* __restrict__ fid,
                                                 uint64_t seed, const float* __restrict__ inj_z, int64_t inj_stride,
                                                 float2* __restrict__ H, float* __restrict__ pstats) {
  extern __shared__ float2 sm[];
  const int N = NC ? NC : g.N, T = N >> 3, spw = WG / T;
  const int slot = threadIdx.x / T, tid = threadIdx.x % T;
  const int64_t gs = (int64_t)blockIdx.x * spw + slot;
  const int per = num_rx * g.n_grp;
  const int b = (int)(gs / per), rr = (int)(gs % per), rx = rr / g.n_grp, grp = rr % g.n_grp;
  const bool active = slot < spw && b < B;
  float2* buf = sm + slot * N;
  float2* hp = sm + spw * N + slot * g.Np;
  if (active) {
    const float sigma = sqrtf(npow_in[(size_t)b * num_rx + rx] * 0.5f);
    const float* zf = inj_z ? inj_z + (size_t)b * inj_stride + (size_t)rx * 2 * g.L : nullptr;
    load_symbol_noisy(buf, y + b * y_frame_stride + rx * y_rx_stride, N, g.cp, grp * 14, sigma, seed, fid[b], rx,
                      zf, g.L, tid, T);
  }
  __syncthreads();
  fft_lds<false, NC>(buf, N, g.log2N, g.tw, tid, active);
  if (active) {
    const float sc = rsqrtf((float)N);
    for (int p = tid; p < g.Np; p += T) {
      const float2 Y = cscale(buf[g.pilot_idx[p]], sc);
      hp[p] = cdiv(Y, g.pilots[p]);
      buf[g.pilot_idx[p]] = Y;  // keep scaled pilots for the SNR stats
    }
  }
  __syncthreads();
  if (active) {
    float2* Hf = H + (((size_t)b * num_rx + rx) * g.n_grp + grp) * N;
    for (int k = tid; k < N; k += T) {
      const int sidx = g.seg[k];
      float2 h;
      if (sidx < 0) h = hp[0];
      else if (sidx >= g.Np - 1) h = hp[g.Np - 1];
      else {
        const float2 v0 = hp[sidx], v1 = hp[sidx + 1];
        const float fk = (float)(k - g.pilot_idx[sidx]);
        const float ig = g.inv_gap[sidx];
        h = make_float2(fk * ((v1.x - v0.x) * ig) + v0.x, fk * ((v1.y - v0.y) * ig) + v0.y);
      }
      Hf[k] = h;
    }
    if (tid == 0) {
      float pp = 0.f, en = 0.f;
      for (int p = 0; p < g.Np; ++p) {
        const float2 Y = buf[g.pilot_idx[p]], X = g.pilots[p];
        pp += Y.x * Y.x + Y.y * Y.y;
        const float2 d = csub(Y, X);
        en += d.x * d.x + d.y * d.y;
      }
      float* st = pstats + (((size_t)b * num_rx + rx) * g.n_grp + grp) * 2;
      st[0] = pp / g.Np;
      st[1] = en / g.Np;
    }
  }
}

// per (frame, rx): P = mean |y|^2 over the stream, noise power = P / SNR (channel.py:44-53, 217-224)
__global__ void k_npow(int B, int num_rx, const float* __restrict__ pow_part, int nblk, int L,
                       const float* __restrict__ snr_lin, float* __restrict__ npow) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * num_rx) return;
  npow[i] = frame_power(pow_part + (size_t)i * nblk, nblk, L) / snr_lin[i / num_rx];
}

int launch_npow(hipStream_t s, int B, int num_rx, const float* pow_part, int nblk, int L, const float* snr_lin,
                float* npow) {
  hipLaunchKernelGGL(k_npow, dim3((B * num_rx + WG - 1) / WG), dim3(WG), 0, s, B, num_rx, pow_part, nblk, L, snr_lin,
                     npow);
  return (int)hipGetLastError();
}

int launch_rx_chest(hipStream_t s, const Grid& g, int B, int num_rx, const float2* y, int64_t y_rx_stride,
                    int64_t y_frame_stride, const float* npow, const uint64_t* fid, uint64_t seed,
                    const float* inj_z, int64_t inj_stride, float2* H, float* pstats) {
  const int spw = WG / (g.N >> 3);
  const int64_t total = (int64_t)B * num_rx * g.n_grp;
  const int blocks = (int)((total + spw - 1) / spw);
  const size_t shm = (size_t)spw * (g.N + g.Np) * sizeof(float2);
  if (g.N == 2048)
    hipLaunchKernelGGL(k_rx_chest<2048>, dim3(blocks), dim3(WG), shm, s, g, B, num_rx, y, y_rx_stride, y_frame_stride,
                       npow, fid, seed, inj_z, inj_stride, H, pstats);
  else
    hipLaunchKernelGGL(k_rx_chest<0>, dim3(blocks), dim3(WG), shm, s, g, B, num_rx, y, y_rx_stride, y_frame_stride,
                       npow, fid, seed, inj_z, inj_stride, H, pstats);
  return (int)hipGetLastError();
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
template <int CHAIN, int BPS, bool SCF = false, int NC = 0>
__global__ __launch_bounds__(WG) void k_rx_data(Grid g, int rayleigh, int B, int num_rx,
                                                const float2* __restrict__ y, int64_t y_rx_stride,
                                                int64_t y_frame_stride, const float2* __restrict__ H,
                                                const float* __restrict__ npow, const float* __restrict__ snr_lin,
                                                const uint64_t* __restrict__ fid, uint64_t seed,
                                                const float* __restrict__ inj_z, int64_t inj_stride,
                                                const uint32_t* __restrict__ pw, int PW, int n_bits,
                                                uint32_t* __restrict__ frame_err, float* __restrict__ llr,
                                                float2* __restrict__ cap_syms, uint8_t* __restrict__ cap_bits,
                                                float* __restrict__ nvo) {
  extern __shared__ float2 sm[];
  const int N = NC ? NC : g.N, T = N >> 3, spw = WG / T;
  const int slot = threadIdx.x / T, tid = threadIdx.x % T;
  const int gs = blockIdx.x * spw + slot;
  const int b = gs / g.n_sym, l = gs - b * g.n_sym;
  const bool active = slot < spw && b < B;
  float2* buf = sm + slot * N;
  const int grp = l / 14;
  const float sc = rsqrtf((float)N);
  constexpr float QS = (float)qam_norm<BPS>();
  constexpr int QM = 4;  // data REs per thread (Nd < N/2 for every LTE profile)
  constexpr int NRX = CHAIN == LTE_CHAIN_SIMO ? 8 : 1;
  float2 num[QM];
  float den[QM];
#pragma unroll
  for (int q = 0; q < QM; ++q) { num[q] = make_float2(0.f, 0.f); den[q] = 0.f; }
  for (int rx = 0; rx < (NRX == 1 ? 1 : num_rx); ++rx) {
    if (active) {
      const float sigma = sqrtf(npow[(size_t)b * num_rx + rx] * 0.5f);
      const float* zf = inj_z ? inj_z + (size_t)b * inj_stride + (size_t)rx * 2 * g.L : nullptr;
      load_symbol_noisy2(buf, y + b * y_frame_stride + rx * y_rx_stride, N, g.cp, l, sigma, seed, fid[b], rx, zf,
                         g.L, tid, T);
    }
    __syncthreads();
    fft_lds<false, NC>(buf, N, g.log2N, g.tw, tid, active);
    if (active) {
      const float2* Hf = H + (((size_t)b * num_rx + rx) * g.n_grp + grp) * N;
#pragma unroll
      for (int q = 0; q < QM; ++q) {
        const int j = tid + q * T;
        if (j < g.Nd) {
          const int k = g.data_idx[j];
          const float2 Y = cscale(buf[k], sc), h = Hf[k];
          if constexpr (CHAIN == LTE_CHAIN_SIMO) {
            num[q] = cadd(num[q], cmulc(Y, h));
            den[q] += h.x * h.x + h.y * h.y;
          } else {
            num[q] = (CHAIN == LTE_CHAIN_UNCODED && g.no_eq) ? Y : zf_div(Y, make_float2(h.x + 1e-6f, h.y));
            den[q] = h.x * h.x + h.y * h.y;
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
        if (j < g.Nd) buf[j] = make_float2(num[q].x, -num[q].y);
      }
      for (int k = g.Nd + tid; k < N; k += T) buf[k] = make_float2(0.f, 0.f);
    }
    dft_bluestein(buf, g, tid, T, active);
    if (active) {
#pragma unroll
      for (int q = 0; q < QM; ++q) {
        const int j = tid + q * T;
        if (j < g.Nd) num[q] = make_float2(buf[j].x, -buf[j].y);
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
    float2 z = num[q];
    if constexpr (CHAIN == LTE_CHAIN_SIMO) {
      const float r = 1.0f / (den[q] + 1e-10f);
      z = make_float2(z.x * r, z.y * r);
    }
    if (cap_syms) cap_syms[fre + re] = z;
    if constexpr (CHAIN == LTE_CHAIN_CODED) {
      const float s2 = 1.0f / snr_lin[b];
      float nv = s2;
      if (rayleigh) nv = fmaxf(s2 / fminf(fmaxf(den[q], 1e-6f), 1e6f), s2 * 0.25f);
      if (nvo) {   // demap in k_dematch_zn: hand over the equalised symbol and its noise variance
        reinterpret_cast<float2*>(llr)[fre + re] = z;
        nvo[fre + re] = nv;
        continue;
      }
      float o[BPS];
      soft_demap<BPS>(z, nv, o);
      float* lo = llr + (fre + re) * BPS;
      if constexpr (BPS == 4) {
        *reinterpret_cast<float4*>(lo) = make_float4(o[0], o[1], o[2], o[3]);
      } else {
#pragma unroll
        for (int m = 0; m < BPS; m += 2) *reinterpret_cast<float2*>(lo + m) = make_float2(o[m], o[m + 1]);
      }
    } else {
      const int idx = hard_index(z, BPS, QS);
      const int64_t pb0 = (int64_t)re * BPS;
#pragma unroll
      for (int m = 0; m < BPS; ++m) {
        const int64_t pbit = pb0 + m;
        if (pbit < n_bits) {
          const uint32_t bit = (idx >> (BPS - 1 - m)) & 1;
          errs += bit ^ getbit(fb, pbit);
          if (cap_bits) cap_bits[(size_t)b * n_bits + pbit] = (uint8_t)bit;
        }
      }
    }
  }
  // one atomic per frame per wave (all lanes reach this point; inactive lanes carry 0)
  if constexpr (CHAIN != LTE_CHAIN_CODED) frame_err_add(frame_err, b, errs);
}

template <int CHAIN, int BPS, bool SCF, int NC = 0>
static void rx_data_inst(hipStream_t s, int blocks, size_t shm, const Grid& g, int rayleigh, int B, int num_rx,
                         const float2* y, int64_t y_rx_stride, int64_t y_frame_stride, const float2* H,
                         const float* npow, const float* snr_lin, const uint64_t* fid, uint64_t seed,
                         const float* inj_z, int64_t inj_stride, const uint32_t* pw, int PW, int n_bits,
                         uint32_t* frame_err, float* llr, float2* cap_syms, uint8_t* cap_bits, float* nvo) {
  hipLaunchKernelGGL((k_rx_data<CHAIN, BPS, SCF, NC>), dim3(blocks), dim3(WG), shm, s, g, rayleigh, B, num_rx, y,
                     y_rx_stride, y_frame_stride, H, npow, snr_lin, fid, seed, inj_z, inj_stride, pw, PW, n_bits,
                     frame_err, llr, cap_syms, cap_bits, nvo);
}

template <int CHAIN, bool SCF = false, int NC = 0>
static void rx_data_bps(int bps, hipStream_t s, int blocks, size_t shm, const Grid& g, int rayleigh, int B,
                        int num_rx, const float2* y, int64_t y_rx_stride, int64_t y_frame_stride, const float2* H,
                        const float* npow, const float* snr_lin, const uint64_t* fid, uint64_t seed,
                        const float* inj_z, int64_t inj_stride, const uint32_t* pw, int PW, int n_bits,
                        uint32_t* frame_err, float* llr, float2* cap_syms, uint8_t* cap_bits, float* nvo) {
  auto* f = bps == 2 ? &rx_data_inst<CHAIN, 2, SCF, NC>
                     : (bps == 4 ? &rx_data_inst<CHAIN, 4, SCF, NC> : &rx_data_inst<CHAIN, 6, SCF, NC>);
  f(s, blocks, shm, g, rayleigh, B, num_rx, y, y_rx_stride, y_frame_stride, H, npow, snr_lin, fid, seed, inj_z,
    inj_stride, pw, PW, n_bits, frame_err, llr, cap_syms, cap_bits, nvo);
}

int launch_rx_data(hipStream_t s, const Grid& g, int chain, int rayleigh, int B, int num_rx, const float2* y,
                   int64_t y_rx_stride, int64_t y_frame_stride, const float2* H, const float* npow,
                   const float* snr_lin, const uint64_t* fid, uint64_t seed, const float* inj_z, int64_t inj_stride,
                   const uint32_t* pw, int PW, int n_bits, uint32_t* frame_err, float* llr, float2* cap_syms,
                   uint8_t* cap_bits, int sc_fdm, float* nv_out) {
  if (g.bps != 2 && g.bps != 4 && g.bps != 6) return (int)hipErrorInvalidValue;
  if (nv_out && chain != LTE_CHAIN_CODED) return (int)hipErrorInvalidValue;
  if (sc_fdm && (chain != LTE_CHAIN_UNCODED || !g.chirp || !g.bhat)) return (int)hipErrorInvalidValue;
  if (chain == LTE_CHAIN_SIMO && num_rx > 8) return (int)hipErrorInvalidValue;
  const int spw = WG / (g.N >> 3);
  const int64_t total = (int64_t)B * g.n_sym;
  if (total > 0x7FFFFFFF - spw) return (int)hipErrorInvalidValue;
  const int blocks = (int)((total + spw - 1) / spw);
  const size_t shm = spw * g.N * sizeof(float2);
  if (chain == LTE_CHAIN_CODED && g.N == 2048)   // the headline chain: compile-time FFT size
    rx_data_bps<LTE_CHAIN_CODED, false, 2048>(g.bps, s, blocks, shm, g, rayleigh, B, num_rx, y, y_rx_stride,
                                              y_frame_stride, H, npow, snr_lin, fid, seed, inj_z, inj_stride, pw, PW,
                                              n_bits, frame_err, llr, cap_syms, cap_bits, nv_out);
  else if (chain == LTE_CHAIN_CODED)
    rx_data_bps<LTE_CHAIN_CODED>(g.bps, s, blocks, shm, g, rayleigh, B, num_rx, y, y_rx_stride, y_frame_stride, H,
                                 npow, snr_lin, fid, seed, inj_z, inj_stride, pw, PW, n_bits, frame_err, llr,
                                 cap_syms, cap_bits, nv_out);
  else if (chain == LTE_CHAIN_SIMO)
    rx_data_bps<LTE_CHAIN_SIMO>(g.bps, s, blocks, shm, g, rayleigh, B, num_rx, y, y_rx_stride, y_frame_stride, H,
                                npow, snr_lin, fid, seed, inj_z, inj_stride, pw, PW, n_bits, frame_err, llr,
                                cap_syms, cap_bits, nullptr);
  else if (sc_fdm)
    rx_data_bps<LTE_CHAIN_UNCODED, true>(g.bps, s, blocks, shm, g, rayleigh, B, num_rx, y, y_rx_stride,
                                         y_frame_stride, H, npow, snr_lin, fid, seed, inj_z, inj_stride, pw, PW,
                                         n_bits, frame_err, llr, cap_syms, cap_bits, nullptr);
  else
    rx_data_bps<LTE_CHAIN_UNCODED>(g.bps, s, blocks, shm, g, rayleigh, B, num_rx, y, y_rx_stride, y_frame_stride,
                                   H, npow, snr_lin, fid, seed, inj_z, inj_stride, pw, PW, n_bits, frame_err, llr,
                                   cap_syms, cap_bits, nullptr);
  return (int)hipGetLastError();
}

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
// Stage kernels for the parity entry points.
__global__ __launch_bounds__(WG) void k_fft_batch(Grid g, int inverse, int64_t batch, const float2* __restrict__ in,
                                                  float2* __restrict__ out) {
  extern __shared__ float2 sm[];
  const int N = g.N, T = N >> 3, spw = WG / T;
  const int slot = threadIdx.x / T, tid = threadIdx.x % T;
  const int64_t i = (int64_t)blockIdx.x * spw + slot;
  const bool active = slot < spw && i < batch;
  float2* buf = sm + slot * N;
  if (active)
    for (int k = tid; k < N; k += T) buf[k] = in[i * N + k];
  __syncthreads();
  if (inverse) fft_lds<true>(buf, N, g.log2N, g.tw, tid, active);
  else fft_lds<false>(buf, N, g.log2N, g.tw, tid, active);
  if (active) {
    const float sc = rsqrtf((float)N);
    for (int k = tid; k < N; k += T) out[i * N + k] = cscale(buf[k], sc);
  }
}

int launch_fft(hipStream_t s, const Grid& g, int inverse, int64_t batch, const float2* in, float2* out) {
  const int spw = WG / (g.N >> 3);
  const int blocks = (int)((batch + spw - 1) / spw);
  hipLaunchKernelGGL(k_fft_batch, dim3(blocks), dim3(WG), spw * g.N * sizeof(float2), s, g, inverse, batch, in, out);
  return (int)hipGetLastError();
}

template <int BPS>
__global__ void k_llr(int64_t n, const float2* __restrict__ syms, const float* __restrict__ nv,
                      float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float o[BPS];
  soft_demap<BPS>(syms[i], nv[i], o);
#pragma unroll
  for (int m = 0; m < BPS; ++m) out[i * BPS + m] = o[m];
}

int launch_llr(hipStream_t s, int bps, int64_t n, const float2* syms, const float* nv, float* llr) {
  const dim3 grid((unsigned)((n + WG - 1) / WG));
  if (bps == 2) hipLaunchKernelGGL(k_llr<2>, grid, dim3(WG), 0, s, n, syms, nv, llr);
  else if (bps == 4) hipLaunchKernelGGL(k_llr<4>, grid, dim3(WG), 0, s, n, syms, nv, llr);
  else if (bps == 6) hipLaunchKernelGGL(k_llr<6>, grid, dim3(WG), 0, s, n, syms, nv, llr);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

template <int BPS>
__global__ void k_hard(int64_t n, const float2* __restrict__ syms, uint8_t* __restrict__ bits) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int idx = hard_index(syms[i], BPS, (float)qam_norm<BPS>());
#pragma unroll
  for (int m = 0; m < BPS; ++m) bits[i * BPS + m] = (idx >> (BPS - 1 - m)) & 1;
}

int launch_hard(hipStream_t s, int bps, int64_t n, const float2* syms, uint8_t* bits) {
  const dim3 grid((unsigned)((n + WG - 1) / WG));
  if (bps == 2) hipLaunchKernelGGL(k_hard<2>, grid, dim3(WG), 0, s, n, syms, bits);
  else if (bps == 4) hipLaunchKernelGGL(k_hard<4>, grid, dim3(WG), 0, s, n, syms, bits);
  else if (bps == 6) hipLaunchKernelGGL(k_hard<6>, grid, dim3(WG), 0, s, n, syms, bits);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Stage entry: batched SC-FDM DFT / IDFT of size M = g.Nd (DFTPrecodifier.
// precoding / IDFTDecodifier.decoding, core/dft_precoding.py:66-118, 199-226)
// on host-supplied vectors; one slot per vector, the same dft_bluestein the
// chains run in-line.
__global__ __launch_bounds__(WG) void k_dft_stage(Grid g, int inverse, int64_t batch, const float2* __restrict__ in,
                                                  float2* __restrict__ out) {
  extern __shared__ float2 sm[];
  const int N = g.N, T = N >> 3, spw = WG / T;
  const int slot = threadIdx.x / T, tid = threadIdx.x % T;
  const int64_t v = (int64_t)blockIdx.x * spw + slot;
  const bool active = slot < spw && v < batch;
  float2* buf = sm + slot * N;
  if (active) {
    for (int k = tid; k < N; k += T) {
      float2 x = k < g.Nd ? in[v * g.Nd + k] : make_float2(0.f, 0.f);
      if (inverse) x.y = -x.y;
      buf[k] = x;
    }
  }
  dft_bluestein(buf, g, tid, T, active);
  if (active)
    for (int k = tid; k < g.Nd; k += T) {
      float2 x = buf[k];
      if (inverse) x.y = -x.y;
      out[v * g.Nd + k] = x;
    }
}

int launch_dft(hipStream_t s, const Grid& g, int inverse, int64_t batch, const float2* in, float2* out) {
  const int spw = WG / (g.N >> 3);
  const int64_t blocks = (batch + spw - 1) / spw;
  if (blocks > 0x7FFFFFFF || !g.chirp || !g.bhat || 2 * g.Nd - 1 > g.N) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_dft_stage, dim3((unsigned)blocks), dim3(WG), spw * g.N * sizeof(float2), s, g, inverse, batch,
                     in, out);
  return (int)hipGetLastError();
}

}  // namespace lte
