// Multi-antenna chains for gfx950:
//  * SFBC Alamouti 2 x num_rx (OFDMSimulator.simulate_miso / simulate_mimo,
//    core/ofdm_core.py:1850-2258; config 4 = the same plus turbo coding),
//  * TM4 spatial multiplexing, 2 / 4 TX, 1-4 RX, rank 1-4, codebook precoder W,
//    MMSE / ZF / SIC / MRC (simulate_spatial_multiplexing,
//    core/ofdm_core.py:2489-2815; config 5 = 4x4 rank 4 MMSE).
// Every kernel is one template over the arithmetic type R: double (the
// default; the reference computes in complex128) or float (fast mode), V =
// cx<R>.  The float64 instances follow the reference's operation order where
// it is cheap to (NumPy scalar semantics in the SFBC combiner, the exact Jakes
// sum per sample for fD != 0); the float32 ones keep their shortcuts.
// Per frame:  TX  one slot per (frame, OFDM symbol, TX antenna): QAM map ->
//                 SFBC pair coding / layer mapping -> per-TX CRS pilots -> IFFT + CP
//             CH  per link path coefficients (Jakes: fD = 0 constant; fD != 0
//                 f64 the exact sum per sample, f32 a per-symbol quadratic
//                 expansion), sum over TX, measured-power noise per RX
//                 (transmit_mimo / transmit_spatial_multiplexing)
//             RX  one slot per (frame, RX, OFDM symbol): noise + CP removal + FFT;
//                 on estimation symbols LS at each TX's pilot subset + linear
//                 interpolation (MIMOChannelEstimatorPeriodic); data SCs to HBM
//             DET SFBC combine averaged over RX -> hard bits / LLRs, or a
//                 float64 MMSE / ZF / SIC / MRC per subcarrier -> hard bits.
#include "lte_common.h"
#include "lte_internal.h"
#include "lte_dev.h"
#include "lte_wfft.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace lte {

constexpr int MWG = 256;

template <class V>
__device__ __forceinline__ V* mimo_lds() {
  extern __shared__ double2 lte_mimo_lds[];
  return reinterpret_cast<V*>(lte_mimo_lds);
}

// ---------------------------------------------------------------------------
// TX.  SFBCAlamouti.encode (core/sfbc_alamouti.py:45-78) + SFBCResourceMapper
// (:213-256): data RE j of symbol l carries, for the pair (s0, s1) =
// (q[l*res + (j&~1)], q[.. + 1]): TX0 [s0, -conj(s1)], TX1 [s1, conj(s0)].
// Spatial (core/ofdm_core.py:2596-2655): layer c = q[R j + c] on data SC j <
// ceil(Nd/R) (Q20), x_t = sum_c W[t][c] layer_c.  Pilots: TX t at its subset
// (cell t % 4).  x = ifft(grid) sqrt(N) (tx_scale), CP prepended.
// QAM code of coded symbol q: the constellation index, or -1 for a padding
// symbol (zero)
template <int CODED, int BPS>
__device__ __forceinline__ int qam_code(int64_t q, const uint32_t* __restrict__ fb, const uint32_t* __restrict__ fe,
                                        const int32_t* __restrict__ tx_map) {
  int idx = 0;
  bool zero = false;
  if constexpr (CODED) {
#pragma unroll
    for (int m = 0; m < BPS; ++m) {
      const int src = tx_map[q * BPS + m];
      zero |= src == -2;
      idx = (idx << 1) | (int)(src >= 0 ? getbit(fe, src) : 0u);
    }
  } else {
    idx = (int)getbits<BPS>(fb, q * BPS, INT64_MAX);
  }
  return zero ? -1 : idx;
}
// the QAM codes of coded symbols q and q + 1 (q even, tx_map 16-B aligned):
// their 2 BPS tx_map entries as BPS / 2 16-B loads instead of 2 BPS 4-B loads
template <int BPS>
__device__ __forceinline__ void qam_code_pair(int64_t q, const uint32_t* __restrict__ fe,
                                              const int32_t* __restrict__ tx_map, int& c0, int& c1) {
  int src[2 * BPS];
  const int4* m4 = reinterpret_cast<const int4*>(tx_map + q * BPS);
#pragma unroll
  for (int i = 0; i < BPS / 2; ++i) {
    const int4 v = m4[i];
    src[4 * i] = v.x;
    src[4 * i + 1] = v.y;
    src[4 * i + 2] = v.z;
    src[4 * i + 3] = v.w;
  }
  int c[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    int idx = 0;
    bool zero = false;
#pragma unroll
    for (int m = 0; m < BPS; ++m) {
      const int sv = src[u * BPS + m];
      zero |= sv == -2;
      idx = (idx << 1) | (int)(sv >= 0 ? getbit(fe, sv) : 0u);
    }
    c[u] = zero ? -1 : idx;
  }
  c0 = c[0];
  c1 = c[1];
}
template <class R, int BPS>
__device__ __forceinline__ cx<R> qam_of(int code) {
  return code < 0 ? mkc((R)0, (R)0) : qam_point<BPS, R>(code);
}
template <class R, int CODED, int BPS>
__device__ __forceinline__ cx<R> qam_at(int64_t q, const uint32_t* __restrict__ fb, const uint32_t* __restrict__ fe,
                                        const int32_t* __restrict__ tx_map) {
  return qam_of<R, BPS>(qam_code<CODED, BPS>(q, fb, fe, tx_map));
}

// transmit_mimo's per-link power pass (core/ofdm_core.py:490-503: each
// Rayleigh link's 100 dB ChannelSimulator measures mean |y0|^2 of its own faded
// signal) done on the symbol while it is in LDS: for every RX r, the power of
// y0[m] = sum_p c_{r,t,p} x[m - d_p] over the CP-extended symbol's samples m in
// [max_delay, S) -- every delayed sample inside the symbol (sample j of the
// extended symbol is buf[(j - cp) mod N] * sc, the values x holds).  The first
// max_delay samples, whose taps reach into the previous symbol, are added by
// k_link_power_fix from x.  Static taps only (n_cs = 1); part[link][l].

#ifndef LTE_TXM_LPG   // receive antennas per group of the TX link-power sums (each delayed sample read once per group)
#define LTE_TXM_LPG 2
#endif
// PF (coded): one slot per frame walking its (OFDM symbol, TX) pairs, the
// frame's coded streams staged in LDS once instead of once per pair (as
// k_ofdm_txf does for SISO); otherwise one slot per (frame, symbol, TX).
template <class R, int MODE, int CODED, int BPS, int NC = 0, bool PF = false>
__global__ __launch_bounds__(MWG, PF ? 3 : 1) void k_ofdm_tx_mimo(Grid g, MimoGrid m, const uint32_t* __restrict__ pw, int PW,
                                                      const uint32_t* __restrict__ enc, int enc_words,
                                                      const int32_t* __restrict__ tx_map, cx<R>* __restrict__ x,
                                                      int B, int stage_enc, TxLinkPower<R> lp) {
  using V = cx<R>;
  V* sm = mimo_lds<V>();
  const int N = NC ? NC : g.N, T = N >> 3, spw = MWG / T;
  const int slot = threadIdx.x / T, tid0 = threadIdx.x % T;
  const int per = g.n_sym * m.num_tx;
  const int gs = blockIdx.x * spw + slot;
  const int b = PF ? gs : gs / per;
  const int lt0 = PF ? 0 : gs - b * per, lt1 = PF ? per : lt0 + 1;
  const bool active = slot < spw && b < B;
  V* buf = sm + slot * N;
  // coded: the frame's coded streams are staged in LDS (coalesced), so the
  // rate-match / interleaver bit gathers hit LDS (as in k_ofdm_tx)
  const uint32_t* fe = enc + (size_t)b * enc_words;
  if (CODED && stage_enc) {
    uint32_t* es = reinterpret_cast<uint32_t*>(sm + spw * N) + slot * enc_words;
    if (active)
      for (int i = tid0; i < enc_words; i += T) es[i] = fe[i];
    fe = es;
  }
  // PF SFBC: each thread's Alamouti pairs (at most SFP per symbol) keep their
  // QAM codes from TX 0 to TX 1 of the same symbol (the bit gathers once)
  constexpr int SFP = 4;
  int qc[SFP][2];
  for (int lt = lt0; lt < lt1; ++lt) {
  const int l = lt / m.num_tx, t = lt - l * m.num_tx;
  // opaque per pair (PF): the FFT's twiddle addressing is not hoisted out of
  // the loop into registers
  int tid = tid0;
  if (PF) asm volatile("" : "+v"(tid));
  if (active)
    for (int k = tid; k < N; k += T) buf[k] = mkc((R)0, (R)0);
  __syncthreads();   // (first pair: also the staged streams)
  if (active && MODE == MIMO_SFBC && PF) {   // one thread per pair, both REs
    const uint32_t* fb = pw + (size_t)b * PW;
    const int64_t q0 = (int64_t)l * m.res;
#pragma unroll
    for (int k = 0; k < SFP; ++k) {
      const int j = 2 * (tid + k * T);
      if (j >= m.n_dsc) break;
      if (t == 0) {
        qc[k][0] = qam_code<CODED, BPS>(q0 + j, fb, fe, tx_map);
        qc[k][1] = qam_code<CODED, BPS>(q0 + j + 1, fb, fe, tx_map);
      }
      const V s0 = qam_of<R, BPS>(qc[k][0]), s1 = qam_of<R, BPS>(qc[k][1]);
      buf[g.data_idx[j]] = t == 0 ? s0 : s1;
      if (j + 1 < m.n_dsc) buf[g.data_idx[j + 1]] = t == 0 ? mkc(-s1.x, s1.y) : mkc(s0.x, -s0.y);
    }
    const int npt = m.np_tx[t];
    const V* pv = MGT<R>::pval(m) + t * m.maxP;
    for (int p = tid; p < npt; p += T) buf[m.ppos[t * m.maxP + p]] = pv[p];
  } else if (active) {
    const uint32_t* fb = pw + (size_t)b * PW;
    const int64_t q0 = (int64_t)l * m.res;
    for (int j = tid; j < m.n_dsc; j += T) {
      V v;
      if constexpr (MODE == MIMO_SFBC) {
        const int64_t qp = q0 + (j & ~1);
        const V s0 = qam_at<R, CODED, BPS>(qp, fb, fe, tx_map), s1 = qam_at<R, CODED, BPS>(qp + 1, fb, fe, tx_map);
        if ((j & 1) == 0) v = t == 0 ? s0 : s1;
        else v = t == 0 ? mkc(-s1.x, s1.y) : mkc(s0.x, -s0.y);   // -conj(s1) / conj(s0)
      } else {
        v = mkc((R)0, (R)0);
        for (int c = 0; c < m.rank; ++c) {
          const int qi = m.rank * j + c;
          if (qi >= m.res) break;
          const V w = mkc((R)m.W[(t * 4 + c) * 2], (R)m.W[(t * 4 + c) * 2 + 1]);
          // a zero precoder entry adds a signed zero to a nonzero sum (every
          // constellation point is nonzero): skip its bit gathers (W = I: 3 of 4)
          if (w.x == (R)0 && w.y == (R)0) continue;
          const V sq = qam_at<R, CODED, BPS>(q0 + qi, fb, fe, tx_map);
          v = cadd(v, cmul(w, sq));
        }
      }
      buf[g.data_idx[j]] = v;
    }
    const int npt = m.np_tx[t];
    const V* pv = MGT<R>::pval(m) + t * m.maxP;
    for (int p = tid; p < npt; p += T) buf[m.ppos[t * m.maxP + p]] = pv[p];
  }
  __syncthreads();
  fft_lds<true, NC>(buf, N, g.log2N, GridT<R>::tw(g), tid, active);
  const R sc = tx_scale<R>(N);
  if (active) {
    V* xo = x + ((size_t)b * m.num_tx + t) * g.L + (size_t)l * (N + g.cp);
    for (int k = tid; k < N; k += T) xo[g.cp + k] = cscale(buf[k], sc);
    for (int k = tid; k < g.cp; k += T) xo[k] = cscale(buf[N - g.cp + k], sc);
  }
  if (lp.part) {   // whole waves per slot (T >= 64): launch_ofdm_tx_mimo checks
    __shared__ R red[MWG / 64];
    constexpr int NCF = mimo_ncf<R>();
    const int S = N + g.cp, D = lp.max_delay, np = lp.n_paths;
    int dl[TXCH_MAXP];
#pragma unroll
    for (int p = 0; p < TXCH_MAXP; ++p) dl[p] = p < np ? g.cp + lp.delays[p] : 0;
    // receive antennas in groups of LPG: each delayed sample x(j - d_p) is
    // read from LDS (and scaled) once for the group's links
    constexpr int LPG = LTE_TXM_LPG;
    for (int r0 = 0; r0 < m.num_rx; r0 += LPG) {
      R pwr[LPG];
#pragma unroll
      for (int q = 0; q < LPG; ++q) pwr[q] = (R)0;
      if (active) {
        V c[LPG][TXCH_MAXP];
#pragma unroll
        for (int q = 0; q < LPG; ++q) {
          const int r = min(r0 + q, m.num_rx - 1);
          const V* cf = lp.coef + (((size_t)b * m.num_rx + r) * m.num_tx + t) * np * NCF;
#pragma unroll
          for (int p = 0; p < TXCH_MAXP; ++p) c[q][p] = p < np ? cf[p * NCF] : mkc((R)0, (R)0);
        }
        for (int j = D + tid; j < S; j += T) {
          V acc[LPG];
#pragma unroll
          for (int q = 0; q < LPG; ++q) acc[q] = mkc((R)0, (R)0);
#pragma unroll
          for (int p = 0; p < TXCH_MAXP; ++p)
            if (p < np) {
              const V xv = cscale(buf[(j - dl[p]) & (N - 1)], sc);
#pragma unroll
              for (int q = 0; q < LPG; ++q) acc[q] = cadd(acc[q], cmul(c[q][p], xv));
            }
#pragma unroll
          for (int q = 0; q < LPG; ++q) pwr[q] += acc[q].x * acc[q].x + acc[q].y * acc[q].y;
        }
      }
#pragma unroll
      for (int q = 0; q < LPG; ++q) {
        if (r0 + q >= m.num_rx) break;
        R pv = pwr[q];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) pv += __shfl_xor(pv, o);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = pv;
        __syncthreads();
        if (active && tid == 0) {
          R tot = (R)0;
          for (int w = 0; w < T / 64; ++w) tot += red[slot * (T / 64) + w];
          lp.part[(((size_t)b * m.num_rx + r0 + q) * m.num_tx + t) * lp.nblk + l] = tot;
        }
        __syncthreads();
      }
    }
  }
  if (PF) __syncthreads();   // the next pair zeroes buf
  }
}

// TX + flat channel in one pass (AWGN links: spatial h ~ CN(0,1), SFBC h =
// exp(j t pi/2)): one slot per (frame, OFDM symbol, RX).  A flat link is a
// scalar, so y_r = sum_t h_rt x_t = IFFT(sum_t h_rt G_t) sqrt(N): the slot
// builds Y = sum_t h_rt G_t (each TX's data REs and its own pilot subset, t in
// order from zero) in LDS, runs ONE IFFT per RX instead of one per TX, and
// writes the received stream y (CP included) and its power partial per symbol
// -- the TX streams x never go through HBM and the channel pass disappears.
// The same sums as ys[r] += hh * xs[t] (core/channel.py:473-491) taken in the
// frequency domain, and for spatial layers through the effective channel h_r W
// (x_t = sum_c W[t][c] s_c): equal up to float64 rounding (the reference adds
// the time-domain products), tests/test_gpu_mimo.py::test_flat_channel_fused_tx.
// PR (spatial): one slot per (frame, OFDM symbol) walking the receive
// antennas, each thread's layer QAM codes formed at the first RX and reused
// for the others (the bit gathers once per symbol instead of once per RX).
template <class R, int MODE, int CODED, int BPS, int NC = 0, bool PR = false>
__global__ __launch_bounds__(MWG) void k_ofdm_txch_flat(Grid g, MimoGrid m, const uint32_t* __restrict__ pw, int PW,
                                                        const uint32_t* __restrict__ enc, int enc_words,
                                                        const int32_t* __restrict__ tx_map,
                                                        const cx<R>* __restrict__ coef, cx<R>* __restrict__ y,
                                                        R* __restrict__ pow_part, int nblk, int B, int stage_enc) {
  using V = cx<R>;
  constexpr int NCF = mimo_ncf<R>();
  __shared__ R red[MWG / 64];
  V* sm = mimo_lds<V>();
  const int N = NC ? NC : g.N, T = N >> 3, spw = MWG / T;
  const int slot = threadIdx.x / T, tid0 = threadIdx.x % T;
  const int per = PR ? g.n_sym : g.n_sym * m.num_rx;
  const int gs = blockIdx.x * spw + slot;
  const int b = gs / per, rr = gs - b * per;
  const int l = PR ? rr : rr / m.num_rx;
  const int r0 = PR ? 0 : rr - l * m.num_rx, r1 = PR ? m.num_rx : r0 + 1;
  const bool active = slot < spw && b < B;
  V* buf = sm + slot * N;
  const uint32_t* fe = enc + (size_t)b * enc_words;
  if (CODED && stage_enc) {
    uint32_t* es = reinterpret_cast<uint32_t*>(sm + spw * N) + slot * enc_words;
    if (active)
      for (int i = tid0; i < enc_words; i += T) es[i] = fe[i];
    fe = es;
  }
  constexpr int QC = 4;   // data subcarriers per thread: n_dsc < N / 2 = QC T
  int codes[QC][4];
#pragma unroll 1
  for (int r = r0; r < r1; ++r) {
  // opaque per RX (PR): the FFT's twiddle addressing is not hoisted out of
  // the loop into registers (as k_ofdm_txf does per symbol)
  int tid = tid0;
  if (PR) asm volatile("" : "+v"(tid));
  if (active)
    for (int k = tid; k < N; k += T) buf[k] = mkc((R)0, (R)0);
  __syncthreads();
  if (active) {
    const uint32_t* fb = pw + (size_t)b * PW;
    const int64_t q0 = (int64_t)l * m.res;
    const V* hr = coef + ((size_t)b * m.num_rx + r) * m.num_tx * NCF;   // h_rt at hr[t * NCF]
    V E[4];   // spatial: the effective channel of RX r, E_c = sum_t h_rt W[t][c]
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      E[c] = mkc((R)0, (R)0);
      if (MODE == MIMO_SPATIAL && c < m.rank)
        for (int t = 0; t < m.num_tx; ++t)
          E[c] = cadd(E[c], cmul(hr[t * NCF], mkc((R)m.W[(t * 4 + c) * 2], (R)m.W[(t * 4 + c) * 2 + 1])));
    }
    if constexpr (PR && MODE == MIMO_SPATIAL) {
#pragma unroll
      for (int k = 0; k < QC; ++k) {
        const int j = tid + k * T;
        if (j >= m.n_dsc) break;
        V acc = mkc((R)0, (R)0);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int qi = m.rank * j + c;
          if (c < m.rank && qi < m.res) {
            if (r == r0) codes[k][c] = qam_code<CODED, BPS>(q0 + qi, fb, fe, tx_map);
            acc = cadd(acc, cmul(E[c], qam_of<R, BPS>(codes[k][c])));
          }
        }
        buf[g.data_idx[j]] = acc;
      }
    } else {
    for (int j = tid; j < m.n_dsc; j += T) {
      V acc = mkc((R)0, (R)0);
      if constexpr (MODE == MIMO_SFBC) {
        const int64_t qp = q0 + (j & ~1);
        const V s0 = qam_at<R, CODED, BPS>(qp, fb, fe, tx_map), s1 = qam_at<R, CODED, BPS>(qp + 1, fb, fe, tx_map);
        const V v0 = (j & 1) == 0 ? s0 : mkc(-s1.x, s1.y);   // TX0 [s0, -conj(s1)]
        const V v1 = (j & 1) == 0 ? s1 : mkc(s0.x, -s0.y);   // TX1 [s1, conj(s0)]
        acc = cadd(cmul(hr[0], v0), cmul(hr[NCF], v1));
      } else {   // sum_t h_rt (W s)_t = sum_c E_c s_c, E = (h_r W) formed once per thread
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int qi = m.rank * j + c;
          if (c < m.rank && qi < m.res) acc = cadd(acc, cmul(E[c], qam_at<R, CODED, BPS>(q0 + qi, fb, fe, tx_map)));
        }
      }
      buf[g.data_idx[j]] = acc;
    }
    }
    for (int t = 0; t < m.num_tx; ++t) {   // each TX's CRS pilots on its own subset
      const V* pv = MGT<R>::pval(m) + t * m.maxP;
      const V h = hr[t * NCF];
      for (int p = tid; p < m.np_tx[t]; p += T) {
        V& e = buf[m.ppos[t * m.maxP + p]];
        e = cadd(e, cmul(h, pv[p]));
      }
    }
  }
  __syncthreads();
  fft_lds<true, NC>(buf, N, g.log2N, GridT<R>::tw(g), tid, active);
  const R sc = tx_scale<R>(N);
  R pwr = (R)0;
  if (active) {
    V* yo = y + ((size_t)b * m.num_rx + r) * g.L + (size_t)l * (N + g.cp);
    for (int k = tid; k < N; k += T) {
      const V v = cscale(buf[k], sc);
      yo[g.cp + k] = v;
      pwr += v.x * v.x + v.y * v.y;
    }
    for (int k = tid; k < g.cp; k += T) {
      const V v = cscale(buf[N - g.cp + k], sc);
      yo[k] = v;
      pwr += v.x * v.x + v.y * v.y;
    }
  }
  if (T >= 64) {   // whole waves per slot
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) pwr += __shfl_xor(pwr, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = pwr;
    __syncthreads();
    if (active && tid == 0) {
      R tot = (R)0;
      for (int w = 0; w < T / 64; ++w) tot += red[slot * (T / 64) + w];
      pow_part[((size_t)b * m.num_rx + r) * nblk + l] = tot;
    }
  }
  if (PR) __syncthreads();   // the next RX zeroes buf and reuses red
  }
}

// Wave-private spatial TX + flat links (float64, N = 2048; k_ofdm_txch_flat's
// outputs): one wave64 per (frame, RX antenna) walks the frame's symbols.  The
// effective channel E_c = sum_t h_rt W[t][c] is formed once per wave.  Per
// symbol, lane c, register q gets bin k = 64 q + c of Y_r = sum_t h_rt G_t
// (formed half a symbol at a time by a rolled loop through the wave's LDS,
// from Grid::kinfo): a data SC j < n_dsc carries
// sum_c E_c s_c (the same terms in the same order as the block kernel), pilot
// i of the grid is TX t = i % step's pilot i / step (plan_mimo_tables' split)
// times h_rt, anything else 0; wfft::fft2048<INV> and the output scale give
// y_r[64 q + c], written with its CP (1 KB per wave store) and summed into the
// symbol's power partial by one wave reduction.  No block barrier, and the
// only LDS is the transform's 16.5 KB per wave.  The transform's and the
// power sum's rounding differ from the block kernel's (a few 1e-14).
constexpr int TXMW_WAVES = 4;
constexpr int TXMW_LDS = wfft::LDS_DOUBLES + 8;   // doubles per wave: the transform + E
#ifndef TXMW_WPE
#define TXMW_WPE 2
#endif
#ifndef TXMW_BIN_UNROLL
#define TXMW_BIN_UNROLL 8
#endif
template <int CODED, int BPS>
__global__ __launch_bounds__(64 * TXMW_WAVES) __attribute__((amdgpu_waves_per_eu(TXMW_WPE, TXMW_WPE)))
void k_ofdm_txch_flat_w(Grid g, MimoGrid m, const uint32_t* __restrict__ pw, int PW, const uint32_t* __restrict__ enc,
                        int enc_words, const int32_t* __restrict__ tx_map, const double2* __restrict__ coef,
                        double2* __restrict__ y, double* __restrict__ pow_part, int nblk, int B) {
  constexpr int N = 2048, NCF = mimo_ncf<double>();
  using V = double2;
  extern __shared__ double lte_txmw_lds[];
  const int lane0 = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int gs = blockIdx.x * TXMW_WAVES + w;
  const int b = gs / m.num_rx, r = gs - b * m.num_rx;
  if (b >= B) return;   // uniform per wave; no block barrier below
  double* tl = lte_txmw_lds + (size_t)w * TXMW_LDS;
  V* Es = reinterpret_cast<V*>(tl + wfft::LDS_DOUBLES);   // [4] E_c (in LDS, not registers: live across
                                                          // the transform they pushed it into spills)
  const uint32_t* fb = pw + (size_t)b * PW;
  const uint32_t* fe = enc + (size_t)b * enc_words;
  const size_t br = (size_t)b * m.num_rx + r;
  const V* hr = coef + br * m.num_tx * NCF;   // h_rt at hr[t * NCF]
  if (lane0 < 4) {
    const int c = lane0;
    V e = mkc(0.0, 0.0);
    if (c < m.rank)
      for (int t = 0; t < m.num_tx; ++t)
        e = cadd(e, cmul(hr[t * NCF], mkc(m.W[(t * 4 + c) * 2], m.W[(t * 4 + c) * 2 + 1])));
    Es[c] = e;
  }
  wfft::wave_lds_fence();
  const int step = m.num_tx <= 4 ? m.num_tx : 4;
  const double sc = tx_scale<double>(N);
  const V* pv64 = MGT<double>::pval(m);
  for (int l = 0; l < g.n_sym; ++l) {
    int lane = lane0;   // opaque per symbol (see k_rx_frame_w)
    asm volatile("" : "+v"(lane));
    const int64_t q0 = (int64_t)l * m.res;
    V v[32];
    V* zs = reinterpret_cast<V*>(tl);   // [16][64]: half a symbol's bins
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      // partly rolled: the bin code TXMW_BIN_UNROLL times (unrolled over 32
      // registers it spilled; fully rolled, each bin's kinfo -> payload-bit
      // load chain waited alone)
#pragma unroll TXMW_BIN_UNROLL
      for (int mm = 0; mm < 16; ++mm) {
        const int kq = g.kinfo[64 * (16 * h + mm) + lane];
        V acc = mkc(0.0, 0.0);
        if (kq >= 0 && kq < m.n_dsc) {   // sum_t h_rt (W s)_t = sum_c E_c s_c
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const int qi = m.rank * kq + c;
            if (c < m.rank && qi < m.res)
              acc = cadd(acc, cmul(Es[c], qam_at<double, CODED, BPS>(q0 + qi, fb, fe, tx_map)));
          }
        } else if (kq <= -2) {   // grid pilot i: TX i % step's pilot i / step
          const int i = -kq - 2, t = i % step;
          acc = cmul(hr[t * NCF], pv64[t * m.maxP + i / step]);
        }
        zs[64 * mm + lane] = acc;
      }
      wfft::wave_lds_fence();
#pragma unroll
      for (int i = 0; i < 16; ++i) v[16 * h + i] = zs[64 * i + lane];
      wfft::wave_lds_fence();
    }
    int lane_f = lane;
    asm volatile("" : "+v"(lane_f));
    wfft::fft2048<true>(v, tl, GridT<double>::tw(g), lane_f);
    V* yo = y + br * g.L + (size_t)l * (N + g.cp);
    const int cs = N - g.cp;   // the CP repeats samples cs .. N - 1
    double pwr = 0.0;
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      const V x = cscale(v[q], sc);
      const int n = 64 * q + lane_f;
      yo[g.cp + n] = x;
      const double e = x.x * x.x + x.y * x.y;
      pwr += e;
      if (q >= 24 && n >= cs) {   // (cp <= 512: only the last 8 registers hold CP samples)
        yo[n - cs] = x;
        pwr += e;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) pwr += __shfl_xor(pwr, o);
    if (lane_f == 0) pow_part[br * nblk + l] = pwr;
  }
}

bool txch_flat_w_supported(const Grid& g, const MimoGrid& m, int f64) {
  return f64 && g.N == 2048 && g.kinfo && m.pval64 && m.mode == MIMO_SPATIAL && m.num_tx >= 1 && m.num_tx <= 4 &&
         m.rank >= 1 && m.rank <= 4 && g.cp >= 0 && g.cp <= 512;
}

// Opt-in (profiles/r6_mimo_tx_wave/): the TX itself runs 22.5 against 23.3 ms
// per 32 768 config-5 frames, but the receiver that follows it loses as much
// (26.8-27.1 against 26.4-26.5 ms), so config 5 does not move.
#ifndef LTE_MIMO_TX_WAVE
#define LTE_MIMO_TX_WAVE 0
#endif

template <class R>
int launch_ofdm_txch_flat(hipStream_t s, const Grid& g, const MimoGrid& m, int coded, const uint32_t* pw, int PW,
                          const uint32_t* enc, int enc_words, const int32_t* tx_map, const cx<R>* coef, cx<R>* y,
                          R* pow_part, int nblk, int B) {
  const int spw = MWG / (g.N >> 3);
  // LTE_TXCH_PR=1 (A/B, off by default): spatial, one slot per (frame, symbol)
  // over the receive antennas -- 25.0 vs 23.9 ms per 32 768 config-5 frames
  // (the saved bit gathers do not pay for a quarter of the slots)
  const char* pre = std::getenv("LTE_TXCH_PR");
  const bool pr = m.mode == MIMO_SPATIAL && g.N == 2048 && m.n_dsc <= 4 * (g.N >> 3) && pre && std::atoi(pre) != 0;
  const int64_t total = (int64_t)B * g.n_sym * (pr ? 1 : m.num_rx);
  if (total > 0x7FFFFFFF - spw || (g.bps != 2 && g.bps != 4 && g.bps != 6) || (g.N >> 3) < 64 || nblk < g.n_sym ||
      m.num_tx > 4)
    return (int)hipErrorInvalidValue;
  if constexpr (sizeof(R) == 8) {   // the wave-private kernel (LTE_MIMO_TX_WAVE=1)
    const char* we = std::getenv("LTE_MIMO_TX_WAVE");
    if ((we ? std::atoi(we) != 0 : LTE_MIMO_TX_WAVE) && !pr && txch_flat_w_supported(g, m, 1)) {
      const int64_t waves = (int64_t)B * m.num_rx;
      if (waves > 0x7FFFFFFF - TXMW_WAVES) return (int)hipErrorInvalidValue;
      const unsigned wb = (unsigned)((waves + TXMW_WAVES - 1) / TXMW_WAVES);
      const size_t wshm = (size_t)TXMW_WAVES * TXMW_LDS * sizeof(double);
#define LTE_TXFW(C_, B_)                                                                                             \
  hipLaunchKernelGGL((k_ofdm_txch_flat_w<C_, B_>), dim3(wb), dim3(64 * TXMW_WAVES), wshm, s, g, m, pw, PW, enc,      \
                     enc_words, tx_map, reinterpret_cast<const double2*>(coef), reinterpret_cast<double2*>(y),       \
                     reinterpret_cast<double*>(pow_part), nblk, B)
      if (coded) {
        if (g.bps == 2) LTE_TXFW(1, 2); else if (g.bps == 4) LTE_TXFW(1, 4); else LTE_TXFW(1, 6);
      } else {
        if (g.bps == 2) LTE_TXFW(0, 2); else if (g.bps == 4) LTE_TXFW(0, 4); else LTE_TXFW(0, 6);
      }
#undef LTE_TXFW
      return (int)hipGetLastError();
    }
  }
  const int blocks = (int)((total + spw - 1) / spw);
  const size_t enc_shm = (size_t)spw * enc_words * sizeof(uint32_t);
  const int stage_enc = coded && enc_shm <= 32768;
  const size_t shm = spw * g.N * sizeof(cx<R>) + (stage_enc ? enc_shm : 0);
#define LTE_TXF(M_, C_, B_)                                                                                          \
  do {                                                                                                               \
    if (g.N == 2048 && pr)                                                                                           \
      hipLaunchKernelGGL((k_ofdm_txch_flat<R, M_, C_, B_, 2048, true>), dim3(blocks), dim3(MWG), shm, s, g, m, pw,   \
                         PW, enc, enc_words, tx_map, coef, y, pow_part, nblk, B, stage_enc);                         \
    else if (g.N == 2048)                                                                                            \
      hipLaunchKernelGGL((k_ofdm_txch_flat<R, M_, C_, B_, 2048>), dim3(blocks), dim3(MWG), shm, s, g, m, pw, PW, enc, \
                         enc_words, tx_map, coef, y, pow_part, nblk, B, stage_enc);                                  \
    else                                                                                                             \
      hipLaunchKernelGGL((k_ofdm_txch_flat<R, M_, C_, B_>), dim3(blocks), dim3(MWG), shm, s, g, m, pw, PW, enc,      \
                         enc_words, tx_map, coef, y, pow_part, nblk, B, stage_enc);                                  \
  } while (0)
#define LTE_TXF_BPS(M_, C_) \
  do { if (g.bps == 2) LTE_TXF(M_, C_, 2); else if (g.bps == 4) LTE_TXF(M_, C_, 4); else LTE_TXF(M_, C_, 6); } while (0)
  if (m.mode == MIMO_SFBC) {
    if (coded) LTE_TXF_BPS(MIMO_SFBC, 1); else LTE_TXF_BPS(MIMO_SFBC, 0);
  } else {
    if (coded) LTE_TXF_BPS(MIMO_SPATIAL, 1); else LTE_TXF_BPS(MIMO_SPATIAL, 0);
  }
#undef LTE_TXF_BPS
#undef LTE_TXF
  return (int)hipGetLastError();
}

// The link power of the first max_delay samples of every symbol (their taps
// reach into the previous symbol; stream-level delay with a zero prefix), from
// x, added to k_ofdm_tx_mimo's partial: one lane per (frame, link, symbol).
template <class R>
__global__ __launch_bounds__(MWG) void k_link_power_fix(int B, int num_rx, int num_tx, int n_sym, int sym_len, int L,
                                                        const cx<R>* __restrict__ x, TxLinkPower<R> lp) {
  using V = cx<R>;
  constexpr int NCF = mimo_ncf<R>();
  const int64_t i = (int64_t)blockIdx.x * MWG + threadIdx.x;
  const int64_t nl = (int64_t)num_rx * num_tx;
  if (i >= (int64_t)B * nl * n_sym) return;
  const int l = (int)(i % n_sym);
  const int64_t bl = i / n_sym;              // b * nl + link
  const int b = (int)(bl / nl), link = (int)(bl % nl), t = link % num_tx;
  const V* xf = x + ((size_t)b * num_tx + t) * L;
  const V* cf = lp.coef + (size_t)bl * lp.n_paths * NCF;
  const int n0 = l * sym_len;
  R pwr = (R)0;
  for (int mm = 0; mm < lp.max_delay; ++mm) {
    V acc = mkc((R)0, (R)0);
    for (int p = 0; p < lp.n_paths; ++p) {
      const int src = n0 + mm - lp.delays[p];
      if (src >= 0) acc = cadd(acc, cmul(cf[p * NCF], xf[src]));
    }
    pwr += acc.x * acc.x + acc.y * acc.y;
  }
  lp.part[(size_t)bl * lp.nblk + l] += pwr;
}

template <class R>
int launch_ofdm_tx_mimo(hipStream_t s, const Grid& g, const MimoGrid& m, int coded, const uint32_t* pw, int PW,
                        const uint32_t* enc, int enc_words, const int32_t* tx_map, cx<R>* x, int B,
                        const TxLinkPower<R>& lp) {
  const int spw = MWG / (g.N >> 3);
  const int64_t total = (int64_t)B * g.n_sym * m.num_tx;
  if (total > 0x7FFFFFFF - spw || (g.bps != 2 && g.bps != 4 && g.bps != 6)) return (int)hipErrorInvalidValue;
  if (lp.part && ((g.N >> 3) < 64 || lp.max_delay > g.cp || lp.nblk < g.n_sym || lp.n_paths > TXCH_MAXP))
    return (int)hipErrorInvalidValue;
  const size_t enc_shm = (size_t)spw * enc_words * sizeof(uint32_t);
  const int stage_enc = coded && enc_shm <= 32768;
  const size_t shm = spw * g.N * sizeof(cx<R>) + (stage_enc ? enc_shm : 0);
  // coded frames: one slot per frame over its (symbol, TX) pairs (LTE_TXM_FRAME=0: one per pair)
  const char* pfe = std::getenv("LTE_TXM_FRAME");
  const bool pf = stage_enc && g.N == 2048 && !(pfe && std::atoi(pfe) == 0);
  const int blocks = pf ? (B + spw - 1) / spw : (int)((total + spw - 1) / spw);
#define LTE_TXM(M_, C_, B_)                                                                                          \
  do {                                                                                                               \
    if (g.N == 2048 && pf)                                                                                           \
      hipLaunchKernelGGL((k_ofdm_tx_mimo<R, M_, C_, B_, 2048, true>), dim3(blocks), dim3(MWG), shm, s, g, m, pw, PW, \
                         enc, enc_words, tx_map, x, B, stage_enc, lp);                                               \
    else if (g.N == 2048)   /* 20 MHz: compile-time N (unrolled passes, twiddle recurrence) */                       \
      hipLaunchKernelGGL((k_ofdm_tx_mimo<R, M_, C_, B_, 2048>), dim3(blocks), dim3(MWG), shm, s, g, m, pw, PW, enc,  \
                         enc_words, tx_map, x, B, stage_enc, lp);                                                    \
    else                                                                                                             \
      hipLaunchKernelGGL((k_ofdm_tx_mimo<R, M_, C_, B_>), dim3(blocks), dim3(MWG), shm, s, g, m, pw, PW, enc,        \
                         enc_words, tx_map, x, B, stage_enc, lp);                                                    \
  } while (0)
#define LTE_TXM_BPS(M_, C_) \
  do { if (g.bps == 2) LTE_TXM(M_, C_, 2); else if (g.bps == 4) LTE_TXM(M_, C_, 4); else LTE_TXM(M_, C_, 6); } while (0)
  if (m.mode == MIMO_SFBC) {
    if (coded) LTE_TXM_BPS(MIMO_SFBC, 1); else LTE_TXM_BPS(MIMO_SFBC, 0);
  } else {
    if (coded) LTE_TXM_BPS(MIMO_SPATIAL, 1); else LTE_TXM_BPS(MIMO_SPATIAL, 0);
  }
#undef LTE_TXM_BPS
#undef LTE_TXM
  if (lp.part && lp.max_delay > 0) {
    const int e = (int)hipGetLastError();
    if (e) return e;
    const int64_t n = total * m.num_rx;   // (frame, link, symbol)
    hipLaunchKernelGGL(k_link_power_fix<R>, dim3((unsigned)((n + MWG - 1) / MWG)), dim3(MWG), 0, s, B, m.num_rx,
                       m.num_tx, g.n_sym, g.N + g.cp, g.L, x, lp);
  }
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Link fading.  One thread per (frame, rx, tx, path).  Rayleigh:
// RayleighChannel.jakes_fading (core/rayleighchannel.py:20-42) with 16 phases
// (injected, or Philox): h(n) = g sqrt(2/16) sum_m exp(j(w_m n / fs + phi_m)),
// w_m = (2 pi fD) cos(2 pi (m+1)/16).
//  * fD == 0: the constant A = g (sqrt(2/16) sum_m exp(j phi_m)) -- f64 in the
//    reference's order (phi_m is then exactly the argument);
//  * fD != 0, f64: per OFDM symbol s with centre c_s the degree-5 Taylor
//    expansion h(c_s + d) = sum_k c_k d^k, c_k = g sqrt(2/16) sum_m a_m
//    (j W_m)^k / k!, a_m = exp(j (w_m t_c + phi_m)) formed like one reference
//    sample, W_m = w_m / fs (|W d| <= 1.3e-3 rad at 3 km/h, 20 MHz: remainder
//    < 1e-17, under float64 rounding); past mimo_taylor_ok the phases are stored
//    and the channel kernels evaluate the sum per sample (exact_jakes);
//  * fD != 0, f32: the same expansion to second order, A + B d + C d^2
//    (truncation ~1e-10 at 3 km/h, far below float32), computed in float64,
//    while mimo_taylor_ok_prec; past it the per-sample sum, rounded to float.
// AWGN links: SFBC h = exp(j t pi/2) (core/ofdm_core.py:476-487); spatial
// h ~ CN(0,1) (core/channel.py:473-480), injected or Philox.
// coef layout: [B][rx][tx][path][n_cs][mimo_ncf<R>()]; phases [B][rx][tx][path][16].
template <class R>
__global__ __launch_bounds__(MWG) void k_fading_mimo(int B, int num_rx, int num_tx, int n_paths, int n_cs, int mode,
                                                     int rayleigh, const R* __restrict__ gains, double fD, double fs,
                                                     int sym_len, const uint64_t* __restrict__ fid, uint64_t seed,
                                                     const R* __restrict__ inj_ph, int64_t inj_ph_stride,
                                                     const R* __restrict__ inj_h, int64_t inj_h_stride,
                                                     cx<R>* __restrict__ coef, R* __restrict__ phases) {
  constexpr bool F64 = sizeof(R) == 8;
  const int per = num_rx * num_tx * n_paths;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * per) return;
  const int b = i / per, rem = i - b * per, link = rem / n_paths, p = rem - link * n_paths;
  const int rx = link / num_tx, tx = link - rx * num_tx;
  constexpr int NCF = mimo_ncf<R>();
  cx<R>* out = coef + (size_t)i * n_cs * NCF;
  if (!rayleigh) {
    double hr = 0.0, hi = 0.0;
    if (mode == MIMO_SFBC) {
      if (tx == 0) { hr = 1.0; hi = 0.0; }
      else {   // np.exp(1j * (t * np.pi / 2))
        const double a = ((double)tx * 3.141592653589793) / 2.0;
        hr = cos(a); hi = sin(a);
      }
    } else if (inj_h) {
      const R* hh = inj_h + (size_t)b * inj_h_stride + (size_t)link * 2;
      hr = hh[0]; hi = hh[1];
    } else {
      const u32x4 r = rng4(seed, fid[b], RNG_STREAM_MIMO_LINK + (uint32_t)link, 0x7FFFFFFFu);
      if constexpr (F64) {
        const double2 z = gauss2<double>(r.x, r.y);
        hr = 0.7071067811865475 * z.x; hi = 0.7071067811865475 * z.y;   // normal(0, 1/np.sqrt(2))
      } else {
        const float2 z = box_muller(r.x, r.y);
        hr = z.x * 0.7071067811865476; hi = z.y * 0.7071067811865476;
      }
    }
    out[0] = mkc((R)hr, (R)hi);
    for (int k = 1; k < NCF; ++k) out[k] = mkc((R)0, (R)0);
    return;
  }
  double ph[16];
  for (int mm = 0; mm < 16; ++mm) {
    if (inj_ph) {
      ph[mm] = inj_ph[(size_t)b * inj_ph_stride + (size_t)rem * 16 + mm];
    } else {
      const u32x4 r = rng4(seed, fid[b], RNG_STREAM_MIMO_FADE + (uint32_t)rem, (uint32_t)(mm >> 2));
      const int q = mm & 3;
      const uint32_t u = q == 0 ? r.x : q == 1 ? r.y : q == 2 ? r.z : r.w;
      ph[mm] = F64 ? 6.283185307179586 * (((double)u + 0.5) * 2.3283064365386962890625e-10)
                   : 6.283185307179586 * ((u >> 8) * (1.0 / 16777216.0));
    }
  }
  if constexpr (F64) {
    const double gn = gains[p];
    if (n_cs > 1) {   // the Taylor sets (fD != 0)
      jakes_symbol_sets<R>(ph, gn, fD, fs, sym_len, n_cs, out);
      return;
    }
    const double k = sqrt(2.0 / 16.0);
    double sr = 0.0, si = 0.0;
    for (int mm = 0; mm < 16; ++mm) {
      double sv, cv;
      sincos(ph[mm], &sv, &cv);
      sr += cv;
      si += sv;
    }
    out[0] = make_double2(gn * (sr * k), gn * (si * k));
    for (int kk = 1; kk < NCF; ++kk) out[kk] = make_double2(0.0, 0.0);
    if (phases)
      for (int mm = 0; mm < 16; ++mm) phases[(size_t)i * 16 + mm] = ph[mm];
    return;
  } else {
    jakes_symbol_sets<R>(ph, (double)gains[p], fD, fs, sym_len, n_cs, out);
    if (phases)   // past the quadratic's bound: the per-sample sum (exact_jakes)
      for (int mm = 0; mm < 16; ++mm) phases[(size_t)i * 16 + mm] = (R)ph[mm];
  }
}

template <class R>
int launch_fading_mimo(hipStream_t s, const Grid& g, const MimoGrid& m, int B, int rayleigh, int n_paths,
                       const R* gains, double fD, double fs, const uint64_t* fid, uint64_t seed, const R* inj_ph,
                       int64_t inj_ph_stride, const R* inj_h, int64_t inj_h_stride, cx<R>* coef, R* phases) {
  const int np = rayleigh ? n_paths : 1;
  const int n = B * m.num_rx * m.num_tx * np;
  if (rayleigh && m.exact_jakes && !phases) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_fading_mimo<R>, dim3((n + MWG - 1) / MWG), dim3(MWG), 0, s, B, m.num_rx, m.num_tx, np, m.n_cs,
                     m.mode, rayleigh, gains, fD, fs, g.N + g.cp, fid, seed, inj_ph, inj_ph_stride, inj_h,
                     inj_h_stride, coef, (rayleigh && m.exact_jakes) ? phases : nullptr);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Channel.  y_rx[n] = sum_tx y_link[n], y_link[n] = sum_p h_{rx,tx,p}(n)
// x_tx[n - d_p] (stream-level delay with a zero prefix, Q4) + (transmit_mimo
// Rayleigh only) the link noise of each link's own 100 dB ChannelSimulator
// (core/ofdm_core.py:490-503: sigma^2 = P_link / 1e10, still drawn).  Power
// partials -> noise per RX: SFBC (P_rx / num_tx) / SNR (:524-534), spatial
// P_rx / SNR (channel.py:457-467).  The f64 instances sum each link from zero
// and then add it to the RX stream, as the reference accumulates signals_rx.

// exact jakes_fading at sample n of a link path (f64): g (sqrt(2/16) sum_m
// exp(j (w_m t + phi_m))), t = n / fs, in the reference's operation order
__device__ __noinline__ double2 jakes_exact(const MimoGrid& m, const double (&ph)[16], double gn, int n, double fs) {
  const double t = (double)n / fs;
  double sr = 0.0, si = 0.0;
#pragma unroll
  for (int mm = 0; mm < 16; ++mm) {
    double sv, cv;
    sincos(m.jw[mm] * t + ph[mm], &sv, &cv);
    sr += cv;
    si += sv;
  }
  const double k = 0.3535533905932738;   // np.sqrt(2 / 16)
  return make_double2(gn * (sr * k), gn * (si * k));
}
// the exact value in the chain's type (float: rounded once)
template <class R>
__device__ __forceinline__ cx<R> jakes_exact_r(const MimoGrid& m, const double (&ph)[16], double gn, int n,
                                               double fs) {
  const double2 h = jakes_exact(m, ph, gn, n, fs);
  return mkc((R)h.x, (R)h.y);
}

// one link's output at a single sample n (link_sample: coefficient triples of
// n's symbol; EX: f64 exact Jakes from the phases ph)
template <class R, bool EX>
__device__ __forceinline__ cx<R> link_value(int n, const cx<R>* __restrict__ cf, int n_cs, int np, int sym_len,
                                            const int32_t* __restrict__ delays, const cx<R>* __restrict__ xf,
                                            const R* __restrict__ ph, const R* __restrict__ gains, const MimoGrid& m,
                                            double fs) {
  using V = cx<R>;
  V acc = mkc((R)0, (R)0);
  if constexpr (EX) {
    for (int p = 0; p < np; ++p) {
      const int src = n - (delays ? delays[p] : 0);
      if (src < 0) continue;
      double phv[16];
#pragma unroll
      for (int mm = 0; mm < 16; ++mm) phv[mm] = ph[p * 16 + mm];
      acc = cadd(acc, cmul(jakes_exact_r<R>(m, phv, (double)gains[p], n, fs), xf[src]));
    }
    return acc;
  }
  constexpr int NCF = mimo_ncf<R>();
  const int sidx = n_cs > 1 ? n / sym_len : 0;
  const R d = n_cs > 1 ? (R)(n - sidx * sym_len) - (R)0.5 * (R)(sym_len - 1) : (R)0;
  for (int p = 0; p < np; ++p) {
    const int src = n - (delays ? delays[p] : 0);
    if (src < 0) continue;
    const V* c = cf + ((size_t)p * n_cs + sidx) * NCF;
    V h = c[0];
    if (n_cs > 1) {   // sum_k c_k d^k (Horner)
      h = c[NCF - 1];
#pragma unroll
      for (int k = NCF - 2; k >= 0; --k) h = mkc(h.x * d + c[k].x, h.y * d + c[k].y);
    }
    acc = cadd(acc, cmul(h, xf[src]));
  }
  return acc;
}

// One block per (frame, OFDM symbol); each thread owns J samples of the
// symbol, n_j = base + tid + j*MWG, so every (link, path) coefficient triple
// (wave-uniform: one symbol) is loaded once per thread and the J delayed loads
// of a path are issued back to back.
template <int J>
struct SymSpan {
  int n[J];
  float d[J];
  bool ok[J];
  __device__ __forceinline__ SymSpan(int base, int nbeg, int nend, float dc, bool fading) {
#pragma unroll
    for (int j = 0; j < J; ++j) {
      n[j] = base + (int)threadIdx.x + j * MWG;
      ok[j] = n[j] < nend;
      d[j] = fading ? (float)(n[j] - nbeg) - dc : 0.f;
    }
  }
};

constexpr int MC_MAXRX = 8;   // receive antennas per launch
constexpr int MC_RXG = 4;     // receive antennas accumulated per pass over the transmit streams
// (kernel template G: MC_RXG, or 2 when the plan has at most 2 receive antennas --
// half the accumulator registers; LTE_CHM_G2 = 0 turns that off for A/B)
#ifndef LTE_CHM_G2
#define LTE_CHM_G2 1
#endif
#ifndef LTE_CHM_G2_WAVES   // f64 G = 2 channel kernel: minimum waves per SIMD asked of the register allocator
#define LTE_CHM_G2_WAVES 5
#endif

// acc[q][j] += sum_p h_{rx q, tx, p}(n_j) x_tx[n_j - delay_p] for the nq <=
// MC_RXG receive antennas of a group and one transmit stream: each delayed TX
// sample is loaded once for all of them (the group's links share the TX
// stream).  cs: the first link's coefficients at this symbol (stride n_cs *
// mimo_ncf per path, cs_q per receive antenna); EX: f64 exact Jakes from the
// phases ph (ph_q per receive antenna) -- a separate instance, so that its
// sincos calls do not set the register budget of the coefficient path.
// acc[q][j] += sum_p h_{rx q, tx, p}(n_j) x_tx[n_j - delay_p] for the nq <=
// MC_RXG receive antennas of a group and one transmit stream: each delayed TX
// sample is loaded once for all of them (the group's links share the TX
// stream).  cs: the first link's coefficients at this symbol (stride n_cs *
// mimo_ncf per path, cs_q per receive antenna); EX: f64 exact Jakes from the
// phases ph (ph_q per receive antenna) -- a separate instance, so that its
// sincos calls do not set the register budget of the coefficient path.
template <class R, int J, bool EX, int G>
__device__ __forceinline__ void links_accumulate(cx<R> (&acc)[G][J], int nq, const SymSpan<J>& sp,
                                                 const cx<R>* __restrict__ cs, size_t cs_q, int n_cs, int np,
                                                 const int32_t* __restrict__ delays, const cx<R>* __restrict__ xf,
                                                 const R* __restrict__ ph, size_t ph_q, const R* __restrict__ gains,
                                                 const MimoGrid& m, double fs) {
  using V = cx<R>;
  constexpr int NCF = mimo_ncf<R>();
  for (int p = 0; p < np; ++p) {
    const int dl = delays ? delays[p] : 0;
    V xs[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int src = sp.n[j] - dl;
      xs[j] = (sp.ok[j] && src >= 0) ? xf[src] : mkc((R)0, (R)0);
    }
#pragma unroll
    for (int q = 0; q < G; ++q) {
      if (q >= nq) break;
      if constexpr (EX) {
          double phv[16];
#pragma unroll
        for (int mm = 0; mm < 16; ++mm) phv[mm] = ph[q * ph_q + p * 16 + mm];
        const double gn = gains[p];
#pragma unroll
        for (int j = 0; j < J; ++j)
          if (sp.ok[j] && sp.n[j] >= dl)
            acc[q][j] = cadd(acc[q][j], cmul(jakes_exact_r<R>(m, phv, gn, sp.n[j], fs), xs[j]));
      } else {
        const V* c = cs + q * cs_q + (size_t)p * n_cs * NCF;
        if (n_cs > 1) {   // sum_k c_k d^k (Horner; f32: A + B d + C d^2)
          V cc[NCF];
#pragma unroll
          for (int k = 0; k < NCF; ++k) cc[k] = c[k];
#pragma unroll
          for (int j = 0; j < J; ++j) {
            const R dj = (R)sp.d[j];
            V h = cc[NCF - 1];
#pragma unroll
            for (int k = NCF - 2; k >= 0; --k) h = mkc(h.x * dj + cc[k].x, h.y * dj + cc[k].y);
            acc[q][j] = cadd(acc[q][j], cmul(h, xs[j]));
          }
        } else {
          const V c0 = c[0];
#pragma unroll
          for (int j = 0; j < J; ++j) acc[q][j] = cadd(acc[q][j], cmul(c0, xs[j]));
        }
      }
    }
  }
}

// The link noise of a SymSpan's J samples (Philox path; the same values as
// link_noise_at per sample).  With an even base, lane pair (2k, 2k+1) holds
// sample pairs (n, n + 1) that share one Philox draw (counter n >> 1): the
// even lane draws for sample j, the odd lane for sample j + 1, and each hands
// its partner the other half through one xor-1 shuffle -- one draw per lane
// per two samples instead of one per sample.
template <class R, int J>
__device__ __forceinline__ void link_noise_span(cx<R> (&acc)[J], const SymSpan<J>& sp, R sg, uint64_t seed,
                                                uint64_t frame, int link, bool even_base) {
  if (!even_base) {
#pragma unroll
    for (int j = 0; j < J; ++j)
      if (sp.ok[j]) acc[j] = link_noise_at<R>(sp.n[j], sg, nullptr, 0, seed, frame, link, acc[j]);
    return;
  }
  const bool odd = threadIdx.x & 1;
#pragma unroll
  for (int j = 0; j < J; j += 2) {
    const int jo = j + 1 < J ? j + 1 : j;
    const u32x4 r = rng4(seed, frame, RNG_STREAM_MIMO_LINK + (uint32_t)link, (uint32_t)(sp.n[odd ? jo : j] >> 1));
    const uint32_t g0 = __shfl_xor(odd ? r.x : r.z, 1), g1 = __shfl_xor(odd ? r.y : r.w, 1);
    // even lane: sample j (even n) its own (x, y), sample jo (even n) the partner's (x, y);
    // odd lane: sample j (odd n) the partner's (z, w), sample jo (odd n) its own (z, w)
    const cx<R> zj = gauss2<R>(odd ? g0 : r.x, odd ? g1 : r.y);
    const cx<R> zo = gauss2<R>(odd ? r.z : g0, odd ? r.w : g1);
    if (sp.ok[j]) acc[j] = mkc(acc[j].x + sg * zj.x, acc[j].y + sg * zj.y);
    if (jo != j && sp.ok[jo]) acc[jo] = mkc(acc[jo].x + sg * zo.x, acc[jo].y + sg * zo.y);
  }
}

// pass 1 (transmit_mimo Rayleigh): per-link power partials of the faded signal,
// one block per (frame, OFDM symbol, TX stream), the receive antennas in groups
template <class R, int J, bool EX, int G>
__global__ __launch_bounds__(MWG) void k_link_power(int L, int num_rx, int num_tx, int np, int n_cs, int sym_len,
                                                    const int32_t* __restrict__ delays, const cx<R>* __restrict__ coef,
                                                    const R* __restrict__ phases, const R* __restrict__ gains,
                                                    double fs, MimoGrid m, const cx<R>* __restrict__ x,
                                                    R* __restrict__ part, int nblk) {
  using V = cx<R>;
  constexpr int NCF = mimo_ncf<R>();
  __shared__ R red[MWG / 64];
  const int blk = blockIdx.x % nblk, b = blockIdx.x / nblk;
  const int tx = blockIdx.y;
  const int sidx = n_cs > 1 ? blk : 0;
  const int nbeg = blk * sym_len, nend = min(nbeg + sym_len, L);
  const float dc = 0.5f * (float)(sym_len - 1);
  const V* xf = x + ((size_t)b * num_tx + tx) * L;
  const size_t cs_q = (size_t)num_tx * np * n_cs * NCF, ph_q = (size_t)num_tx * np * 16;
  for (int rg = 0; rg < num_rx; rg += G) {
    const int nq = min(G, num_rx - rg);
    const size_t lk0 = ((size_t)b * num_rx + rg) * num_tx + tx;
    const V* cs = coef + lk0 * np * n_cs * NCF + (size_t)sidx * NCF;
    const R* ph = EX ? phases + lk0 * np * 16 : nullptr;
    R pw[G];
#pragma unroll
    for (int q = 0; q < G; ++q) pw[q] = (R)0;
    for (int base = nbeg; base < nend; base += J * MWG) {
      const SymSpan<J> sp(base, nbeg, nend, dc, n_cs > 1);
      V acc[G][J];
#pragma unroll
      for (int q = 0; q < G; ++q)
#pragma unroll
        for (int j = 0; j < J; ++j) acc[q][j] = mkc((R)0, (R)0);
      links_accumulate<R, J, EX, G>(acc, nq, sp, cs, cs_q, n_cs, np, delays, xf, ph, ph_q, gains, m, fs);
#pragma unroll
      for (int q = 0; q < G; ++q)
#pragma unroll
        for (int j = 0; j < J; ++j)
          if (sp.ok[j]) pw[q] += acc[q][j].x * acc[q][j].x + acc[q][j].y * acc[q][j].y;
    }
#pragma unroll
    for (int q = 0; q < G; ++q) {
      if (q >= nq) break;
      const R t = block_sum(pw[q], red);
      if (threadIdx.x == 0) part[(lk0 + (size_t)q * num_tx) * nblk + blk] = t;
      __syncthreads();
    }
  }
}

// sigma of the link noise: sqrt((mean|y0|^2 / 10^(100/10)) / 2)
template <class R>
__global__ void k_link_sigma(int n_links_total, const R* __restrict__ part, int nblk, int L, R* __restrict__ sigma) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_links_total) return;
  double acc = 0.0;
  for (int k = 0; k < nblk; ++k) acc += part[(size_t)i * nblk + k];
  sigma[i] = (R)sqrt(((acc / L) / 1e10) / 2.0);
}

// ---------------------------------------------------------------------------
// Config 4's TX and its static-tap Rayleigh links in one pass (SFBC 2 x NRX,
// transmit_mimo core/ofdm_core.py:434-543 with every link a 100 dB
// ChannelSimulator, :490-503).  One slot (the block's 256 threads) per frame
// walks the frame's OFDM symbols.  Per symbol both TX grids (the Alamouti pairs
// of SFBCAlamouti.encode + SFBCResourceMapper, core/sfbc_alamouti.py:45-78,
// 213-256, each thread's pairs for both TX at once; each TX's CRS subset) are
// built and IFFT'd in two LDS buffers, the last pass applying NumPy's sqrt(N)/N
// output scale, so the buffers hold x_t.  Then for every sample n of the
// CP-extended symbol and every RX r: y0_rt = sum_p c_rtp x_t[n - d_p] (each
// link from zero, in path order) and y0_r = y0_r0 + y0_r1 (the links summed in
// TX order, as mimo_oracle.transmit_mimo sums them); the delayed samples that
// reach into the previous symbol come from its last TL samples of each TX,
// kept in LDS -- the frame walks its symbols in order, so no fix-up pass is
// needed.  Each link's power sum_n |y0_rt|^2 accumulates over the frame (the
// link noise's standard deviation, k_link_sigma).  y0 goes to HBM once; the
// TX streams x never do.  k_link_noise_pairs then adds the link noise and forms
// the RX power partials.  Static taps only (n_cs = 1), N = 2048 (two 32 KB
// grids and the staged streams: two slots per CU, each of TPB threads).
constexpr int SFX_TL = 32;   // largest max_delay (samples) the kept tails cover
// timing probes for A/B builds only (wrong results): bit 0 skips the Alamouti
// mapping, bit 1 the IFFTs, bit 2 the link taps (y = x_0 + x_1 at n)
#ifndef LTE_SFX_PROBE
#define LTE_SFX_PROBE 0
#endif
// TPB = 256: one thread per radix-8 butterfly of each grid, both grids in one
// dual-buffer sweep; TPB = 512: each half of the block transforms one grid
// (the same operations per element), twice the waves per slot.
// MRG (the merged link noise, launch_npow_sfbc_merged): the two link
// accumulators of each RX hold instead sum_t |y0_rt|^2 (the links' powers
// summed) and |y0_r|^2 (the RX stream's power) -- the same register count.
template <class R, int CODED, int BPS, int NRX, int NP = 0, int TPB = MWG, int NC = 2048, bool MRG = false>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(TPB / 128, TPB / 128))) void k_ofdm_txch_sfbc(Grid g, MimoGrid m, const uint32_t* __restrict__ pw, int PW,
                                                          const uint32_t* __restrict__ enc, int enc_words,
                                                          const int32_t* __restrict__ tx_map, TxLinkPower<R> lp,
                                                          cx<R>* __restrict__ y, int B, int stage_enc) {
  using V = cx<R>;
  constexpr int N = NC, T = N >> 3, NTX = 2, NCF = mimo_ncf<R>();
  static_assert(TPB == T || TPB == 2 * T, "one slot per block");
  __shared__ R red[TPB / 64];
  // LDS: grids / x_t at [t * N, (t + 1) * N), then [NTX][SFX_TL] the previous
  // symbol's last TL samples of each x_t (one array, so that a delayed sample's
  // address is one index expression), the frame's taps [NRX][NTX][PM], then
  // the staged coded streams
  V* sm = mimo_lds<V>();
  constexpr int TB0 = 2 * N;
  const int tid0 = threadIdx.x, b = blockIdx.x;
  const bool active = b < B;   // (grid = B blocks: always; kept for the shared FFT helper)
  // NP > 0: the path count at compile time (only NP taps formed; a runtime
  // count computed all TXCH_MAXP unrolled taps under selects)
  constexpr int PM = NP ? NP : TXCH_MAXP;
  const int S = N + g.cp, TL = lp.max_delay, np = NP ? NP : lp.n_paths;
  const uint32_t* fb = pw + (size_t)b * PW;
  const uint32_t* fe = enc + (size_t)b * enc_words;
  // the frame's static taps c_rtp (coef [B][num_rx][num_tx][np][NCF], n_cs = 1)
  // copied to LDS once; each symbol's sample loop reads them from there
  V* ct = sm + TB0 + NTX * SFX_TL;
  for (int i = tid0; i < NRX * NTX * PM; i += TPB) {
    const int p = i % PM, rt = i / PM;
    ct[i] = p < np ? lp.coef[(((size_t)b * NRX * NTX + rt) * np + p) * NCF] : mkc((R)0, (R)0);
  }
  if (CODED && stage_enc) {
    uint32_t* es = reinterpret_cast<uint32_t*>(ct + NRX * NTX * PM);
    for (int i = tid0; i < enc_words; i += TPB) es[i] = fe[i];
    fe = es;
  }
  for (int i = tid0; i < NTX * SFX_TL; i += TPB) sm[TB0 + i] = mkc((R)0, (R)0);   // zero prefix of the stream
  int dl[PM];
#pragma unroll
  for (int p = 0; p < PM; ++p) dl[p] = p < np ? lp.delays[p] : 0;
  R pwr[NRX][NTX];
#pragma unroll
  for (int r = 0; r < NRX; ++r)
#pragma unroll
    for (int t = 0; t < NTX; ++t) pwr[r][t] = (R)0;
  const R sc = tx_scale<R>(N);
  constexpr int SFP = 4 * T / TPB;   // Alamouti pairs per thread per symbol (n_dsc / 2 <= SFP TPB)
  // (each pair's grid positions held in registers across the symbols instead of
  // re-read per symbol: 28.06 / 27.77 vs 27.53 / 27.52 ms, the 4 registers spill)
  for (int l = 0; l < g.n_sym; ++l) {
    int tid = tid0;   // opaque per symbol: the FFT's addressing is not hoisted into registers
    asm volatile("" : "+v"(tid));
    for (int k = tid; k < 2 * N; k += TPB) sm[k] = mkc((R)0, (R)0);
    __syncthreads();   // (first symbol: also the staged streams and the zeroed tails)
    if (!(LTE_SFX_PROBE & 1)) {
      const int64_t q0 = (int64_t)l * m.res;
#pragma unroll
      for (int k = 0; k < SFP; ++k) {   // TX0 [s0, -conj(s1)], TX1 [s1, conj(s0)]
        const int j = 2 * (tid + k * TPB);
        if (j >= m.n_dsc) break;
        int c0, c1;
        if constexpr (CODED) {   // (m.res even: q0 + j even)
          qam_code_pair<BPS>(q0 + j, fe, tx_map, c0, c1);
        } else {
          c0 = qam_code<CODED, BPS>(q0 + j, fb, fe, tx_map);
          c1 = qam_code<CODED, BPS>(q0 + j + 1, fb, fe, tx_map);
        }
        const V s0 = qam_of<R, BPS>(c0);
        const V s1 = qam_of<R, BPS>(c1);
        const int k0 = g.data_idx[j];
        sm[k0] = s0;
        sm[N + k0] = s1;
        if (j + 1 < m.n_dsc) {
          const int k1 = g.data_idx[j + 1];
          sm[k1] = mkc(-s1.x, s1.y);
          sm[N + k1] = mkc(s0.x, -s0.y);
        }
      }
#pragma unroll
      for (int t = 0; t < NTX; ++t) {
        const V* pv = MGT<R>::pval(m) + t * m.maxP;
        for (int p = tid; p < m.np_tx[t]; p += TPB) sm[t * N + m.ppos[t * m.maxP + p]] = pv[p];
      }
    }
    __syncthreads();
    // x_t = ifft(G_t) sqrt(N), both grids in one sweep (ends with a barrier)
    if (!(LTE_SFX_PROBE & 2)) {
      if constexpr (TPB == T) fft2_lds<true, NC, true>(sm, sm + N, GridT<R>::tw(g), tid, active, sc);
      else fft_lds<true, NC, true, true>(sm + (tid >= T ? N : 0), N, 0, GridT<R>::tw(g), tid & (T - 1), active, sc);
    }
    // the taps into VGPRs from LDS for the sample loop only: as wave-uniform
    // values the compiler would keep them in SGPRs and spill them to VGPR
    // lanes inside the loop; held across the FFTs they would crowd them
    V c[NRX][NTX][PM];
#pragma unroll
    for (int r = 0; r < NRX; ++r)
#pragma unroll
      for (int t = 0; t < NTX; ++t)
#pragma unroll
        for (int p = 0; p < PM; ++p) {
          c[r][t][p] = ct[(r * NTX + t) * PM + p];
          asm volatile("" : "+v"(c[r][t][p].x), "+v"(c[r][t][p].y));
        }
    V* yl = y + (size_t)b * NRX * g.L + (size_t)l * S;
    for (int n = tid; n < S; n += TPB) {
      if (LTE_SFX_PROBE & 4) {
        const V a = cadd(sm[(n - g.cp) & (N - 1)], sm[N + ((n - g.cp) & (N - 1))]);
#pragma unroll
        for (int r = 0; r < NRX; ++r) {
          yl[(size_t)r * g.L + n] = a;
          pwr[r][0] += a.x * a.x;
        }
        continue;
      }
      V xs[NTX][PM];   // x_t at CP-extended position n - d_p (negative: the previous symbol's tail)
      if (n >= g.cp + TL) {   // every tap inside the symbol's own samples, past the CP: grid index n - cp - d_p
        const int i0 = n - g.cp;
#pragma unroll
        for (int p = 0; p < PM; ++p)
          if (p < np) {
#pragma unroll
            for (int t = 0; t < NTX; ++t) xs[t][p] = sm[t * N + i0 - dl[p]];
          }
      } else {
#pragma unroll
        for (int p = 0; p < PM; ++p)
          if (p < np) {
            const int i = n - dl[p];
#pragma unroll
            for (int t = 0; t < NTX; ++t)
              xs[t][p] = sm[i >= 0 ? t * N + ((i - g.cp) & (N - 1)) : TB0 + t * SFX_TL + TL + i];
          }
      }
#pragma unroll
      for (int r = 0; r < NRX; ++r) {
        V a[NTX];
#pragma unroll
        for (int t = 0; t < NTX; ++t) {
          a[t] = mkc((R)0, (R)0);
#pragma unroll
          for (int p = 0; p < PM; ++p)
            if (p < np) a[t] = cadd(a[t], cmul(c[r][t][p], xs[t][p]));
          if (!MRG) pwr[r][t] += a[t].x * a[t].x + a[t].y * a[t].y;
        }
        const V yr = cadd(a[0], a[1]);
        yl[(size_t)r * g.L + n] = yr;
        if constexpr (MRG) {
          pwr[r][0] += (a[0].x * a[0].x + a[0].y * a[0].y) + (a[1].x * a[1].x + a[1].y * a[1].y);
          pwr[r][1] += yr.x * yr.x + yr.y * yr.y;
        }
      }
    }
    __syncthreads();   // every read of the old tails and of the grids done
    for (int i = tid; i < NTX * TL; i += TPB) {
      const int t = i / TL, k = i - t * TL;
      sm[TB0 + t * SFX_TL + k] = sm[t * N + ((S - TL + k - g.cp) & (N - 1))];
    }
    __syncthreads();   // the tails are in place before the next symbol zeroes the grids
  }
#pragma unroll
  for (int r = 0; r < NRX; ++r)
#pragma unroll
    for (int t = 0; t < NTX; ++t) {
      const R v = block_sum(pwr[r][t], red);
      // one partial per link (nblk 1); MRG: per RX the links' sum, then the RX stream's
      if (threadIdx.x == 0) lp.part[((size_t)b * NRX + r) * NTX + t] = v;
      __syncthreads();
    }
}

// launch_npow_sfbc_merged (lte_internal.h): npow_eff per (frame, RX), in the
// order oracle/mimo_oracle.transmit_mimo (merged) forms it
template <class R>
__global__ void k_npow_sfbc_merged(int n, int num_rx, const R* __restrict__ part, int L,
                                   const R* __restrict__ snr_lin, double num_tx, R* __restrict__ npow) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double s2 = (((double)part[2 * i] / L) / 1e10) / 2.0;   // sum_t s_rt^2
  const double P = (double)part[2 * i + 1] / L + 2.0 * s2;
  const double na = (P / num_tx) / (double)snr_lin[i / num_rx];
  npow[i] = (R)(2.0 * s2 + na);
}

template <class R>
int launch_npow_sfbc_merged(hipStream_t s, int B, int num_rx, int num_tx, const R* link_part, int L, const R* snr_lin,
                            R* npow) {
  if (num_tx != 2) return (int)hipErrorInvalidValue;   // k_ofdm_txch_sfbc<.., MRG>'s two partials per RX
  const int n = B * num_rx;
  hipLaunchKernelGGL(k_npow_sfbc_merged<R>, dim3((n + 255) / 256), dim3(256), 0, s, n, num_rx, link_part, L, snr_lin,
                     (double)num_tx, npow);
  return (int)hipGetLastError();
}

// transmit_mimo's link noise on the Philox path after k_ofdm_txch_sfbc: y0_r +
// the RX's combined 100 dB link noise (rx_link_sigma, one draw per sample on
// link (r, 0)'s stream, the values and the order k_channel_tay adds them in),
// written back, and the RX power of the result for the (P / num_tx) / SNR rule
// (core/ofdm_core.py:524-534).  One block per (frame, RX antenna) walking the
// whole frame in sample pairs: lane k of a round takes pair p = (2p, 2p+1), the
// two halves of one Philox draw (counter p, as link_noise_at), so there is one
// draw per two samples with no lane exchange.  Loads for U pairs are issued
// before the first draw.  One RX power partial per (frame, RX): nblk = 1 for
// k_npow_mimo.  (Measured against drawing the link noise a second time in the
// receiver instead of writing it here: the receiver is VALU-bound and lost
// more, 12.5 ms, than the write saved, 9.3 ms per 65 536 frames; against the
// per-(frame, symbol) form with J-sample spans and lane-pair shuffles: 32.1 vs
// 32.9 ms.)
// LT: the float64 Box-Muller tables read from an LDS copy (bm_tables_lds)
// instead of the __constant__ arrays.
template <class R, int U, bool LT>
__global__ __launch_bounds__(MWG) void k_link_noise_pairs(int L, int num_rx, int num_tx, cx<R>* __restrict__ y,
                                                          const R* __restrict__ link_sigma,
                                                          const uint64_t* __restrict__ fid, uint64_t seed,
                                                          R* __restrict__ pow_part) {
  using V = cx<R>;
  __shared__ R red[MWG / 64];
  constexpr bool TL = LT && sizeof(R) == 8;
  __shared__ double2 bmt[TL ? BM_LDS_BYTES / 16 : 1];
  BmTabL tbl{};
  if constexpr (TL) {
    tbl = bm_tables_lds(bmt, threadIdx.x, MWG);
    __syncthreads();
  }
  const int br = blockIdx.x, r = br % num_rx;
  const size_t b = (size_t)(br / num_rx);
  const R sg = rx_link_sigma(link_sigma, (size_t)br * num_tx, num_tx);
  const uint64_t frame = fid[b];
  const uint32_t stream = RNG_STREAM_MIMO_LINK + (uint32_t)(r * num_tx);
  V* yb = y + (size_t)br * L;
  const int npair = (L + 1) >> 1;
  R pw = (R)0;
  for (int p0 = threadIdx.x; p0 < npair; p0 += U * MWG) {
    V va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = p0 + u * MWG, n = 2 * p;
      va[u] = p < npair ? yb[n] : mkc((R)0, (R)0);
      vb[u] = n + 1 < L ? yb[n + 1] : mkc((R)0, (R)0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = p0 + u * MWG, n = 2 * p;
      if (p >= npair) break;
      const u32x4 q = rng4(seed, frame, stream, (uint32_t)p);
      const V z0 = TL ? gauss2t<R>(q.x, q.y, tbl) : gauss2<R>(q.x, q.y);
      const V a = mkc(va[u].x + sg * z0.x, va[u].y + sg * z0.y);
      yb[n] = a;
      pw += a.x * a.x + a.y * a.y;
      if (n + 1 < L) {
        const V z1 = TL ? gauss2t<R>(q.z, q.w, tbl) : gauss2<R>(q.z, q.w);
        const V c = mkc(vb[u].x + sg * z1.x, vb[u].y + sg * z1.y);
        yb[n + 1] = c;
        pw += c.x * c.x + c.y * c.y;
      }
    }
  }
  const R t = block_sum(pw, red);
  if (threadIdx.x == 0) pow_part[br] = t;
}

template <class R>
bool sfbc_txch_supported(const Grid& g, const MimoGrid& m, int n_paths, int max_delay) {
  return m.mode == MIMO_SFBC && m.num_tx == 2 && (m.num_rx == 1 || m.num_rx == 2) && g.N == 2048 && m.n_cs == 1 &&
         (m.res & 1) == 0 &&
         !m.exact_jakes && n_paths >= 1 && n_paths <= TXCH_MAXP && max_delay >= 0 && max_delay <= SFX_TL &&
         max_delay <= g.cp && m.n_dsc <= 2 * 4 * (g.N >> 3) && (g.bps == 2 || g.bps == 4 || g.bps == 6);
}

#ifndef LTE_SFX_TPB   // threads per frame slot of k_ofdm_txch_sfbc (256 or 512)
#define LTE_SFX_TPB 512
#endif
template <class R>
int launch_ofdm_txch_sfbc(hipStream_t s, const Grid& g, const MimoGrid& m, int coded, const uint32_t* pw, int PW,
                          const uint32_t* enc, int enc_words, const int32_t* tx_map, const TxLinkPower<R>& lp,
                          cx<R>* y, int B) {
  if (!sfbc_txch_supported<R>(g, m, lp.n_paths, lp.max_delay) || !lp.part) return (int)hipErrorInvalidValue;
  const size_t enc_shm = (size_t)enc_words * sizeof(uint32_t);
  const int stage_enc = coded && enc_shm <= 32768;
  const size_t shm = (2 * (size_t)g.N + 2 * SFX_TL + (size_t)m.num_rx * 2 * TXCH_MAXP) * sizeof(cx<R>) +
                     (stage_enc ? enc_shm : 0);
#define LTE_SFX(C_, B_, NR_)                                                                                          \
  do {                                                                                                                \
    const int tpb = lp.n_paths == 4 ? LTE_SFX_TPB : MWG;                                                              \
    auto k = lp.n_paths == 4 ? (lp.merged ? k_ofdm_txch_sfbc<R, C_, B_, NR_, 4, LTE_SFX_TPB, 2048, true>          \
                                          : k_ofdm_txch_sfbc<R, C_, B_, NR_, 4, LTE_SFX_TPB>)                         \
                             : (lp.merged ? k_ofdm_txch_sfbc<R, C_, B_, NR_, 0, MWG, 2048, true>                     \
                                          : k_ofdm_txch_sfbc<R, C_, B_, NR_, 0>);                                    \
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);                  \
    hipLaunchKernelGGL(k, dim3(B), dim3(tpb), shm, s, g, m, pw, PW, enc, enc_words, tx_map, lp, y, B, stage_enc);     \
  } while (0)
#define LTE_SFX_NR(C_, B_) do { if (m.num_rx == 1) LTE_SFX(C_, B_, 1); else LTE_SFX(C_, B_, 2); } while (0)
#define LTE_SFX_B(C_) \
  do { if (g.bps == 2) LTE_SFX_NR(C_, 2); else if (g.bps == 4) LTE_SFX_NR(C_, 4); else LTE_SFX_NR(C_, 6); } while (0)
  if (coded) LTE_SFX_B(1); else LTE_SFX_B(0);
#undef LTE_SFX_B
#undef LTE_SFX_NR
#undef LTE_SFX
  return (int)hipGetLastError();
}

template <class R>
int launch_link_noise_add(hipStream_t s, const Grid& g, const MimoGrid& m, int B, const R* link_part, R* link_sigma,
                          cx<R>* y, const uint64_t* fid, uint64_t seed, R* pow_part, int* pow_nblk) {
  if (m.num_rx < 1 || m.num_rx > 2) return (int)hipErrorInvalidValue;
  const int nl = B * m.num_rx * m.num_tx;   // one partial per link (k_ofdm_txch_sfbc)
  hipLaunchKernelGGL(k_link_sigma<R>, dim3((nl + 255) / 256), dim3(256), 0, s, nl, link_part, 1, g.L, link_sigma);
  *pow_nblk = 1;
#ifndef LTE_LN_U   // sample pairs per lane in flight in k_link_noise_pairs (A/B)
#define LTE_LN_U 8
#endif
  hipLaunchKernelGGL((k_link_noise_pairs<R, LTE_LN_U, LTE_BM_LDS != 0>), dim3(B * m.num_rx), dim3(MWG), 0, s, g.L, m.num_rx,
                     m.num_tx, y, link_sigma, fid, seed, pow_part);
  return (int)hipGetLastError();
}

// One block per (frame, OFDM symbol): the symbol index -- hence every link
// path's fading coefficients -- is uniform over the block, so they are scalar
// loads; the sample offset d from the symbol centre is per lane.  All RX of
// the frame per block: each delayed TX sample is loaded once for a group of
// MC_RXG receive antennas (links_accumulate), one power reduction per RX.
template <class R, int J, bool EX, int G>
__global__ __launch_bounds__(MWG, (G == 2 && sizeof(R) == 8 && !EX) ? LTE_CHM_G2_WAVES : 1) void k_channel_mimo(int L, int num_rx, int num_tx, int np, int n_cs, int sym_len,
                                                      const int32_t* __restrict__ delays,
                                                      const cx<R>* __restrict__ coef, const R* __restrict__ phases,
                                                      const R* __restrict__ gains, double fs, MimoGrid m,
                                                      const cx<R>* __restrict__ x, cx<R>* __restrict__ y,
                                                      const R* __restrict__ link_sigma,
                                                      const uint64_t* __restrict__ fid, uint64_t seed,
                                                      const R* __restrict__ inj_lz, int64_t inj_lz_stride,
                                                      R* __restrict__ pow_part, int nblk) {
  using V = cx<R>;
  constexpr bool F64 = sizeof(R) == 8;
  constexpr int NCF = mimo_ncf<R>();
  __shared__ R red[MWG / 64];
  const int blk = blockIdx.x % nblk, b = blockIdx.x / nblk;   // blk = OFDM symbol (block of sym_len samples)
  const int sidx = n_cs > 1 ? blk : 0;
  const int nbeg = blk * sym_len, nend = min(nbeg + sym_len, L);
  const float dc = 0.5f * (float)(sym_len - 1);
  const size_t nl = (size_t)num_rx * num_tx;
  const size_t cs_q = (size_t)num_tx * np * n_cs * NCF, ph_q = (size_t)num_tx * np * 16;
  for (int rg = 0; rg < num_rx; rg += G) {
    const int nq = min(G, num_rx - rg);
    R pw[G];
#pragma unroll
    for (int q = 0; q < G; ++q) pw[q] = (R)0;
    for (int base = nbeg; base < nend; base += J * MWG) {
      const SymSpan<J> sp(base, nbeg, nend, dc, n_cs > 1);
      V v[G][J];
#pragma unroll
      for (int q = 0; q < G; ++q)
#pragma unroll
        for (int j = 0; j < J; ++j) v[q][j] = mkc((R)0, (R)0);
      for (int tx = 0; tx < num_tx; ++tx) {
        const V* xf = x + ((size_t)b * num_tx + tx) * L;
        const size_t lk0 = (size_t)b * nl + (size_t)rg * num_tx + tx;
        const V* cs = coef + lk0 * np * n_cs * NCF + (size_t)sidx * NCF;
        const R* ph = EX ? phases + lk0 * np * 16 : nullptr;
        // f64: each link's y from zero, then signals_rx += y_link (the
        // reference's order); f32 accumulates into the RX sums directly
        V vl[G][J];
        V (&acc)[G][J] = F64 ? vl : v;
        if constexpr (F64) {
#pragma unroll
          for (int q = 0; q < G; ++q)
#pragma unroll
            for (int j = 0; j < J; ++j) vl[q][j] = mkc((R)0, (R)0);
        }
        links_accumulate<R, J, EX, G>(acc, nq, sp, cs, cs_q, n_cs, np, delays, xf, ph, ph_q, gains, m, fs);
#pragma unroll
        for (int q = 0; q < G; ++q) {
          if (q >= nq) break;
          const int link = (rg + q) * num_tx + tx;
          if (link_sigma && inj_lz) {
            const R sg = link_sigma[(size_t)b * nl + link];
            const R* zf = inj_lz + (size_t)b * inj_lz_stride + (size_t)link * 2 * L;
#pragma unroll
            for (int j = 0; j < J; ++j)
              if (sp.ok[j]) acc[q][j] = link_noise_at<R>(sp.n[j], sg, zf, L, seed, fid[b], link, acc[q][j]);
          }
          if constexpr (F64) {
#pragma unroll
            for (int j = 0; j < J; ++j) v[q][j] = cadd(v[q][j], vl[q][j]);
          }
        }
      }
      if (link_sigma && !inj_lz) {   // Philox: one draw per RX sample (rx_link_sigma)
#pragma unroll
        for (int q = 0; q < G; ++q) {
          if (q >= nq) break;
          const int r = rg + q;
          const R sr = rx_link_sigma(link_sigma, (size_t)b * nl + (size_t)r * num_tx, num_tx);
          link_noise_span<R, J>(v[q], sp, sr, seed, fid[b], r * num_tx, (nbeg & 1) == 0);
        }
      }
#pragma unroll
      for (int q = 0; q < G; ++q) {
        if (q >= nq) break;
        const int r = rg + q;
#pragma unroll
        for (int j = 0; j < J; ++j)
          if (sp.ok[j]) {
            y[((size_t)b * num_rx + r) * L + sp.n[j]] = v[q][j];
            pw[q] += v[q][j].x * v[q][j].x + v[q][j].y * v[q][j].y;
          }
      }
    }
#pragma unroll
    for (int q = 0; q < G; ++q) {
      if (q >= nq) break;
      const R t = block_sum(pw[q], red);
      if (threadIdx.x == 0) pow_part[((size_t)b * num_rx + rg + q) * nblk + blk] = t;
      __syncthreads();
    }
  }
}

// The coefficient-path channel (per-symbol Taylor sets, TAY, or one static
// tap set per link path): the same sums as k_channel_mimo without the exact
// Jakes instance, laid out for the f64 FMA pipe.
//  * The block's (link, path) coefficient sets of its OFDM symbol are staged
//    in LDS once (nl np K complex values) and read back as wave-uniform
//    broadcasts: scalar registers cannot hold them for four receive
//    antennas without spilling inside the FMA loop.
//  * Each delayed TX sample is loaded once for the G receive antennas of a
//    group (G divides num_rx: no runtime antenna guard in the unrolled loops,
//    which made the compiler hold every antenna's coefficients at once);
//    every receive stream accumulates h x with two FMAs per component.
//  * Link noise (LN: its own instance) and the power partials as in
//    k_channel_mimo; the f64 streams
//    add each (link, path) product straight into the RX sum (the reference
//    sums each link first -- a different rounding order only, within the
//    1e-12 stream bars).
#ifndef LTE_CHT_SB   // 1: a scheduling barrier after each antenna (its coefficient reads not hoisted)
#define LTE_CHT_SB 0
#endif
#if LTE_CHT_SB
#define LTE_CHT_SCHED_BARRIER() __builtin_amdgcn_sched_barrier(0)
#else
#define LTE_CHT_SCHED_BARRIER() ((void)0)
#endif
#ifndef LTE_CHT_WAVES   // k_channel_tay: minimum waves per SIMD asked of the register allocator
#define LTE_CHT_WAVES 4
#endif
template <class R, int J, int G, bool TAY, bool LN, bool EC = false>
__global__ __launch_bounds__(MWG, LTE_CHT_WAVES) void k_channel_tay(int L, int num_rx, int num_tx, int np, int n_cs, int sym_len,
                                                     const int32_t* __restrict__ delays,
                                                     const cx<R>* __restrict__ coef, const cx<R>* __restrict__ x,
                                                     cx<R>* __restrict__ y, const R* __restrict__ link_sigma,
                                                     const uint64_t* __restrict__ fid, uint64_t seed,
                                                     const R* __restrict__ inj_lz, int64_t inj_lz_stride,
                                                     R* __restrict__ pow_part, int nblk) {
  using V = cx<R>;
  constexpr int NCF = mimo_ncf<R>();   // stored terms per (path, symbol)
  constexpr int K = TAY ? (EC ? NCF - 1 : NCF) : 1;   // terms evaluated
  __shared__ R red[MWG / 64];
  V* cl = mimo_lds<V>();               // [num_rx][num_tx][np][K]
  const int blk = blockIdx.x % nblk, b = blockIdx.x / nblk;
  const int sidx = TAY ? blk : 0;
  const int nbeg = blk * sym_len, nend = min(nbeg + sym_len, L);
  const float dc = 0.5f * (float)(sym_len - 1);
  const int nl = num_rx * num_tx;
  {
    const size_t ps = (size_t)n_cs * NCF;
    const V* cb = coef + (size_t)b * nl * np * ps + (size_t)sidx * NCF;
    // EC: the degree-5 set economised to degree 4 over the symbol, d in
    // [-D, D]: c5 d^5 = c5 D^5 (T5(u) + 20 u^3 - 5 u) / 16, u = d / D, keeps
    // c3 + (5/4) D^2 c5 and c1 - (5/16) D^4 c5 and drops c5 D^5 T5(u) / 16
    // (|T5| <= 1; the host enables it while that is below 1e-17 of the gain)
    const R D = (R)0.5 * (R)(sym_len - 1);
    for (int i = threadIdx.x; i < nl * np * K; i += MWG) {
      const int lp = i / K, k = i - lp * K;
      V c = cb[(size_t)lp * ps + k];
      if constexpr (EC) {
        if (k == 1 || k == 3) {
          const V c5 = cb[(size_t)lp * ps + 5];
          const R f = k == 1 ? -(R)0.3125 * (D * D) * (D * D) : (R)1.25 * (D * D);
          c = mkc(c.x + f * c5.x, c.y + f * c5.y);
        }
      }
      cl[i] = c;
    }
  }
  __syncthreads();
  for (int rg = 0; rg < num_rx; rg += G) {
    R pw[G];
#pragma unroll
    for (int q = 0; q < G; ++q) pw[q] = (R)0;
    for (int base = nbeg; base < nend; base += J * MWG) {
      const SymSpan<J> sp(base, nbeg, nend, dc, TAY);
      V v[G][J];
#pragma unroll
      for (int q = 0; q < G; ++q)
#pragma unroll
        for (int j = 0; j < J; ++j) v[q][j] = mkc((R)0, (R)0);
#pragma unroll 1
      for (int tx = 0; tx < num_tx; ++tx) {
        const V* xf = x + ((size_t)b * num_tx + tx) * L;
#pragma unroll 1
        for (int p = 0; p < np; ++p) {
          const int dl = delays ? delays[p] : 0;
          V xs[J];
#pragma unroll
          for (int j = 0; j < J; ++j) {
            const int src = sp.n[j] - dl;
            xs[j] = (sp.ok[j] && src >= 0) ? xf[src] : mkc((R)0, (R)0);
          }
#pragma unroll
          for (int q = 0; q < G; ++q) {
            const V* c = cl + (((rg + q) * num_tx + tx) * np + p) * K;
            // Horner over the J samples together, one coefficient live at a time
            V h[J];
            const V ct = c[K - 1];
#pragma unroll
            for (int j = 0; j < J; ++j) h[j] = ct;
#pragma unroll
            for (int k = K - 2; k >= 0; --k) {
              const V ck = c[k];
#pragma unroll
              for (int j = 0; j < J; ++j) {
                const R dj = (R)sp.d[j];
                h[j] = mkc(h[j].x * dj + ck.x, h[j].y * dj + ck.y);
              }
            }
#pragma unroll
            for (int j = 0; j < J; ++j) {
              v[q][j].x = fma(h[j].x, xs[j].x, fma(-h[j].y, xs[j].y, v[q][j].x));
              v[q][j].y = fma(h[j].x, xs[j].y, fma(h[j].y, xs[j].x, v[q][j].y));
            }
            LTE_CHT_SCHED_BARRIER();
          }
        }
        if (LN && inj_lz) {   // the reference's own draws: per link
#pragma unroll
          for (int q = 0; q < G; ++q) {
            const int link = (rg + q) * num_tx + tx;
            const R sg = link_sigma[(size_t)b * nl + link];
            const R* zf = inj_lz + (size_t)b * inj_lz_stride + (size_t)link * 2 * L;
#pragma unroll
            for (int j = 0; j < J; ++j)
              if (sp.ok[j]) v[q][j] = link_noise_at<R>(sp.n[j], sg, zf, L, seed, fid[b], link, v[q][j]);
          }
        }
      }
      if (LN && !inj_lz) {   // Philox: one draw per RX sample (rx_link_sigma)
#pragma unroll
        for (int q = 0; q < G; ++q) {
          const int r = rg + q;
          const R sr = rx_link_sigma(link_sigma, (size_t)b * nl + (size_t)r * num_tx, num_tx);
          link_noise_span<R, J>(v[q], sp, sr, seed, fid[b], r * num_tx, (nbeg & 1) == 0);
        }
      }
#pragma unroll
      for (int q = 0; q < G; ++q) {
        const int r = rg + q;
#pragma unroll
        for (int j = 0; j < J; ++j)
          if (sp.ok[j]) {
            y[((size_t)b * num_rx + r) * L + sp.n[j]] = v[q][j];
            pw[q] += v[q][j].x * v[q][j].x + v[q][j].y * v[q][j].y;
          }
      }
    }
#pragma unroll
    for (int q = 0; q < G; ++q) {
      const R t = block_sum(pw[q], red);
      if (threadIdx.x == 0) pow_part[((size_t)b * num_rx + rg + q) * nblk + blk] = t;
      __syncthreads();
    }
  }
}

// LDS bytes of k_channel_tay's coefficient stage
template <class R>
size_t channel_tay_lds(const MimoGrid& m, int np) {
  return (size_t)m.num_rx * m.num_tx * np * (m.n_cs > 1 ? mimo_ncf<R>() : 1) * sizeof(cx<R>);
}

// k_channel_tay's degree-4 economisation holds the per-sample error under
// 1e-17 of the path gain: |c5| <= sqrt(2/16) 16 W^5 / 5! for the fastest
// sinusoid W = max |w_m| / fs, so |c5| D^5 / 16 <= 5.657 (W D)^5 / 1920 with D
// the half symbol (3 km/h at 20 MHz: W D = 1.245e-3, 2.5 % inside the bound)
static bool channel_tay_econ(const MimoGrid& m, int sym_len, double fs) {
  if (const char* e = std::getenv("LTE_CHT_ECON"))
    if (std::atoi(e) == 0) return false;
  double w = 0.0;
  for (int k = 0; k < 16; ++k) w = std::max(w, std::fabs(m.jw[k]));
  const double x = w / fs * 0.5 * (sym_len - 1);
  return 5.657 * x * x * x * x * x / 1920.0 <= 1e-17;
}

int mimo_channel_nblk(int L, int sym_len) { return (L + sym_len - 1) / sym_len; }

// k_channel_tay's launch: G receive antennas per group (a divisor of num_rx);
// J (samples per thread per pass, 1..3) the one covering a symbol with the
// fewest idle lanes (20 MHz: 3 -> 2304 lanes for 2192 samples)
template <class R>
static void launch_channel_tay(hipStream_t s, int B, int nch, int L, const MimoGrid& m, int np, int sym_len,
                               double fs, const int32_t* delays, const cx<R>* coef, const cx<R>* x, cx<R>* y,
                               const R* link_sigma, const uint64_t* fid, uint64_t seed, const R* inj_lz,
                               int64_t inj_lz_stride, R* pow_part) {
  int J = 1;
  long best = -1;
  for (int j = 1; j <= 3; ++j) {
    const long cover = (long)((sym_len + j * MWG - 1) / (j * MWG)) * j * MWG;
    if (best < 0 || cover <= best) { best = cover; J = j; }
  }
  const bool tay = m.n_cs > 1;
  const size_t shm = channel_tay_lds<R>(m, np);
  // receive antennas per group: a divisor of num_rx, at most 4
  int G = m.num_rx <= 4 ? m.num_rx : m.num_rx % 4 == 0 ? 4 : m.num_rx % 3 == 0 ? 3 : m.num_rx % 2 == 0 ? 2 : 1;
  // A/B overrides (LTE_CHT_J in 1..3; LTE_CHT_G a divisor of num_rx up to 4)
  if (const char* e = std::getenv("LTE_CHT_J")) J = std::min(3, std::max(1, std::atoi(e)));
  if (const char* e = std::getenv("LTE_CHT_G")) {
    const int g = std::atoi(e);
    if (g >= 1 && g <= 4 && m.num_rx % g == 0) G = g;
  }
#define LTE_CHT(J_, G_, T_, E_)                                                                                      \
  do {                                                                                                               \
    if (link_sigma)                                                                                                  \
      hipLaunchKernelGGL((k_channel_tay<R, J_, G_, T_, true, E_>), dim3(nch * B), dim3(MWG), shm, s, L, m.num_rx,   \
                         m.num_tx, np, m.n_cs, sym_len, delays, coef, x, y, link_sigma, fid, seed, inj_lz,          \
                         inj_lz_stride, pow_part, nch);                                                              \
    else                                                                                                             \
      hipLaunchKernelGGL((k_channel_tay<R, J_, G_, T_, false, E_>), dim3(nch * B), dim3(MWG), shm, s, L, m.num_rx,  \
                         m.num_tx, np, m.n_cs, sym_len, delays, coef, x, y, nullptr, fid, seed, nullptr, 0,         \
                         pow_part, nch);                                                                             \
  } while (0)
#define LTE_CHT_G(J_, T_, E_)                                                                                        \
  do {                                                                                                               \
    switch (G) {                                                                                                     \
      case 4: LTE_CHT(J_, 4, T_, E_); break;                                                                         \
      case 3: LTE_CHT(J_, 3, T_, E_); break;                                                                         \
      case 2: LTE_CHT(J_, 2, T_, E_); break;                                                                         \
      default: LTE_CHT(J_, 1, T_, E_); break;                                                                        \
    }                                                                                                                \
  } while (0)
#define LTE_CHT_J(T_)                                                                                                \
  do {                                                                                                               \
    if (J == 1) LTE_CHT_G(1, T_, false); else if (J == 2) LTE_CHT_G(2, T_, false); else LTE_CHT_G(3, T_, false);     \
  } while (0)
  if constexpr (sizeof(R) == 8) {   // the economised degree-4 sets (f64 Taylor path, J = 3)
    if (tay && J == 3 && channel_tay_econ(m, sym_len, fs)) {
      LTE_CHT_G(3, true, true);
      return;
    }
  }
  if (tay) LTE_CHT_J(true); else LTE_CHT_J(false);
#undef LTE_CHT_J
#undef LTE_CHT_G
#undef LTE_CHT
}

template <class R>
int launch_channel_mimo(hipStream_t s, const Grid& g, const MimoGrid& m, int B, int n_paths, const int32_t* delays,
                        const cx<R>* coef, const R* phases, const R* gains, double fs, const cx<R>* x, cx<R>* y,
                        int link_noise, const uint64_t* fid, uint64_t seed, const R* inj_lz, int64_t inj_lz_stride,
                        R* link_part, R* link_sigma, R* pow_part, int nblk, int link_part_done) {
  const int sym_len = g.N + g.cp;
  if (m.num_rx > MC_MAXRX) return (int)hipErrorInvalidValue;
  const int nch = mimo_channel_nblk(g.L, sym_len);
  if (nch > nblk) return (int)hipErrorInvalidValue;   // partial buffers are sized for nblk blocks
  const R* ph = m.exact_jakes ? phases : nullptr;
  if (m.exact_jakes && (!phases || !gains)) return (int)hipErrorInvalidValue;
  // samples per thread per pass: the smallest instantiated J covering one
  // symbol, at most 2 (f64) / 3 (f32) -- larger symbols loop.  The RX-group
  // accumulators take 4 MC_RXG J VGPRs per component pair (f64: v and the
  // per-link vl); measured J = 1 / 2 / 3 / 5 at 20 MHz, f64 config 5 channel
  // 6.0 / 6.0 / 6.8 / 11.2 ms and 3 km/h 26.9 / 19.3 / 27.1 / 41.9 ms per 8192
  // frames; f32 4.2 / 3.1 / 3.0 / 3.2 and 15.9 / 11.0 / 9.6 / 11.3 ms
  // the coefficient path runs k_channel_tay (LTE_CHM_TAY=0: k_channel_mimo, for A/B)
  const char* tye = std::getenv("LTE_CHM_TAY");
  const bool tay_on = !(tye && std::atoi(tye) == 0);
  const int jn = (sym_len + MWG - 1) / MWG;
  const int jmax = sizeof(R) == 8 ? 2 : 3;
  const int J = jn <= 1 ? 1 : jn <= 2 || jmax == 2 ? 2 : 3;
#define LTE_CHM_EX(J_, EX_)                                                                                         \
  do {                                                                                                             \
    if (LTE_CHM_G2 && m.num_rx <= 2) LTE_CHM_EXG(J_, EX_, 2);                                                     \
    else LTE_CHM_EXG(J_, EX_, MC_RXG);                                                                             \
  } while (0)
#define LTE_CHM_EXG(J_, EX_, G_)                                                                                    \
  do {                                                                                                             \
    if (link_noise) {                                                                                              \
      if (!link_part_done)   /* else k_ofdm_tx_mimo + k_link_power_fix wrote the partials */                      \
        hipLaunchKernelGGL((k_link_power<R, J_, EX_, G_>), dim3(nch * B, m.num_tx), dim3(MWG), 0, s, g.L,         \
                           m.num_rx, m.num_tx, n_paths, m.n_cs, sym_len, delays, coef, ph, gains, fs, m, x,        \
                           link_part, nch);                                                                        \
      const int nl = B * m.num_rx * m.num_tx;                                                                      \
      hipLaunchKernelGGL(k_link_sigma<R>, dim3((nl + 255) / 256), dim3(256), 0, s, nl, link_part, nch, g.L,        \
                         link_sigma);                                                                              \
    }                                                                                                              \
    if (!(EX_) && tay_on && channel_tay_lds<R>(m, n_paths) <= 32768)                                               \
      launch_channel_tay<R>(s, B, nch, g.L, m, n_paths, sym_len, fs, delays, coef, x, y,                           \
                            link_noise ? link_sigma : nullptr, fid, seed, inj_lz, inj_lz_stride, pow_part);        \
    else                                                                                                           \
      hipLaunchKernelGGL((k_channel_mimo<R, J_, EX_, G_>), dim3(nch * B), dim3(MWG), 0, s, g.L, m.num_rx,         \
                         m.num_tx, n_paths, m.n_cs, sym_len, delays, coef, ph, gains, fs, m, x, y,                 \
                         link_noise ? link_sigma : nullptr, fid, seed, inj_lz, inj_lz_stride, pow_part, nch);      \
  } while (0)
#define LTE_CHM(J_)                                                                                                 \
  do {                                                                                                             \
    if (m.exact_jakes) { LTE_CHM_EX(J_, true); break; }                                                            \
    LTE_CHM_EX(J_, false);                                                                                         \
  } while (0)
  switch (J) {
    case 1: LTE_CHM(1); break;
    case 2: LTE_CHM(2); break;
    default: LTE_CHM(3); break;
  }
#undef LTE_CHM
#undef LTE_CHM_EX
#undef LTE_CHM_EXG
  return (int)hipGetLastError();
}

// Per-link statistics for the reported channel matrix (transmit_mimo,
// core/ofdm_core.py:505-516): mean|x|^2, mean|y_link|^2, mean(y_link conj(x)),
// y_link with its link noise when link_sigma is set (the reference's y; on the
// Philox path each link its own draw, while the RX streams take one combined
// draw per RX, rx_link_sigma).
template <class R, bool EX>
__global__ __launch_bounds__(MWG) void k_link_stats_part(int L, int num_rx, int num_tx, int np, int n_cs, int sym_len,
                                                         const int32_t* __restrict__ delays,
                                                         const cx<R>* __restrict__ coef, const R* __restrict__ phases,
                                                         const R* __restrict__ gains, double fs, MimoGrid m,
                                                         const cx<R>* __restrict__ x,
                                                         const R* __restrict__ link_sigma,
                                                         const uint64_t* __restrict__ fid, uint64_t seed,
                                                         const R* __restrict__ inj_lz, int64_t inj_lz_stride,
                                                         R* __restrict__ part, int nblk) {
  using V = cx<R>;
  __shared__ R red[MWG / 64];
  const int blk = blockIdx.x % nblk, b = blockIdx.x / nblk;
  const int link = blockIdx.y, rx = link / num_tx, tx = link - rx * num_tx;
  const int n = blk * MWG + threadIdx.x;
  const size_t lk = ((size_t)b * num_rx + rx) * num_tx + tx;
  R v[4] = {(R)0, (R)0, (R)0, (R)0};
  if (n < L) {
    const V* xf = x + ((size_t)b * num_tx + tx) * L;
    const V* cf = coef + lk * np * n_cs * mimo_ncf<R>();
    V yv = link_value<R, EX>(n, cf, n_cs, np, sym_len, delays, xf, EX ? phases + lk * np * 16 : nullptr, gains, m, fs);
    if (link_sigma) {
      const R* zf = inj_lz ? inj_lz + (size_t)b * inj_lz_stride + (size_t)link * 2 * L : nullptr;
      yv = link_noise_at<R>(n, link_sigma[lk], zf, L, seed, fid[b], link, yv);
    }
    const V xv = xf[n];
    v[0] = xv.x * xv.x + xv.y * xv.y;
    v[1] = yv.x * yv.x + yv.y * yv.y;
    const V c = cmulc(yv, xv);
    v[2] = c.x;
    v[3] = c.y;
  }
  for (int q = 0; q < 4; ++q) {
    const R t = block_sum(v[q], red);
    if (threadIdx.x == 0) part[((((size_t)b * num_rx * num_tx) + link) * 4 + q) * nblk + blk] = t;
    __syncthreads();
  }
}

template <class R>
__global__ void k_link_stats_fin(int n, const R* __restrict__ part, int nblk, int L, R* __restrict__ stats) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double acc = 0.0;
  for (int k = 0; k < nblk; ++k) acc += part[(size_t)i * nblk + k];
  stats[i] = (R)(acc / L);
}

template <class R>
int launch_link_stats(hipStream_t s, const Grid& g, const MimoGrid& m, int B, int n_paths, const int32_t* delays,
                      const cx<R>* coef, const R* phases, const R* gains, double fs, const cx<R>* x,
                      const R* link_sigma, const uint64_t* fid, uint64_t seed, const R* inj_lz, int64_t inj_lz_stride,
                      R* part, int nblk, R* stats) {
  if (nblk < (g.L + MWG - 1) / MWG) return (int)hipErrorInvalidValue;
  if (m.exact_jakes && !phases) return (int)hipErrorInvalidValue;
#define LTE_LSP(EX_)                                                                                                 \
  hipLaunchKernelGGL((k_link_stats_part<R, EX_>), dim3(nblk * B, m.num_rx * m.num_tx), dim3(MWG), 0, s, g.L,         \
                     m.num_rx, m.num_tx, n_paths, m.n_cs, g.N + g.cp, delays, coef, phases, gains, fs, m, x,          \
                     link_sigma, fid, seed, inj_lz, inj_lz_stride, part, nblk)
  if (m.exact_jakes) LTE_LSP(true);
  else LTE_LSP(false);
#undef LTE_LSP
  const int n = B * m.num_rx * m.num_tx * 4;
  hipLaunchKernelGGL(k_link_stats_fin<R>, dim3((n + 255) / 256), dim3(256), 0, s, n, part, nblk, g.L, stats);
  return (int)hipGetLastError();
}

template <class R>
__global__ void k_npow_mimo(int n, const R* __restrict__ pow_part, int nblk, int L, const R* __restrict__ snr_lin,
                            int num_rx, double div, R* __restrict__ npow) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double acc = 0.0;
  for (int k = 0; k < nblk; ++k) acc += pow_part[(size_t)i * nblk + k];
  npow[i] = (R)(((acc / L) / div) / (double)snr_lin[i / num_rx]);
}

template <class R>
int launch_npow_mimo(hipStream_t s, int B, int num_rx, const R* pow_part, int nblk, int L, const R* snr_lin,
                     double div, R* npow) {
  const int n = B * num_rx;
  hipLaunchKernelGGL(k_npow_mimo<R>, dim3((n + 255) / 256), dim3(256), 0, s, n, pow_part, nblk, L, snr_lin, num_rx,
                     div, npow);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// RX FFT + MIMO CRS estimation.  One slot per (frame, rx) walking the frame's
// OFDM symbols (per symbol the same work as one slot per (frame, rx, symbol)
// did; the walk amortises the slot's setup and the LDS copy of the Box-Muller
// tables over 14 symbols): noise + CP removal + FFT/sqrt(N)
// (demodulate_and_estimate_mimo, core/mimo_channel_estimator_periodic.py:
// 236-273); the n_dsc data SCs go to Y[b][l][rx][n_dsc].  On estimation
// symbols (SFBC: first of each 14-symbol group, :195-234; spatial: every
// symbol, core/ofdm_core.py:2752) LS at each TX's pilot subset + linear
// interpolation with edge hold (:108-185 + lte_receiver.py:98-133:
// np.linspace, k (delta / gap) + start) at the data SCs ->
// H[b][rx][e][tx][n_dsc].
// TX t's estimate at data SC j from its LS pilot estimates hpt (np_t of them):
// linear interpolation with edge hold (mimo_channel_estimator_periodic.py:
// 108-185), the one expression k_rx_fft_mimo and k_rx_sfbc share
template <class R>
__device__ __forceinline__ cx<R> mimo_interp(const Grid& g, const MimoGrid& m, const cx<R>* hpt, int npt,
                                             const R* __restrict__ pig, int t, int j) {
  const int sidx = m.pseg[t * m.n_dsc + j];
  if (sidx < 0) return hpt[0];
  if (sidx >= npt - 1) return hpt[npt - 1];
  const cx<R> v0 = hpt[sidx], v1 = hpt[sidx + 1];
  const R fk = (R)(g.data_idx[j] - m.ppos[t * m.maxP + sidx]);
  const R ig = pig[t * m.maxP + sidx];
  return mkc(fk * ((v1.x - v0.x) * ig) + v0.x, fk * ((v1.y - v0.y) * ig) + v0.y);
}

// mimo_interp at a looked-up point (segment sidx, offset fk, 1 / gap ig):
// the same expression
template <class R>
__device__ __forceinline__ cx<R> mimo_interp_at(const cx<R>* hpt, int npt, int sidx, R fk, R ig) {
  if (sidx < 0) return hpt[0];
  if (sidx >= npt - 1) return hpt[npt - 1];
  const cx<R> v0 = hpt[sidx], v1 = hpt[sidx + 1];
  return mkc(fk * ((v1.x - v0.x) * ig) + v0.x, fk * ((v1.y - v0.y) * ig) + v0.y);
}

template <class R, int NC = 0, bool HPO = false>
__global__ __launch_bounds__(MWG) void k_rx_fft_mimo(Grid g, MimoGrid m, int B, const cx<R>* __restrict__ y,
                                                     const R* __restrict__ npow, const uint64_t* __restrict__ fid,
                                                     uint64_t seed, const R* __restrict__ inj_z, int64_t inj_stride,
                                                     cx<R>* __restrict__ Y, cx<R>* __restrict__ H) {
  using V = cx<R>;
  V* sm = mimo_lds<V>();
  const int N = NC ? NC : g.N, T = N >> 3, spw = MWG / T;
  const int slot = threadIdx.x / T, tid0 = threadIdx.x % T;
  const int gs = blockIdx.x * spw + slot;
  const int b = gs / m.num_rx, rx = gs - b * m.num_rx;
  const bool active = slot < spw && b < B;
  V* buf = sm + slot * N;
  V* hp = sm + spw * N + slot * (m.num_tx * m.maxP);
  LTE_BM_LDS_DECL(R);
  const auto bmt = bm_stage<R>(lte_bmt);
  const R sc = rx_scale<R>(N);
  const V* pv = MGT<R>::pval(m);
  const size_t br = (size_t)(active ? b : 0) * m.num_rx + rx;
  const R sigma = active ? sqrt(npow[br] * (R)0.5) : (R)0;
  const uint64_t fr = active ? fid[b] : 0ull;
  const R* zf = (inj_z && active) ? inj_z + (size_t)b * inj_stride + (size_t)rx * 2 * g.L : nullptr;
  const V* yf = y + br * g.L;
  __syncthreads();
  for (int l = 0; l < g.n_sym; ++l) {
    int tid = tid0;   // opaque per symbol (see k_rx_frame)
    asm volatile("" : "+v"(tid));
    if (active) load_symbol_noisy2<true>(buf, yf, N, g.cp, l, sigma, seed, fr, rx, zf, g.L, tid, T, bmt);
    __syncthreads();
    fft_lds<false, NC, false, (NC > 0), true>(buf, N, g.log2N, GridT<R>::tw(g), tid, active);
    const int e = m.mode == MIMO_SFBC ? l / 14 : l;
    const bool est = m.mode == MIMO_SFBC ? (l % 14) == 0 : true;
    if (active && est) {
      for (int t = 0; t < m.num_tx; ++t)
        for (int p = tid; p < m.np_tx[t]; p += T) {
          const V h = cdiv(cscale(buf[m.ppos[t * m.maxP + p]], sc), pv[t * m.maxP + p]);
          if constexpr (HPO) H[((br * m.n_est + e) * m.num_tx + t) * m.maxP + p] = h;
          else hp[t * m.maxP + p] = h;
        }
    }
    if constexpr (!HPO) __syncthreads();
    if (active) {
      V* Yo = Y + (((size_t)b * g.n_sym + l) * m.num_rx + rx) * m.n_dsc;
      for (int j = tid; j < m.n_dsc; j += T) Yo[j] = cscale(buf[g.data_idx[j]], sc);
      if (!HPO && est) {
        const R* pig = MGT<R>::pig(m);
        for (int t = 0; t < m.num_tx; ++t) {
          const V* hpt = hp + t * m.maxP;
          const int npt = m.np_tx[t];
          V* Ho = H + (((br * m.n_est + e) * m.num_tx + t)) * m.n_dsc;
          for (int j = tid; j < m.n_dsc; j += T) Ho[j] = mimo_interp<R>(g, m, hpt, npt, pig, t, j);
        }
      }
    }
    __syncthreads();   // buf and hp are rewritten by the next symbol
  }
}

template <class R>
int launch_rx_fft_mimo(hipStream_t s, const Grid& g, const MimoGrid& m, int B, const cx<R>* y, const R* npow,
                       const uint64_t* fid, uint64_t seed, const R* inj_z, int64_t inj_stride, cx<R>* Y, cx<R>* H,
                       int h_pilots) {
  if constexpr (sizeof(R) == 8)
    if (rx_fft_mimo_w_supported(g, m, 1, h_pilots) && mimo_rx_wave_enabled())
      return launch_rx_fft_mimo_w(s, g, m, B, y, npow, fid, seed, inj_z, inj_stride, Y, H);
  const int spw = MWG / (g.N >> 3);
  const int64_t total = (int64_t)B * m.num_rx;
  if (total > 0x7FFFFFFF - spw) return (int)hipErrorInvalidValue;
  const int blocks = (int)((total + spw - 1) / spw);
  const size_t shm = spw * (g.N + m.num_tx * m.maxP) * sizeof(cx<R>);
  if (g.N == 2048 && h_pilots)
    hipLaunchKernelGGL((k_rx_fft_mimo<R, 2048, true>), dim3(blocks), dim3(MWG), shm, s, g, m, B, y, npow, fid, seed,
                       inj_z, inj_stride, Y, H);
  else if (h_pilots)
    hipLaunchKernelGGL((k_rx_fft_mimo<R, 0, true>), dim3(blocks), dim3(MWG), shm, s, g, m, B, y, npow, fid, seed, inj_z,
                       inj_stride, Y, H);
  else if (g.N == 2048)   // 20 MHz: compile-time N (unrolled passes, twiddle recurrence)
    hipLaunchKernelGGL((k_rx_fft_mimo<R, 2048>), dim3(blocks), dim3(MWG), shm, s, g, m, B, y, npow, fid, seed, inj_z,
                       inj_stride, Y, H);
  else
    hipLaunchKernelGGL((k_rx_fft_mimo<R>), dim3(blocks), dim3(MWG), shm, s, g, m, B, y, npow, fid, seed, inj_z,
                       inj_stride, Y, H);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// SFBCAlamouti.decode's combiner for one subcarrier pair (core/sfbc_alamouti.py:
// 139-161), shared by the chain's detector (k_det_sfbc) and the stage entry
// (lte_sfbc_decode_host64): s0 = conj(h0k) rk + h1k1 conj(rk1), s1 = conj(h1k)
// rk - h0k1 conj(rk1), norm = |avg(h0)|**2 + |avg(h1)|**2 + reg.  f64 in the
// reference's NumPy complex128 scalar semantics: |z| = hypot, s / norm = s *
// (1 / norm) (NumPy's complex / real division multiplies by the reciprocal of
// its real denominator).  d0 = s0 / norm, d1 = s1 / norm; returns norm.
template <class R>
__device__ __forceinline__ R sfbc_combine(cx<R> rk, cx<R> rk1, cx<R> h0k, cx<R> h1k, cx<R> h0k1, cx<R> h1k1, R reg,
                                          cx<R>& d0, cx<R>& d1) {
  using V = cx<R>;
  const V rc = mkc(rk1.x, -rk1.y);
  const V s0 = cadd(cmulc(rk, h0k), cmul(h1k1, rc));      // conj(h0k) rk + h1k1 conj(rk1)
  const V s1 = csub(cmulc(rk, h1k), cmul(h0k1, rc));      // conj(h1k) rk - h0k1 conj(rk1)
  const V a0 = mkc((R)0.5 * (h0k.x + h0k1.x), (R)0.5 * (h0k.y + h0k1.y));
  const V a1 = mkc((R)0.5 * (h1k.x + h1k1.x), (R)0.5 * (h1k.y + h1k1.y));
  if constexpr (sizeof(R) == 8) {
    const double n0 = hypot(a0.x, a0.y), n1 = hypot(a1.x, a1.y);
    const double nrm = (n0 * n0 + n1 * n1) + reg;
    const double rn = 1.0 / nrm;
    d0 = make_double2(s0.x * rn, s0.y * rn);
    d1 = make_double2(s1.x * rn, s1.y * rn);
    return nrm;
  } else {
    const float nrm = (a0.x * a0.x + a0.y * a0.y) + (a1.x * a1.x + a1.y * a1.y) + reg;
    d0 = make_float2(s0.x / nrm, s0.y / nrm);
    d1 = make_float2(s1.x / nrm, s1.y / nrm);
    return nrm;
  }
}

// ---------------------------------------------------------------------------
// SFBC detection.  One thread per (frame, OFDM symbol, SC pair).
// SFBCAlamouti.decode (core/sfbc_alamouti.py:80-163) per RX with that RX's
// slot estimate, averaged over RX (core/ofdm_core.py:2204, Q17).  f64 in the
// reference's NumPy complex128 scalar semantics (sfbc_combine, reg = 1e-10),
// the RX mean (sum_r d_r) * (1 / num_rx).  Uncoded:
// nearest-point hard bits vs the payload (bit errors).  Coded (config 4):
// max-log LLRs (core/ofdm_core.py:791-923) with the per-RE noise variance of
// the combined estimate, sigma^2 / R^2 * sum_r 1 / clip(norm_r, 1e-6, 1e6),
// floored at sigma^2 / 4 as in the SISO rule (ofdm_core.py:1224-1243) -- the
// reference has no coded SFBC chain; DESIGN.md documents this composition.
template <class R, int CODED, int BPS>
__global__ __launch_bounds__(MWG) void k_det_sfbc(Grid g, MimoGrid m, int B, const cx<R>* __restrict__ Y,
                                                  const cx<R>* __restrict__ H, const R* __restrict__ snr_lin,
                                                  const uint32_t* __restrict__ pw, int PW, int n_bits,
                                                  uint32_t* __restrict__ frame_err, R* __restrict__ llr,
                                                  cx<R>* __restrict__ cap_syms, uint8_t* __restrict__ cap_bits,
                                                  cx<R>* __restrict__ zo, R* __restrict__ nvo) {
  using V = cx<R>;
  constexpr bool F64 = sizeof(R) == 8;
  const int npair = m.n_dsc >> 1;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t per = (int64_t)g.n_sym * npair;
  // lanes past the batch stay in the wave (convergent error reduction) and
  // work on a clamped, valid index without storing anything
  const bool act = i < (int64_t)B * per;
  const int b = act ? (int)(i / per) : B - 1;
  const int rem = act ? (int)(i - (int64_t)b * per) : 0, l = rem / npair, pr = rem - l * npair, j = 2 * pr;
  const int e = l / 14;
  V z0 = mkc((R)0, (R)0), z1 = mkc((R)0, (R)0);
  R inv_g = (R)0;
  for (int rx = 0; rx < m.num_rx; ++rx) {
    const V* Yr = Y + (((size_t)b * g.n_sym + l) * m.num_rx + rx) * m.n_dsc;
    const V* H0 = H + ((((size_t)b * m.num_rx + rx) * m.n_est + e) * m.num_tx + 0) * m.n_dsc;
    const V* H1 = H0 + m.n_dsc;
    V d0, d1;
    const R nrm = sfbc_combine<R>(Yr[j], Yr[j + 1], H0[j], H1[j], H0[j + 1], H1[j + 1], (R)1e-10, d0, d1);
    z0 = cadd(z0, d0);
    z1 = cadd(z1, d1);
    if constexpr (F64) inv_g += 1.0 / fmin(fmax(nrm, 1e-6), 1e6);
    else inv_g += 1.0f / fminf(fmaxf(nrm, 1e-6f), 1e6f);
  }
  const R ir = (R)1 / (R)m.num_rx;
  z0 = mkc(z0.x * ir, z0.y * ir);
  z1 = mkc(z1.x * ir, z1.y * ir);
  const int64_t re = (int64_t)l * m.res + j;
  if (cap_syms && act) {
    cap_syms[(size_t)b * g.n_sym * m.res + re] = z0;
    cap_syms[(size_t)b * g.n_sym * m.res + re + 1] = z1;
  }
  if constexpr (CODED) {
    const R s2 = (R)1 / snr_lin[b];
    const R nv = F64 ? fmax((s2 / (R)(m.num_rx * m.num_rx)) * inv_g, s2 / (R)4) : fmax(s2 * ir * ir * inv_g, s2 * (R)0.25);
    if (zo) {   // k_dematch_zn demaps: (z0, z1) and the pair's sigma^2_eff (24 B per RE instead of 8 bps)
      if (!act) return;
      zo[(size_t)b * g.n_sym * m.res + re] = z0;
      zo[(size_t)b * g.n_sym * m.res + re + 1] = z1;
      nvo[(size_t)b * g.n_sym * (m.res >> 1) + (size_t)l * (m.res >> 1) + pr] = nv;
      return;
    }
    R o[BPS];
    R* lo = llr + ((size_t)b * g.n_sym * m.res + re) * BPS;
    if (!act) return;
    soft_demap<BPS>(z0, nv, o);
#pragma unroll
    for (int q = 0; q < BPS; ++q) lo[q] = o[q];
    soft_demap<BPS>(z1, nv, o);
#pragma unroll
    for (int q = 0; q < BPS; ++q) lo[BPS + q] = o[q];
  } else {
    const uint32_t* fb = pw + (size_t)b * PW;
    uint32_t errs = 0;
    for (int h = 0; h < 2; ++h) {
      const int idx = hard_index(h ? z1 : z0, BPS, (R)qam_norm<BPS>());
      const int64_t pb0 = (re + h) * BPS;
      if (act) {
        errs += __popc(((uint32_t)idx ^ getbits<BPS>(fb, pb0, n_bits)) & bits_valid<BPS>(pb0, n_bits));
        if (cap_bits) {
#pragma unroll
          for (int q = 0; q < BPS; ++q)
            if (pb0 + q < n_bits) cap_bits[(size_t)b * n_bits + pb0 + q] = (uint8_t)((idx >> (BPS - 1 - q)) & 1);
        }
      }
    }
    frame_err_add(frame_err, b, errs);
  }
}

template <class R>
int launch_det_sfbc(hipStream_t s, const Grid& g, const MimoGrid& m, int coded, int rayleigh, int B, const cx<R>* Y,
                    const cx<R>* H, const R* snr_lin, const uint32_t* pw, int PW, int n_bits, uint32_t* frame_err,
                    R* llr, cx<R>* cap_syms, uint8_t* cap_bits, cx<R>* zo, R* nvo) {
  (void)rayleigh;
  if (zo && (!coded || !nvo || (m.res & 1) || m.n_dsc > m.res)) return (int)hipErrorInvalidValue;
  const int64_t n = (int64_t)B * g.n_sym * (m.n_dsc >> 1);
  const dim3 grid((unsigned)((n + MWG - 1) / MWG));
#define LTE_DS(C_, B_) \
  hipLaunchKernelGGL((k_det_sfbc<R, C_, B_>), grid, dim3(MWG), 0, s, g, m, B, Y, H, snr_lin, pw, PW, n_bits, \
                     frame_err, llr, cap_syms, cap_bits, zo, nvo)
  if (coded) {
    if (g.bps == 2) LTE_DS(1, 2); else if (g.bps == 4) LTE_DS(1, 4); else LTE_DS(1, 6);
  } else {
    if (g.bps == 2) LTE_DS(0, 2); else if (g.bps == 4) LTE_DS(0, 4); else LTE_DS(0, 6);
  }
#undef LTE_DS
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Config 4's receiver and SFBC detector in one pass: one slot per frame walks
// its OFDM symbols; per symbol each RX in order is loaded with its noise and
// FFT'd (k_rx_fft_mimo's per-symbol work), on the group's first symbol its LS
// pilot estimates per TX stay in LDS, and each thread's Alamouti pairs are
// combined (sfbc_combine with the estimates interpolated at the pair's
// subcarriers, mimo_interp) and summed over RX in RX order -- k_det_sfbc's
// arithmetic.  Y and H never go through HBM.  Outputs: the combined symbols and
// each pair's sigma^2_eff for k_dematch_zn (coded), or the bit errors
// (uncoded).  N = 2048, one slot per block.
template <class R, int CODED, int BPS, int NC = 2048>
__global__ __launch_bounds__(MWG) void k_rx_sfbc(Grid g, MimoGrid m, int B, const cx<R>* __restrict__ y,
                                                 const R* __restrict__ npow, const uint64_t* __restrict__ fid,
                                                 uint64_t seed, const R* __restrict__ snr_lin,
                                                 const uint32_t* __restrict__ pw, int PW, int n_bits,
                                                 uint32_t* __restrict__ frame_err, cx<R>* __restrict__ zo,
                                                 R* __restrict__ nvo) {
  using V = cx<R>;
  constexpr bool F64 = sizeof(R) == 8;
  constexpr int N = NC, T = N >> 3, PP = 3;   // Alamouti pairs per thread: n_dsc / 2 <= PP T
  static_assert(T == MWG, "one slot per block");
  V* sm = mimo_lds<V>();
  V* buf = sm;
  V* hpa = sm + N;   // [num_rx][num_tx][maxP] LS pilot estimates of the current group
  LTE_BM_LDS_DECL(R);
  const auto bmt = bm_stage<R>(lte_bmt);
  const int b = blockIdx.x, tid0 = threadIdx.x;
  const bool active = b < B;   // (grid = B blocks)
  const int npair = m.n_dsc >> 1;
  const R sc = rx_scale<R>(N);
  const V* pv = MGT<R>::pval(m);
  const R* pig = MGT<R>::pig(m);
  const uint64_t fr = fid[b];
  const R s2 = (R)1 / snr_lin[b];
  const R ir = (R)1 / (R)m.num_rx;
  uint32_t errs = 0;
  __syncthreads();
  for (int l = 0; l < g.n_sym; ++l) {
    const bool est = (l % 14) == 0;
    V z[PP][2];
    R inv_g[PP];
#pragma unroll
    for (int k = 0; k < PP; ++k) {
      z[k][0] = z[k][1] = mkc((R)0, (R)0);
      inv_g[k] = (R)0;
    }
    for (int rx = 0; rx < m.num_rx; ++rx) {
      int tid = tid0;   // opaque per pass (see k_rx_frame)
      asm volatile("" : "+v"(tid));
      const size_t br = (size_t)b * m.num_rx + rx;
      const R sigma = sqrt(npow[br] * (R)0.5);
      load_symbol_noisy2<true>(buf, y + br * g.L, N, g.cp, l, sigma, seed, fr, rx, (const R*)nullptr, g.L, tid, T,
                               bmt);
      __syncthreads();
      fft_lds<false, NC, false, true, true>(buf, N, g.log2N, GridT<R>::tw(g), tid, active);
      V* hp = hpa + rx * (m.num_tx * m.maxP);
      if (est) {
        for (int t = 0; t < m.num_tx; ++t)
          for (int p = tid; p < m.np_tx[t]; p += T)
            hp[t * m.maxP + p] = cdiv(cscale(buf[m.ppos[t * m.maxP + p]], sc), pv[t * m.maxP + p]);
        __syncthreads();
      }
#pragma unroll
      for (int k = 0; k < PP; ++k) {
        const int pr = tid + k * T;
        if (pr >= npair) break;
        const int j = 2 * pr;
        const V Y0 = cscale(buf[g.data_idx[j]], sc), Y1 = cscale(buf[g.data_idx[j + 1]], sc);
        const V h0k = mimo_interp<R>(g, m, hp, m.np_tx[0], pig, 0, j);
        const V h1k = mimo_interp<R>(g, m, hp + m.maxP, m.np_tx[1], pig, 1, j);
        const V h0k1 = mimo_interp<R>(g, m, hp, m.np_tx[0], pig, 0, j + 1);
        const V h1k1 = mimo_interp<R>(g, m, hp + m.maxP, m.np_tx[1], pig, 1, j + 1);
        V d0, d1;
        const R nrm = sfbc_combine<R>(Y0, Y1, h0k, h1k, h0k1, h1k1, (R)1e-10, d0, d1);
        z[k][0] = cadd(z[k][0], d0);
        z[k][1] = cadd(z[k][1], d1);
        if constexpr (F64) inv_g[k] += 1.0 / fmin(fmax(nrm, 1e-6), 1e6);
        else inv_g[k] += 1.0f / fminf(fmaxf(nrm, 1e-6f), 1e6f);
      }
      __syncthreads();   // buf (and on estimate symbols hp) rewritten by the next pass
    }
#pragma unroll
    for (int k = 0; k < PP; ++k) {
      const int pr = tid0 + k * T;
      if (pr >= npair) break;
      const int j = 2 * pr;
      const V z0 = mkc(z[k][0].x * ir, z[k][0].y * ir), z1 = mkc(z[k][1].x * ir, z[k][1].y * ir);
      const int64_t re = (int64_t)l * m.res + j;
      if constexpr (CODED) {
        const R nv = F64 ? fmax((s2 / (R)(m.num_rx * m.num_rx)) * inv_g[k], s2 / (R)4)
                         : fmax(s2 * ir * ir * inv_g[k], s2 * (R)0.25);
        zo[(size_t)b * g.n_sym * m.res + re] = z0;
        zo[(size_t)b * g.n_sym * m.res + re + 1] = z1;
        nvo[(size_t)b * g.n_sym * (m.res >> 1) + (size_t)l * (m.res >> 1) + pr] = nv;
      } else {
        const uint32_t* fb = pw + (size_t)b * PW;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int idx = hard_index(h ? z1 : z0, BPS, (R)qam_norm<BPS>());
          const int64_t pb0 = (re + h) * BPS;
          errs += __popc(((uint32_t)idx ^ getbits<BPS>(fb, pb0, n_bits)) & bits_valid<BPS>(pb0, n_bits));
        }
      }
    }
  }
  if constexpr (!CODED) frame_err_add(frame_err, b, errs);
}

template <class R>
bool rx_sfbc_supported(const Grid& g, const MimoGrid& m) {
  return m.mode == MIMO_SFBC && m.num_tx == 2 && m.num_rx >= 1 && m.num_rx <= 4 && g.N == 2048 &&
         (m.n_dsc >> 1) <= 3 * (g.N >> 3) && (m.res & 1) == 0 && m.n_dsc <= m.res && m.n_est == (g.n_sym + 13) / 14 &&
         (g.bps == 2 || g.bps == 4 || g.bps == 6);
}

template <class R>
int launch_rx_sfbc(hipStream_t s, const Grid& g, const MimoGrid& m, int coded, int B, const cx<R>* y, const R* npow,
                   const uint64_t* fid, uint64_t seed, const R* snr_lin, const uint32_t* pw, int PW, int n_bits,
                   uint32_t* frame_err, cx<R>* zo, R* nvo) {
  if (!rx_sfbc_supported<R>(g, m) || (coded && (!zo || !nvo))) return (int)hipErrorInvalidValue;
  const size_t shm = ((size_t)g.N + (size_t)m.num_rx * m.num_tx * m.maxP) * sizeof(cx<R>);
#define LTE_RS(C_, B_)                                                                                        \
  hipLaunchKernelGGL((k_rx_sfbc<R, C_, B_>), dim3(B), dim3(MWG), shm, s, g, m, B, y, npow, fid, seed, snr_lin, pw, \
                     PW, n_bits, frame_err, zo, nvo)
  if (coded) {
    if (g.bps == 2) LTE_RS(1, 2); else if (g.bps == 4) LTE_RS(1, 4); else LTE_RS(1, 6);
  } else {
    if (g.bps == 2) LTE_RS(0, 2); else if (g.bps == 4) LTE_RS(0, 4); else LTE_RS(0, 6);
  }
#undef LTE_RS
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// TM4 detection (MIMODetector, core/mimo_detector.py:55-369) per (frame,
// symbol, data SC j < ceil(Nd/rank)): H_eff = H W (num_rx x rank, W the TM4
// codebook precoder), nominal s2 = 10^(-SNR/10) (core/ofdm_core.py:2737):
//   MMSE / IRC  s = (He^H He + s2 I)^-1 He^H y                      (:135-173)
//   ZF          s = pinv(He) y = (He^H He)^-1 He^H y (full column rank) (:175-198)
//   SIC         layers ordered by ||h_i||^2 / (sum_{j!=i} ||h_j||^2 + s2 + 1e-10)
//               (np.argsort()[::-1]: descending, ties -> higher index), each
//               detected by MMSE over the still-undetected columns, sliced to
//               the nearest constellation point (first index on ties) and
//               cancelled with its original column                  (:200-350)
//   MRC         rank 1: s = conj(h) y / ||h||^2                      (:352-369)
// Layer t of SC j is QAM symbol rank*j + t of the OFDM symbol
// (LayerMapper.demap_from_layers, core/layer_mapper.py:81-115).  Float64 in
// registers throughout: every dimension is unrolled to 4 with runtime guards
// (num_rx, rank <= 4), so nothing is indexed dynamically (no scratch).  An
// undetected / absent layer is a zero column: the masked normal matrix is then
// block diagonal with s2 on the masked diagonal, and the Cholesky solve of the
// full 4x4 system equals the solve over the remaining columns.
struct dc { double x, y; };
__device__ __forceinline__ dc dmul(dc a, dc b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
__device__ __forceinline__ dc dmulc(dc a, dc b) { return {a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y}; }  // a*conj(b)
__device__ __forceinline__ dc dsub(dc a, dc b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ dc dadd(dc a, dc b) { return {a.x + b.x, a.y + b.y}; }

constexpr int DMAX = 4;   // num_rx, rank <= 4 on the GPU path

// Solve (He_m^H He_m + s2 I) s = He_m^H y over the columns with mask bit set
// (others -> 0) by Cholesky; s2 = 0 gives the ZF normal equations.
__device__ __forceinline__ void masked_solve(const dc (&He)[DMAX][DMAX], const dc (&y)[DMAX], int mask, double s2,
                                             dc (&sv)[DMAX]) {
  dc A[DMAX][DMAX], rhs[DMAX];
#pragma unroll
  for (int a = 0; a < DMAX; ++a) {
    const bool ia = (mask >> a) & 1;
#pragma unroll
    for (int c = 0; c <= a; ++c) {
      const bool ic = (mask >> c) & 1;
      dc acc = {0.0, 0.0};
      if (ia && ic) {
#pragma unroll
        for (int r = 0; r < DMAX; ++r) {
          const dc p = dmulc(He[r][c], He[r][a]);   // conj(He[r][a]) He[r][c] = (He^H He)[a][c]
          acc.x += p.x; acc.y += p.y;
        }
      }
      if (a == c) acc.x += ia ? s2 : 1.0;
      A[a][c] = acc;
    }
    dc acc = {0.0, 0.0};
    if (ia) {
#pragma unroll
      for (int r = 0; r < DMAX; ++r) {
        const dc p = dmulc(y[r], He[r][a]);
        acc.x += p.x; acc.y += p.y;
      }
    }
    rhs[a] = acc;
  }
  dc Lm[DMAX][DMAX];
  double ld[DMAX];
#pragma unroll
  for (int i = 0; i < DMAX; ++i) {
    double d = A[i][i].x;
#pragma unroll
    for (int k = 0; k < i; ++k) d -= Lm[i][k].x * Lm[i][k].x + Lm[i][k].y * Lm[i][k].y;
    ld[i] = sqrt(fmax(d, 1e-300));
    const double inv = 1.0 / ld[i];
#pragma unroll
    for (int j = i + 1; j < DMAX; ++j) {
      dc v = A[j][i];
#pragma unroll
      for (int k = 0; k < i; ++k) v = dsub(v, dmulc(Lm[j][k], Lm[i][k]));   // L[j][k] conj(L[i][k])
      Lm[j][i] = {v.x * inv, v.y * inv};
    }
  }
  dc u[DMAX];
#pragma unroll
  for (int i = 0; i < DMAX; ++i) {
    dc v = rhs[i];
#pragma unroll
    for (int k = 0; k < i; ++k) v = dsub(v, dmul(Lm[i][k], u[k]));
    u[i] = {v.x / ld[i], v.y / ld[i]};
  }
#pragma unroll
  for (int i = DMAX - 1; i >= 0; --i) {
    dc v = u[i];
#pragma unroll
    for (int k = i + 1; k < DMAX; ++k) v = dsub(v, dmulc(sv[k], Lm[k][i]));  // conj(L[k][i]) s[k]
    sv[i] = ((mask >> i) & 1) ? dc{v.x / ld[i], v.y / ld[i]} : dc{0.0, 0.0};
  }
}

// nearest constellation point in float64 (QAMModulator constellation,
// core/modulator.py:28-59; argmin |c - s| with the first index on ties)
__device__ __forceinline__ int level_idx_d(double v, double scale, int nl) {
  const double t = (v * scale + (double)(nl - 1)) * 0.5;
  int i = (int)ceil(t - 0.5);
  return i < 0 ? 0 : (i > nl - 1 ? nl - 1 : i);
}

__device__ __forceinline__ dc slice_d(dc s, int bps) {
  if (bps == 2) {
    const double a = 1.0 / 1.4142135623730951;
    return {s.x < 0.0 ? -a : a, s.y < 0.0 ? -a : a};
  }
  const int nl = 1 << (bps >> 1);
  const double S = bps == 4 ? 3.1622776601683795 : 6.48074069840786;
  const int i = level_idx_d(s.x, S, nl), q = level_idx_d(s.y, S, nl);
  const double inv = 1.0 / S;   // NumPy's complex / real scalar multiplies by the reciprocal
  return {(2.0 * i - (nl - 1)) * inv, (2.0 * q - (nl - 1)) * inv};
}

// One subcarrier.  He rows >= num_rx and columns >= R are zero on entry.
// SIC_ON = false compiles only the linear detectors (the SIC branch would
// otherwise set the register budget of every launch).
template <bool SIC_ON>
__device__ __forceinline__ void detect_sc(const dc (&He)[DMAX][DMAX], const dc (&y)[DMAX], int R, int det, double s2,
                                          int bps, dc (&sv)[DMAX]) {
  const int full = (1 << R) - 1;
  if (det == LTE_DET_MRC) {
    double n2 = 0.0;
    dc acc = {0.0, 0.0};
#pragma unroll
    for (int r = 0; r < DMAX; ++r) {
      n2 += He[r][0].x * He[r][0].x + He[r][0].y * He[r][0].y;
      const dc p = dmulc(y[r], He[r][0]);
      acc.x += p.x; acc.y += p.y;
    }
    sv[0] = {acc.x / n2, acc.y / n2};
#pragma unroll
    for (int l = 1; l < DMAX; ++l) sv[l] = {0.0, 0.0};
    return;
  }
  if (!SIC_ON || det != LTE_DET_SIC || bps == 0) {   // MMSE / IRC / ZF; SIC without a constellation -> MMSE (:225-228)
    masked_solve(He, y, full, det == LTE_DET_ZF ? 0.0 : s2, sv);
    return;
  }
  // SIC: detection position of every layer (descending SINR, ties -> higher index first)
  double nrm[DMAX];
#pragma unroll
  for (int l = 0; l < DMAX; ++l) {
    double a = 0.0;
#pragma unroll
    for (int r = 0; r < DMAX; ++r) a += He[r][l].x * He[r][l].x + He[r][l].y * He[r][l].y;
    nrm[l] = a;
  }
  double sinr[DMAX];
#pragma unroll
  for (int l = 0; l < DMAX; ++l) {
    double itf = 0.0;
#pragma unroll
    for (int j = 0; j < DMAX; ++j)
      if (j != l && j < R) itf += nrm[j];
    sinr[l] = nrm[l] / (itf + s2 + 1e-10);
  }
  int pos[DMAX];
#pragma unroll
  for (int l = 0; l < DMAX; ++l) {
    int p = 0;
#pragma unroll
    for (int j = 0; j < DMAX; ++j)
      if (j < R && j != l) p += (sinr[j] > sinr[l]) || (sinr[j] == sinr[l] && j > l);
    pos[l] = p;
  }
  dc yr[DMAX];
#pragma unroll
  for (int r = 0; r < DMAX; ++r) yr[r] = y[r];
  int mask = full;
#pragma unroll
  for (int it = 0; it < DMAX; ++it) {
    if (it < R) {
      dc est[DMAX];
      masked_solve(He, yr, mask, s2, est);
#pragma unroll
      for (int l = 0; l < DMAX; ++l) {
        if (l < R && pos[l] == it) {
          const dc sh = slice_d(est[l], bps);
          sv[l] = sh;
#pragma unroll
          for (int r = 0; r < DMAX; ++r) yr[r] = dsub(yr[r], dmul(He[r][l], sh));
          mask &= ~(1 << l);
        }
      }
    }
  }
#pragma unroll
  for (int l = 0; l < DMAX; ++l)
    if (l >= R) sv[l] = {0.0, 0.0};
}

#ifndef LTE_DSP_WAVES
#define LTE_DSP_WAVES 4
#endif
// linear detectors: 4 waves per SIMD (<= 128 VGPRs; the kernel waits on its
// loads at 3, 131 VGPRs)
// STG (with HPI): one block per (frame, symbol); the symbol's pilot estimates
// of every (RX, TX) link are staged in LDS with coalesced loads before the
// block's REs interpolate them (each RE's 2 x NR x NT interpolation reads then
// hit LDS instead of gathers through L1 / L2); the block's threads loop over
// the symbol's n_dsc data SCs.
#ifndef LTE_DSP_STG_WAVES   // the staged form's register budget (waves per SIMD)
#define LTE_DSP_STG_WAVES 3
#endif
template <class R, int BPS, bool SIC_ON, bool HPI = false, bool STG = false>
__global__ __launch_bounds__(MWG) __attribute__((amdgpu_waves_per_eu(SIC_ON ? 1 : (STG ? LTE_DSP_STG_WAVES : LTE_DSP_WAVES))))
void k_det_spatial(Grid g, MimoGrid m, int B, const cx<R>* __restrict__ Y,
                                                     const cx<R>* __restrict__ H, const double* __restrict__ nvar,
                                                     const uint32_t* __restrict__ pw, int PW, int n_bits,
                                                     uint32_t* __restrict__ frame_err, cx<R>* __restrict__ cap_syms,
                                                     uint8_t* __restrict__ cap_bits) {
  using V = cx<R>;
  static_assert(!STG || HPI, "staging is of the pilot estimates");
  const int NR = m.num_rx, NT = m.num_tx, R_ = m.rank;
  const int64_t per = (int64_t)g.n_sym * m.n_dsc;
  V* hs = mimo_lds<V>();   // STG: [NR][NT][maxP] this symbol's pilot estimates
  if constexpr (STG) {
    const int bs = blockIdx.x / g.n_sym, ls = blockIdx.x - bs * g.n_sym;
    const int nl = NT * m.maxP;
    for (int k = threadIdx.x; k < NR * nl; k += blockDim.x) {
      const int r = k / nl, q = k - r * nl;
      hs[k] = H[(((size_t)bs * NR + r) * m.n_est + ls) * nl + q];
    }
    __syncthreads();
  }
  for (int jb = 0; jb < (STG ? m.n_dsc : 1); jb += MWG) {
  const int64_t i = STG ? (int64_t)blockIdx.x * per / g.n_sym + jb + threadIdx.x
                        : (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // lanes past the batch (or, STG, past the symbol's data SCs) stay in the wave
  // (convergent error reduction) and work on a clamped, valid index without
  // storing anything
  const bool act = STG ? jb + (int)threadIdx.x < m.n_dsc : i < (int64_t)B * per;
  const int64_t ic = act ? i : (STG ? (int64_t)blockIdx.x * per / g.n_sym : 0);
  const int b = act || STG ? (int)(ic / per) : B - 1;
  const int rem = act || STG ? (int)(ic - (int64_t)b * per) : 0, l = rem / m.n_dsc, j = rem - l * m.n_dsc;
  dc He[DMAX][DMAX], yv[DMAX];
#pragma unroll
  for (int r = 0; r < DMAX; ++r) {
    yv[r] = {0.0, 0.0};
#pragma unroll
    for (int c = 0; c < DMAX; ++c) He[r][c] = {0.0, 0.0};
    if (r < NR) {
      const V v = Y[(((size_t)b * g.n_sym + l) * NR + r) * m.n_dsc + j];
      yv[r] = {(double)v.x, (double)v.y};
    }
  }
  // He[r][c] = sum_t H[r][t] W[t][c], each (r, c) summed in t order; with the
  // pilot estimates (HPI) TX t's interpolation point (segment, offset, 1 / gap)
  // is looked up once for every RX
  const size_t hrs = STG ? (size_t)NT * m.maxP : (size_t)m.n_est * NT * (HPI ? m.maxP : m.n_dsc);
  const V* H0 = STG ? hs : H + ((size_t)b * NR * m.n_est + l) * NT * (HPI ? m.maxP : m.n_dsc) + (HPI ? 0 : j);
#pragma unroll
  for (int t = 0; t < DMAX; ++t) {   // unrolled: the four TX's table and estimate loads in flight together
    if (t >= NT) break;
    int sidx = 0, npt = 0;
    R fk = (R)0, ig = (R)0;
    if constexpr (HPI) {
      npt = m.np_tx[t];
      sidx = m.pseg[t * m.n_dsc + j];
      if (sidx >= 0 && sidx < npt - 1) {
        fk = (R)(g.data_idx[j] - m.ppos[t * m.maxP + sidx]);
        ig = MGT<R>::pig(m)[t * m.maxP + sidx];
      }
    }
#pragma unroll
    for (int r = 0; r < DMAX; ++r) {
      if (r >= NR) break;
      const V* Hr = H0 + r * hrs;
      const V hv = HPI ? mimo_interp_at<R>(Hr + (size_t)t * m.maxP, npt, sidx, fk, ig) : Hr[(size_t)t * m.n_dsc];
      const dc h = {(double)hv.x, (double)hv.y};
#pragma unroll
      for (int c = 0; c < DMAX; ++c)
        if (c < R_) He[r][c] = dadd(He[r][c], dmul(h, dc{m.W[(t * DMAX + c) * 2], m.W[(t * DMAX + c) * 2 + 1]}));
    }
  }
  dc sv[DMAX];
  detect_sc<SIC_ON>(He, yv, R_, m.det, nvar[b], BPS, sv);
  const uint32_t* fb = pw + (size_t)b * PW;
  uint32_t errs = 0;
#pragma unroll
  for (int t = 0; t < DMAX; ++t) {
    const int qi = R_ * j + t;
    if (t >= R_ || qi >= m.res) break;
    const V z = mkc((R)sv[t].x, (R)sv[t].y);
    const int64_t re = (int64_t)l * m.res + qi;
    if (cap_syms && act) cap_syms[(size_t)b * g.n_sym * m.res + re] = z;
    const int idx = hard_index(z, BPS, (R)qam_norm<BPS>());
    const int64_t pb0 = re * BPS;
    if (act) {
      errs += __popc(((uint32_t)idx ^ getbits<BPS>(fb, pb0, n_bits)) & bits_valid<BPS>(pb0, n_bits));
      if (cap_bits) {
#pragma unroll
        for (int q = 0; q < BPS; ++q)
          if (pb0 + q < n_bits) cap_bits[(size_t)b * n_bits + pb0 + q] = (uint8_t)((idx >> (BPS - 1 - q)) & 1);
      }
    }
  }
  frame_err_add(frame_err, b, errs);
  }
}

static int env_flag(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}

template <class R>
int launch_det_spatial(hipStream_t s, const Grid& g, const MimoGrid& m, int B, const cx<R>* Y, const cx<R>* H,
                       const double* nvar, const uint32_t* pw, int PW, int n_bits, uint32_t* frame_err,
                       cx<R>* cap_syms, uint8_t* cap_bits, int h_pilots) {
  if (m.num_tx < 1 || m.num_tx > DMAX || m.num_rx < 1 || m.num_rx > DMAX || m.rank < 1 || m.rank > m.num_rx ||
      m.rank > m.num_tx || !m.W)
    return (int)hipErrorInvalidValue;
  const int64_t n = (int64_t)B * g.n_sym * m.n_dsc;
  const dim3 grid((unsigned)((n + MWG - 1) / MWG));
  // the pilot estimates staged per (frame, symbol) (LTE_DSP_STAGE=0: gathered per RE)
  const size_t hshm = (size_t)m.num_rx * m.num_tx * m.maxP * sizeof(cx<R>);
  const bool stg = h_pilots && hshm <= 32768 && (int64_t)B * g.n_sym < 0x7FFFFFFF && env_flag("LTE_DSP_STAGE", 1);
  const dim3 sgrid((unsigned)((int64_t)B * g.n_sym));
#define LTE_DSP(B_, S_)                                                                                            \
  do {                                                                                                             \
    if (stg)                                                                                                       \
      hipLaunchKernelGGL((k_det_spatial<R, B_, S_, true, true>), sgrid, dim3(MWG), hshm, s, g, m, B, Y, H, nvar,   \
                         pw, PW, n_bits, frame_err, cap_syms, cap_bits);                                           \
    else if (h_pilots)                                                                                             \
      hipLaunchKernelGGL((k_det_spatial<R, B_, S_, true>), grid, dim3(MWG), 0, s, g, m, B, Y, H, nvar, pw, PW,      \
                         n_bits, frame_err, cap_syms, cap_bits);                                                   \
    else                                                                                                           \
      hipLaunchKernelGGL((k_det_spatial<R, B_, S_>), grid, dim3(MWG), 0, s, g, m, B, Y, H, nvar, pw, PW, n_bits,    \
                         frame_err, cap_syms, cap_bits);                                                           \
  } while (0)
  const bool sic = m.det == LTE_DET_SIC;
  if (g.bps == 2) { if (sic) LTE_DSP(2, true); else LTE_DSP(2, false); }
  else if (g.bps == 4) { if (sic) LTE_DSP(4, true); else LTE_DSP(4, false); }
  else { if (sic) LTE_DSP(6, true); else LTE_DSP(6, false); }
#undef LTE_DSP
  return (int)hipGetLastError();
}

// Stage entries (SFBCAlamouti.encode / .decode on host arrays, float64): one
// thread per subcarrier pair.  encode: TX0 [s0, -conj(s1)], TX1 [s1, conj(s0)]
// (core/sfbc_alamouti.py:45-78) -- the same pair rule the chain's TX kernels
// apply; decode: sfbc_combine with the caller's regularization (:80-163).
__global__ __launch_bounds__(MWG) void k_sfbc_encode_stage(int64_t npair, const double2* __restrict__ s,
                                                           double2* __restrict__ tx0, double2* __restrict__ tx1) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npair) return;
  const double2 s0 = s[2 * i], s1 = s[2 * i + 1];
  tx0[2 * i] = s0;
  tx1[2 * i] = s1;
  tx0[2 * i + 1] = make_double2(-s1.x, s1.y);   // -conj(s1)
  tx1[2 * i + 1] = make_double2(s0.x, -s0.y);   // conj(s0)
}

__global__ __launch_bounds__(MWG) void k_sfbc_decode_stage(int64_t npair, const double2* __restrict__ rx,
                                                           const double2* __restrict__ H0,
                                                           const double2* __restrict__ H1, double reg,
                                                           double2* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npair) return;
  const int64_t k = 2 * i;
  double2 d0, d1;
  sfbc_combine<double>(rx[k], rx[k + 1], H0[k], H1[k], H0[k + 1], H1[k + 1], reg, d0, d1);
  out[k] = d0;
  out[k + 1] = d1;
}

int launch_sfbc_stage(hipStream_t s, int decode, int64_t n, const double* a, const double* h0, const double* h1,
                      double reg, double* o0, double* o1) {
  if (n < 2 || (n & 1)) return (int)hipErrorInvalidValue;
  const int64_t np = n >> 1;
  const dim3 grid((unsigned)((np + MWG - 1) / MWG));
  if (decode)
    hipLaunchKernelGGL(k_sfbc_decode_stage, grid, dim3(MWG), 0, s, np, (const double2*)a, (const double2*)h0,
                       (const double2*)h1, reg, (double2*)o0);
  else
    hipLaunchKernelGGL(k_sfbc_encode_stage, grid, dim3(MWG), 0, s, np, (const double2*)a, (double2*)o0,
                       (double2*)o1);
  return (int)hipGetLastError();
}

// Stage entry (MIMODetector.detect on host arrays): one thread per subcarrier,
// float64 y [num_rx][n], H [num_rx][num_tx][n], W [4][4] -> out [rank][n].
__global__ __launch_bounds__(MWG) void k_det_stage(int det, int NR, int NT, int R, int bps, int64_t n,
                                                   const double* __restrict__ y, const double* __restrict__ H,
                                                   const double* __restrict__ W, double s2, double* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  dc He[DMAX][DMAX], yv[DMAX];
#pragma unroll
  for (int r = 0; r < DMAX; ++r) {
    yv[r] = {0.0, 0.0};
#pragma unroll
    for (int c = 0; c < DMAX; ++c) He[r][c] = {0.0, 0.0};
    if (r < NR) {
      yv[r] = {y[((size_t)r * n + k) * 2], y[((size_t)r * n + k) * 2 + 1]};
      for (int t = 0; t < NT; ++t) {
        const dc h = {H[(((size_t)r * NT + t) * n + k) * 2], H[(((size_t)r * NT + t) * n + k) * 2 + 1]};
#pragma unroll
        for (int c = 0; c < DMAX; ++c)
          if (c < R) He[r][c] = dadd(He[r][c], dmul(h, dc{W[(t * DMAX + c) * 2], W[(t * DMAX + c) * 2 + 1]}));
      }
    }
  }
  dc sv[DMAX];
  detect_sc<true>(He, yv, R, det, s2, bps, sv);
#pragma unroll
  for (int l = 0; l < DMAX; ++l)
    if (l < R) {
      out[((size_t)l * n + k) * 2] = sv[l].x;
      out[((size_t)l * n + k) * 2 + 1] = sv[l].y;
    }
}

int launch_det_stage(hipStream_t s, int det, int NR, int NT, int R, int bps, int64_t n, const double* y,
                     const double* H, const double* W, double s2, double* out) {
  hipLaunchKernelGGL(k_det_stage, dim3((unsigned)((n + MWG - 1) / MWG)), dim3(MWG), 0, s, det, NR, NT, R, bps, n, y,
                     H, W, s2, out);
  return (int)hipGetLastError();
}

// explicit instances: float (fast mode) and double (the reference's precision)
#define LTE_MIMO_INST(R)                                                                                           \
  template int launch_ofdm_txch_sfbc<R>(hipStream_t, const Grid&, const MimoGrid&, int, const uint32_t*, int,     \
                                        const uint32_t*, int, const int32_t*, const TxLinkPower<R>&, cx<R>*, int); \
  template int launch_npow_sfbc_merged<R>(hipStream_t, int, int, int, const R*, int, const R*, R*);             \
  template int launch_link_noise_add<R>(hipStream_t, const Grid&, const MimoGrid&, int, const R*, R*, cx<R>*,      \
                                        const uint64_t*, uint64_t, R*, int*);                                      \
  template bool sfbc_txch_supported<R>(const Grid&, const MimoGrid&, int, int);                                   \
  template int launch_ofdm_tx_mimo<R>(hipStream_t, const Grid&, const MimoGrid&, int, const uint32_t*, int,       \
                                      const uint32_t*, int, const int32_t*, cx<R>*, int, const TxLinkPower<R>&);   \
  template int launch_ofdm_txch_flat<R>(hipStream_t, const Grid&, const MimoGrid&, int, const uint32_t*, int,     \
                                        const uint32_t*, int, const int32_t*, const cx<R>*, cx<R>*, R*, int, int); \
  template int launch_fading_mimo<R>(hipStream_t, const Grid&, const MimoGrid&, int, int, int, const R*, double,   \
                                     double, const uint64_t*, uint64_t, const R*, int64_t, const R*, int64_t,      \
                                     cx<R>*, R*);                                                                  \
  template int launch_channel_mimo<R>(hipStream_t, const Grid&, const MimoGrid&, int, int, const int32_t*,         \
                                      const cx<R>*, const R*, const R*, double, const cx<R>*, cx<R>*, int,         \
                                      const uint64_t*, uint64_t, const R*, int64_t, R*, R*, R*, int, int);    \
  template int launch_link_stats<R>(hipStream_t, const Grid&, const MimoGrid&, int, int, const int32_t*,           \
                                    const cx<R>*, const R*, const R*, double, const cx<R>*, const R*,              \
                                    const uint64_t*, uint64_t, const R*, int64_t, R*, int, R*);                    \
  template int launch_npow_mimo<R>(hipStream_t, int, int, const R*, int, int, const R*, double, R*);               \
  template int launch_rx_fft_mimo<R>(hipStream_t, const Grid&, const MimoGrid&, int, const cx<R>*, const R*,       \
                                     const uint64_t*, uint64_t, const R*, int64_t, cx<R>*, cx<R>*, int);                \
  template bool rx_sfbc_supported<R>(const Grid&, const MimoGrid&);                                                \
  template int launch_rx_sfbc<R>(hipStream_t, const Grid&, const MimoGrid&, int, int, const cx<R>*, const R*,      \
                                 const uint64_t*, uint64_t, const R*, const uint32_t*, int, int, uint32_t*, cx<R>*,  \
                                 R*);                                                                              \
  template int launch_det_sfbc<R>(hipStream_t, const Grid&, const MimoGrid&, int, int, int, const cx<R>*,          \
                                  const cx<R>*, const R*, const uint32_t*, int, int, uint32_t*, R*, cx<R>*,        \
                                  uint8_t*, cx<R>*, R*);                                                           \
  template int launch_det_spatial<R>(hipStream_t, const Grid&, const MimoGrid&, int, const cx<R>*, const cx<R>*,   \
                                     const double*, const uint32_t*, int, int, uint32_t*, cx<R>*, uint8_t*, int);
LTE_MIMO_INST(float)
LTE_MIMO_INST(double)
#undef LTE_MIMO_INST

}  // namespace lte
