// Device helpers shared by the kernel translation units (lte_kernels.hip,
// lte_turbo.hip, lte_mimo.hip, lte_bf.hip): QAM points / slicers / max-log
// demappers, the noisy symbol loader and block reductions.  The SISO / SIMO
// chains instantiate them for both precisions (R = float / double, V =
// cx<R>); the multi-antenna chains use the float instances.
#pragma once
#include "lte_common.h"
#include "lte_internal.h"

namespace lte {

// QAM point of natural-binary index idx (modulator.py:28-59, I-major; QPSK
// [1+1j, 1-1j, -1+1j, -1-1j]/sqrt 2).  f64: NumPy's complex128 table exactly
// -- level * (1/S) (NumPy's complex / real divide multiplies by the
// reciprocal); f32: the float64 table's values cast to float.
template <int BPS, class R = float>
__device__ __forceinline__ cx<R> qam_point(int idx) {
  if constexpr (sizeof(R) == 8) {
    constexpr double S = BPS == 2 ? 1.4142135623730951 : (BPS == 4 ? 3.1622776601683795 : 6.48074069840786);
    constexpr double inv = 1.0 / S;
    if constexpr (BPS == 2) {
      return make_double2((idx & 2) ? -inv : inv, (idx & 1) ? -inv : inv);
    } else {
      constexpr int H = BPS / 2, NL = 1 << H;
      return make_double2((double)(2 * (idx >> H) - (NL - 1)) * inv, (double)(2 * (idx & (NL - 1)) - (NL - 1)) * inv);
    }
  } else if constexpr (BPS == 2) {
    constexpr float a = (float)(1.0 / 1.4142135623730951);
    return make_float2((idx & 2) ? -a : a, (idx & 1) ? -a : a);
  } else {
    constexpr int H = BPS / 2, NL = 1 << H;
    constexpr double S = BPS == 4 ? 3.1622776601683795 : 6.48074069840786;
    float lv[NL];
#pragma unroll
    for (int i = 0; i < NL; ++i) lv[i] = (float)((2.0 * i - (NL - 1)) / S);
    return make_float2(lv[idx >> H], lv[idx & (NL - 1)]);
  }
}

// TX output scale: f32 1/sqrt(N); f64 sqrt(N)/N, which for a power-of-two N
// is exactly NumPy's ifft(.) * sqrt(N) (the 1/N is a power of two)
template <class R>
__device__ __forceinline__ R tx_scale(int N) {
  if constexpr (sizeof(R) == 8) return sqrt((double)N) / (double)N;
  else return rsqrtf((float)N);
}
// RX FFT scale: fft(.) / sqrt(N); NumPy's complex / real divide multiplies by
// the reciprocal, so f64 uses 1.0 / sqrt(N)
template <class R>
__device__ __forceinline__ R rx_scale(int N) {
  if constexpr (sizeof(R) == 8) return 1.0 / sqrt((double)N);
  else return rsqrtf((float)N);
}

template <class R>
__device__ __forceinline__ R block_sum(R v, R* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  R t = (R)0;
  if (threadIdx.x == 0) {
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
  }
  return t;
}

// Load one OFDM symbol (CP removed) of (frame, rx) into LDS adding AWGN:
// noise = sigma * z, sigma = sqrt(P/SNR/2) (channel.py:52-60).
// SW: samples land in the FFT's swizzled layout (fft_sw<V>, read by
// fft_lds<.., ISW = true>).
template <bool SW = false, class V>
__device__ __forceinline__ void load_symbol_noisy(V* buf, const V* __restrict__ yf, int N, int cp, int l,
                                                  re_t<V> sigma, uint64_t seed, uint64_t frame, int rx,
                                                  const re_t<V>* __restrict__ zf /*inj: [2][L] or null*/, int L,
                                                  int tid, int T) {
  using R = re_t<V>;
  const int off = l * (N + cp) + cp;
  for (int k = tid; k < N; k += T) {
    const int n = off + k;
    V z;
    if (zf) {
      z = mkc(zf[n], zf[L + n]);
    } else {
      const u32x4 r = rng4(seed, frame, RNG_STREAM_NOISE + (uint32_t)rx, (uint32_t)(n >> 1));
      z = (n & 1) ? gauss2<R>(r.z, r.w) : gauss2<R>(r.x, r.y);
    }
    const V v = yf[n];
    buf[SW ? fft_sw<V>(k) : k] = mkc(v.x + sigma * z.x, v.y + sigma * z.y);
  }
}

__device__ __forceinline__ int level_idx(float v, float scale, int nl) {
  // nearest of the nl levels (2i-(nl-1))/scale, ties -> lower level (argmin
  // returns the first index, modulator.py:106)
  const float t = (v * scale + (float)(nl - 1)) * 0.5f;
  int i = (int)ceilf(t - 0.5f);
  return i < 0 ? 0 : (i > nl - 1 ? nl - 1 : i);
}
__device__ __forceinline__ int level_idx(double v, double scale, int nl) {
  const double t = (v * scale + (double)(nl - 1)) * 0.5;
  int i = (int)ceil(t - 0.5);
  return i < 0 ? 0 : (i > nl - 1 ? nl - 1 : i);
}

template <class V>
__device__ __forceinline__ int hard_index(V y, int bps, re_t<V> scale) {
  using R = re_t<V>;
  if (bps == 2) return (y.x < (R)0 ? 2 : 0) | (y.y < (R)0 ? 1 : 0);  // [1+1j,1-1j,-1+1j,-1-1j]
  const int nl = 1 << (bps >> 1);
  return (level_idx(y.x, scale, nl) << (bps >> 1)) | level_idx(y.y, scale, nl);
}

// sqrt(2), sqrt(10), sqrt(42): the QAM normalisations of modulator.py:28-59
template <int BPS>
__host__ __device__ constexpr double qam_norm() { return BPS == 2 ? 1.4142135623730951 : (BPS == 4 ? 3.1622776601683795 : 6.48074069840786); }

// max-log LLRs (core/ofdm_core.py:791-923): QPSK 2*sqrt(2)*y/nv (no clip);
// 16/64-QAM (min_{b=1} d^2 - min_{b=0} d^2)/(2 nv) clipped to +-10.  The
// natural-binary map makes the metric separable per axis.  NB bits per axis.
// f32: levels folded to constants, 1/(2 nv) as a multiplier (q = 1/(2 nv));
// f64: NumPy's level values and the reference's division (q = 2 nv).
template <int NB, class R>
__device__ __forceinline__ void llr_axis(R v, R q, R* out) {
  constexpr int NL = 1 << NB;
  constexpr double S = NB == 2 ? 3.1622776601683795 : 6.48074069840786;
  R m0[NB], m1[NB];
#pragma unroll
  for (int bb = 0; bb < NB; ++bb) { m0[bb] = (R)3.4e38f; m1[bb] = (R)3.4e38f; }
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const R lv = sizeof(R) == 8 ? (R)((double)(2 * i - (NL - 1)) * (1.0 / S)) : (R)((2.0 * i - (NL - 1)) / S);
    const R d = (v - lv) * (v - lv);
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
      if ((i >> (NB - 1 - bb)) & 1) m1[bb] = fmin(m1[bb], d);
      else m0[bb] = fmin(m0[bb], d);
    }
  }
#pragma unroll
  for (int bb = 0; bb < NB; ++bb) {
    const R x = sizeof(R) == 8 ? (m1[bb] - m0[bb]) / q : (m1[bb] - m0[bb]) * q;
    out[bb] = fmin((R)10, fmax((R)-10, x));
  }
}

template <int BPS, class V>
__device__ __forceinline__ void soft_demap(V y, re_t<V> nv, re_t<V>* out) {
  using R = re_t<V>;
  if constexpr (BPS == 2) {
    const R s2 = sizeof(R) == 8 ? (R)1.4142135623730951 : (R)1.41421356237309515f;
    out[0] = ((R)2 / nv) * y.x * s2;
    out[1] = ((R)2 / nv) * y.y * s2;
  } else {
    const R q = sizeof(R) == 8 ? (R)2 * nv : (R)1 / ((R)2 * nv);
    llr_axis<BPS / 2, R>(y.x, q, out);
    llr_axis<BPS / 2, R>(y.y, q, out + BPS / 2);
  }
}

// y / h (lte_receiver.py:154-180 divides by H + 1e-6): multiply by the conjugate
// over |h|^2; f32 relative error a few ulp (no over/underflow at these magnitudes).
__device__ __forceinline__ float2 zf_div(float2 y, float2 h) {
  const float r = 1.0f / (h.x * h.x + h.y * h.y);
  return make_float2((y.x * h.x + y.y * h.y) * r, (y.y * h.x - y.x * h.y) * r);
}
// ZF equaliser Y / (H + 1e-6): f32 as above; f64 NumPy's complex division
// (Smith's algorithm)
__device__ __forceinline__ float2 zf_eq(float2 y, float2 h) { return zf_div(y, make_float2(h.x + 1e-6f, h.y)); }
__device__ __forceinline__ double2 zf_eq(double2 y, double2 h) { return cdiv(y, make_double2(h.x + 1e-6, h.y)); }

// the link's 100 dB noise: y + (s z_re + j s z_im) (injected [2][L] or Philox)
template <class R>
__device__ __forceinline__ cx<R> link_noise_at(int n, R sg, const R* __restrict__ zf, int L, uint64_t seed,
                                               uint64_t frame, int link, cx<R> v) {
  cx<R> z;
  if (zf) {
    z = mkc(zf[n], zf[L + n]);
  } else {
    const u32x4 rr = rng4(seed, frame, RNG_STREAM_MIMO_LINK + (uint32_t)link, (uint32_t)(n >> 1));
    z = (n & 1) ? gauss2<R>(rr.z, rr.w) : gauss2<R>(rr.x, rr.y);
  }
  return mkc(v.x + sg * z.x, v.y + sg * z.y);
}

// transmit_mimo's 100 dB link noise on the Philox path, per receive antenna:
// the num_tx links' independent complex Gaussians (standard deviations s_rt,
// k_link_sigma) sum to one complex Gaussian of standard deviation
// sqrt(sum_t s_rt^2), drawn once per RX sample on link (r, 0)'s stream -- the
// same distribution as one draw per link at 1 / num_tx of the draws.  (Injected
// link noise, the reference's own draws, is still added per link.)
template <class R>
__device__ __forceinline__ R rx_link_sigma(const R* __restrict__ link_sigma, size_t lk0, int num_tx) {
#pragma clang fp contract(off)
  R s2 = (R)0;
  for (int t = 0; t < num_tx; ++t) {
    const R s = link_sigma[lk0 + t];
    s2 = s2 + s * s;
  }
  return sqrt(s2);
}

// The float64 Box-Muller tables of a block's noise draws: staged into its
// static LDS array bmt (BM_LDS_BYTES; the 4-8 table gathers per draw then hit
// LDS instead of the L1 / L2: the config-4 link-noise pass 32.0 -> 27.1 ms per
// 65 536 frames); float32 draws use no tables.  A barrier must follow before
// the first draw.
#ifndef LTE_BM_LDS   // 0: the __constant__ tables (A/B builds)
#define LTE_BM_LDS 1
#endif
template <class R>
__device__ __forceinline__ auto bm_stage(double2* bmt) {
  if constexpr (sizeof(R) == 8 && LTE_BM_LDS) return bm_tables_lds(bmt, threadIdx.x, blockDim.x);
  else return BmTabC{};
}
#define LTE_BM_LDS_DECL(R) __shared__ double2 lte_bmt[sizeof(R) == 8 && LTE_BM_LDS ? BM_LDS_BYTES / 16 : 1]

// Noise-add for one OFDM symbol into LDS, one Philox call per pair of
// samples (sample n uses half (n&1) of counter n>>1 -- same draws as
// load_symbol_noisy, at half the generator cost).  Lane t stores samples 2t
// and 2t + 1 (a stride-2 ds_write pattern, 2-way on 16-B and 8-B elements);
// SW = true stores them swizzled (conflict-free) for fft_lds<.., ISW = true>.
// tb: where the float64 Box-Muller tables are read (bm_stage).
template <bool SW = false, class V, class TB = BmTabC>
__device__ __forceinline__ void load_symbol_noisy2(V* buf, const V* __restrict__ yf, int N, int cp, int l,
                                                   re_t<V> sigma, uint64_t seed, uint64_t frame, int rx,
                                                   const re_t<V>* __restrict__ zf, int L, int tid, int T,
                                                   const TB& tb = TB{}) {
  using R = re_t<V>;
  const int off = l * (N + cp) + cp;
  if (zf) {
    load_symbol_noisy<SW>(buf, yf, N, cp, l, sigma, seed, frame, rx, zf, L, tid, T);
    return;
  }
  const int p0 = off >> 1, p1 = (off + N - 1) >> 1;
  // every sample load of this thread is issued before the first Philox call
  // (the loop was latency bound with one pair in flight); T = N/8 threads
  // cover the N/2 (+1) pairs in at most 5 rounds
  constexpr int MAXR = 5;
  V va[MAXR], vb[MAXR];
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int p = p0 + tid + i * T, n0 = 2 * p;
    va[i] = (p <= p1 && n0 >= off) ? yf[n0] : mkc((R)0, (R)0);
    vb[i] = (p <= p1 && n0 + 1 < off + N) ? yf[n0 + 1] : mkc((R)0, (R)0);
  }
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int p = p0 + tid + i * T, n0 = 2 * p;
    if (p > p1) break;
    const u32x4 r = rng4(seed, frame, RNG_STREAM_NOISE + (uint32_t)rx, (uint32_t)p);
    if (n0 >= off) {
      const V z = gauss2t<R>(r.x, r.y, tb);
      buf[SW ? fft_sw<V>(n0 - off) : n0 - off] = mkc(va[i].x + sigma * z.x, va[i].y + sigma * z.y);
    }
    if (n0 + 1 < off + N) {
      const V z = gauss2t<R>(r.z, r.w, tb);
      buf[SW ? fft_sw<V>(n0 + 1 - off) : n0 + 1 - off] = mkc(vb[i].x + sigma * z.x, vb[i].y + sigma * z.y);
    }
  }
}

// SC-FDM DFT (DFTPrecodifier, core/dft_precoding.py:43-90: X_k = sum_n x_n
// exp(-2 pi i k n / M) / sqrt(M), M = Nd) in place on buf[0, M), buf[M, N)
// zero on entry.  Bluestein: X_k = conj(w_k) sum_n (x_n conj(w_n)) w_{k-n},
// w_m = exp(i pi m^2 / M), the convolution by N-point LDS FFTs (N >= 2M - 1
// since Nd < N/2).  The inverse (IDFTDecodifier) is conj(DFT(conj(x))).  All
// threads of the block call it; it begins and ends with a barrier.
template <class V>
__device__ __forceinline__ void dft_bluestein(V* buf, const Grid& g, int tid, int T, bool active) {
  using G = GridT<re_t<V>>;
  __syncthreads();
  if (active)
    for (int n = tid; n < g.Nd; n += T) buf[n] = cmul(buf[n], G::chirp(g)[n]);
  __syncthreads();
  fft_lds<false>(buf, g.N, g.log2N, G::tw(g), tid, active);
  if (active)
    for (int k = tid; k < g.N; k += T) buf[k] = cmul(buf[k], G::bhat(g)[k]);
  __syncthreads();
  fft_lds<true>(buf, g.N, g.log2N, G::tw(g), tid, active);
  if (active)
    for (int k = tid; k < g.Nd; k += T) buf[k] = cmul(buf[k], G::chirp(g)[k]);
  __syncthreads();
}

// frame_err[b] += errs for every lane, with one atomic per distinct frame per
// wave instead of one per lane (thousands of lanes of a frame otherwise
// serialise on the same L2 address).  Must be reached by all lanes of the
// wave; lanes without work pass errs = 0.
__device__ __forceinline__ void frame_err_add(uint32_t* __restrict__ frame_err, int b, uint32_t errs) {
  unsigned long long pending = __ballot(errs != 0u);
  while (pending) {
    const int src = __ffsll((long long)pending) - 1;
    const int bb = __shfl(b, src);
    const bool mine = errs != 0u && b == bb;
    uint32_t v = mine ? errs : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((int)__lane_id() == src) atomicAdd(frame_err + bb, v);
    pending &= ~__ballot(mine);
  }
}

// Per-OFDM-symbol Taylor sets of one path's Jakes sum (jakes_fading,
// core/rayleighchannel.py:20-42): for symbol s with centre c_s (samples
// s * sym_len + (sym_len - 1) / 2), h(c_s + d) = sum_k c_k d^k with
//  * f64: degree 5, c_k = g sqrt(2/16) sum_m a_m (j W_m)^k / k!, a_m =
//    exp(j (w_m t_c + phi_m)) formed like one reference sample, W_m = w_m / fs
//    (valid while mimo_taylor_ok: remainder under float64 rounding);
//  * f32: A + B d + C d^2 computed in float64 (truncation ~1e-10 at 3 km/h),
//    each sinusoid's phasor rotated from symbol to symbol.
// out: n_cs sets of mimo_ncf<R>() terms.  Shared by k_fading_mimo (the
// multi-antenna links) and k_jakes_sets (the fused SISO TX channel).
template <class R>
__device__ __forceinline__ void jakes_symbol_sets(const double (&ph)[16], double gain, double fD, double fs,
                                                  int sym_len, int n_cs, cx<R>* __restrict__ out) {
  constexpr int NCF = mimo_ncf<R>();
  if constexpr (sizeof(R) == 8) {
    const double k = sqrt(2.0 / 16.0), gn = gain;
    for (int sidx = 0; sidx < n_cs; ++sidx) {
      const double tc = ((double)sidx * sym_len + 0.5 * (sym_len - 1)) / fs;
      double cr[NCF], ci[NCF];
      for (int kk = 0; kk < NCF; ++kk) cr[kk] = ci[kk] = 0.0;
      for (int mm = 0; mm < 16; ++mm) {
        const double w = 6.283185307179586 * fD * cos(6.283185307179586 * (double)(mm + 1) / 16.0);
        double sv, cv;
        sincos(w * tc + ph[mm], &sv, &cv);
        const double W = w / fs;
#pragma unroll
        for (int kk = 0; kk < NCF; ++kk) {   // a_m (j W)^k / k!
          cr[kk] += cv;
          ci[kk] += sv;
          const double nr = -sv * (W / (kk + 1)), ni = cv * (W / (kk + 1));
          cv = nr;
          sv = ni;
        }
      }
      for (int kk = 0; kk < NCF; ++kk) out[sidx * NCF + kk] = make_double2(gn * (cr[kk] * k), gn * (ci[kk] * k));
    }
  } else {
    const double k = sqrt(2.0 / 16.0) * gain;
    // per sinusoid: phasor at the first symbol centre, then rotate by w * sym_len
    // per symbol (float64 recurrence: 2 sincos per sinusoid instead of one per symbol)
    double w[16], zr[16], zi[16], rr[16], ri[16];
    const double c0 = fD == 0.0 ? 0.0 : 0.5 * (sym_len - 1);
    for (int mm = 0; mm < 16; ++mm) {
      w[mm] = fD == 0.0 ? 0.0 : 6.283185307179586 * fD * cos(6.283185307179586 * (mm + 1) / 16.0) / fs;
      sincos(w[mm] * c0 + ph[mm], &zi[mm], &zr[mm]);
      sincos(w[mm] * (double)sym_len, &ri[mm], &rr[mm]);
    }
    for (int sidx = 0; sidx < n_cs; ++sidx) {
      double ar = 0, ai = 0, br = 0, bi = 0, cr = 0, ci = 0;
      for (int mm = 0; mm < 16; ++mm) {
        const double cv = zr[mm], sv = zi[mm], wm = w[mm];
        ar += cv; ai += sv;
        br += -wm * sv; bi += wm * cv;                   // j w e^{j th}
        cr += -0.5 * wm * wm * cv; ci += -0.5 * wm * wm * sv;
        zr[mm] = cv * rr[mm] - sv * ri[mm];
        zi[mm] = cv * ri[mm] + sv * rr[mm];
      }
      out[sidx * 3 + 0] = make_float2((float)(ar * k), (float)(ai * k));
      out[sidx * 3 + 1] = make_float2((float)(br * k), (float)(bi * k));
      out[sidx * 3 + 2] = make_float2((float)(cr * k), (float)(ci * k));
    }
  }
}

}  // namespace lte
