// Device helpers shared by the kernel translation units (lte_kernels.hip,
// lte_mimo.hip): QAM points / slicers / max-log demappers, the noisy symbol
// loader and block reductions.
#pragma once
#include "lte_common.h"
#include "lte_internal.h"

namespace lte {

// QAM point of natural-binary index idx (modulator.py:28-59, I-major; QPSK
// [1+1j, 1-1j, -1+1j, -1-1j]/sqrt 2), levels folded to float constants equal
// to the float64 table cast to float.
template <int BPS>
__device__ __forceinline__ float2 qam_point(int idx) {
  if constexpr (BPS == 2) {
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


__device__ __forceinline__ float block_sum(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x == 0) {
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
  }
  return t;
}


__device__ __forceinline__ void load_symbol_noisy(float2* buf, const float2* __restrict__ yf, int N, int cp, int l,
                                                  float sigma, uint64_t seed, uint64_t frame, int rx,
                                                  const float* __restrict__ zf /*inj: [2][L] or null*/, int L,
                                                  int tid, int T) {
  const int off = l * (N + cp) + cp;
  for (int k = tid; k < N; k += T) {
    const int n = off + k;
    float2 z;
    if (zf) {
      z = make_float2(zf[n], zf[L + n]);
    } else {
      const u32x4 r = rng4(seed, frame, RNG_STREAM_NOISE + (uint32_t)rx, (uint32_t)(n >> 1));
      z = (n & 1) ? box_muller(r.z, r.w) : box_muller(r.x, r.y);
    }
    const float2 v = yf[n];
    buf[k] = make_float2(v.x + sigma * z.x, v.y + sigma * z.y);
  }
}


__device__ __forceinline__ int level_idx(float v, float scale, int nl) {
  // nearest of the nl levels (2i-(nl-1))/scale, ties -> lower level (argmin
  // returns the first index, modulator.py:106)
  const float t = (v * scale + (float)(nl - 1)) * 0.5f;
  int i = (int)ceilf(t - 0.5f);
  return i < 0 ? 0 : (i > nl - 1 ? nl - 1 : i);
}

__device__ __forceinline__ int hard_index(float2 y, int bps, float scale) {
  if (bps == 2) return (y.x < 0.f ? 2 : 0) | (y.y < 0.f ? 1 : 0);  // [1+1j,1-1j,-1+1j,-1-1j]
  const int nl = 1 << (bps >> 1);
  return (level_idx(y.x, scale, nl) << (bps >> 1)) | level_idx(y.y, scale, nl);
}

// sqrt(2), sqrt(10), sqrt(42): the QAM normalisations of modulator.py:28-59
template <int BPS>
__host__ __device__ constexpr double qam_norm() { return BPS == 2 ? 1.4142135623730951 : (BPS == 4 ? 3.1622776601683795 : 6.48074069840786); }

// max-log LLRs (core/ofdm_core.py:791-923): QPSK 2*sqrt(2)*y/nv (no clip);
// 16/64-QAM (min_{b=1} d^2 - min_{b=0} d^2)/(2 nv) clipped to +-10.  The
// natural-binary map makes the metric separable per axis.  NB bits per axis,
// levels folded to constants (correctly rounded from the float64 grid).
template <int NB>
__device__ __forceinline__ void llr_axis(float v, float inv2nv, float* out) {
  constexpr int NL = 1 << NB;
  constexpr double S = NB == 2 ? 3.1622776601683795 : 6.48074069840786;
  float m0[NB], m1[NB];
#pragma unroll
  for (int bb = 0; bb < NB; ++bb) { m0[bb] = 3.4e38f; m1[bb] = 3.4e38f; }
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const float lv = (float)((2.0 * i - (NL - 1)) / S);
    const float d = (v - lv) * (v - lv);
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
      if ((i >> (NB - 1 - bb)) & 1) m1[bb] = fminf(m1[bb], d);
      else m0[bb] = fminf(m0[bb], d);
    }
  }
#pragma unroll
  for (int bb = 0; bb < NB; ++bb) out[bb] = fminf(10.f, fmaxf(-10.f, (m1[bb] - m0[bb]) * inv2nv));
}

template <int BPS>
__device__ __forceinline__ void soft_demap(float2 y, float nv, float* out) {
  if constexpr (BPS == 2) {
    out[0] = (2.0f / nv) * y.x * 1.41421356237309515f;
    out[1] = (2.0f / nv) * y.y * 1.41421356237309515f;
  } else {
    const float inv2nv = 1.0f / (2.0f * nv);
    llr_axis<BPS / 2>(y.x, inv2nv, out);
    llr_axis<BPS / 2>(y.y, inv2nv, out + BPS / 2);
  }
}

// y / h (lte_receiver.py:154-180 divides by H + 1e-6): multiply by the conjugate
// over |h|^2; f32 relative error a few ulp (no over/underflow at these magnitudes).
__device__ __forceinline__ float2 zf_div(float2 y, float2 h) {
  const float r = 1.0f / (h.x * h.x + h.y * h.y);
  return make_float2((y.x * h.x + y.y * h.y) * r, (y.y * h.x - y.x * h.y) * r);
}

// Noise-add for one OFDM symbol into LDS, one Philox call per pair of
// samples (sample n uses half (n&1) of counter n>>1 -- same draws as
// load_symbol_noisy, at half the generator cost).
__device__ __forceinline__ void load_symbol_noisy2(float2* buf, const float2* __restrict__ yf, int N, int cp, int l,
                                                   float sigma, uint64_t seed, uint64_t frame, int rx,
                                                   const float* __restrict__ zf, int L, int tid, int T) {
  const int off = l * (N + cp) + cp;
  if (zf) {
    load_symbol_noisy(buf, yf, N, cp, l, sigma, seed, frame, rx, zf, L, tid, T);
    return;
  }
  const int p0 = off >> 1, p1 = (off + N - 1) >> 1;
  // every sample load of this thread is issued before the first Philox call
  // (the loop was latency bound with one pair in flight); T = N/8 threads
  // cover the N/2 (+1) pairs in at most 5 rounds
  constexpr int MAXR = 5;
  float2 va[MAXR], vb[MAXR];
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int p = p0 + tid + i * T, n0 = 2 * p;
    va[i] = (p <= p1 && n0 >= off) ? yf[n0] : make_float2(0.f, 0.f);
    vb[i] = (p <= p1 && n0 + 1 < off + N) ? yf[n0 + 1] : make_float2(0.f, 0.f);
  }
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int p = p0 + tid + i * T, n0 = 2 * p;
    if (p > p1) break;
    const u32x4 r = rng4(seed, frame, RNG_STREAM_NOISE + (uint32_t)rx, (uint32_t)p);
    if (n0 >= off) {
      const float2 z = box_muller(r.x, r.y);
      buf[n0 - off] = make_float2(va[i].x + sigma * z.x, va[i].y + sigma * z.y);
    }
    if (n0 + 1 < off + N) {
      const float2 z = box_muller(r.z, r.w);
      buf[n0 + 1 - off] = make_float2(vb[i].x + sigma * z.x, vb[i].y + sigma * z.y);
    }
  }
}

// SC-FDM DFT (DFTPrecodifier, core/dft_precoding.py:43-90: X_k = sum_n x_n
// exp(-2 pi i k n / M) / sqrt(M), M = Nd) in place on buf[0, M), buf[M, N)
// zero on entry.  Bluestein: X_k = conj(w_k) sum_n (x_n conj(w_n)) w_{k-n},
// w_m = exp(i pi m^2 / M), the convolution by N-point LDS FFTs (N >= 2M - 1
// since Nd < N/2).  The inverse (IDFTDecodifier) is conj(DFT(conj(x))).  All
// threads of the block call it; it begins and ends with a barrier.
__device__ __forceinline__ void dft_bluestein(float2* buf, const Grid& g, int tid, int T, bool active) {
  __syncthreads();
  if (active)
    for (int n = tid; n < g.Nd; n += T) buf[n] = cmul(buf[n], g.chirp[n]);
  __syncthreads();
  fft_lds<false>(buf, g.N, g.log2N, g.tw, tid, active);
  if (active)
    for (int k = tid; k < g.N; k += T) buf[k] = cmul(buf[k], g.bhat[k]);
  __syncthreads();
  fft_lds<true>(buf, g.N, g.log2N, g.tw, tid, active);
  if (active)
    for (int k = tid; k < g.Nd; k += T) buf[k] = cmul(buf[k], g.chirp[k]);
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

}  // namespace lte
