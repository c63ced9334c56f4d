// Beamforming chain for gfx950:
// OFDMSimulator.simulate_beamforming (core/ofdm_core.py:2260-2477).  The
// reference runs it in the frequency domain only (no OFDM modulation): one flat
// channel matrix H [num_rx][num_tx] per frame, CSI feedback picks the rank-1
// codebook PMI (CSIFeedback, core/csi_feedback.py:64-190), the precoder is
// that codebook vector (update_mode 'static') or the MRT vector conj(mean_r
// H) / norm (AdaptiveBeamforming 'adaptive', core/beamforming_precoder.py:
// 35-60, 113-140); per data RE x = W s, y = H x + n, n ~ CN(0, 10^(-SNR/10));
// MRC with H_eff = H W; nearest-point bits.
//   k_bf_setup  one thread per frame: H, PMI, W, H_eff, gain (float64 math)
//   k_bf_data   one thread per (frame, OFDM symbol, data RE): QAM map,
//               precode, channel, noise, MRC, slice, bit errors
// Both are templated on the chain's arithmetic R: double (the default, the
// reference's complex128, with NumPy's own forms where they are cheap:
// |.| as hypot, complex / real as a multiply by the reciprocal, noise
// (z_re, z_im) * sqrt(s2 / 2) with s2 = 10^(-SNR/10)) or float (fast mode).
#include "lte_common.h"
#include "lte_internal.h"
#include "lte_dev.h"

namespace lte {

constexpr int BWG = 256;

// |z|^2 as the reference forms it: np.abs (hypot) squared
__device__ __forceinline__ double abs2_np(double2 z) {
  const double a = hypot(z.x, z.y);
  return a * a;
}

template <class R>
__global__ __launch_bounds__(BWG) void k_bf_setup(int B, int num_tx, int num_rx, int adaptive, int ncb,
                                                  const double* __restrict__ cb, const uint64_t* __restrict__ fid,
                                                  uint64_t seed, const R* __restrict__ inj_h, int64_t inj_stride,
                                                  BfFrameT<R>* __restrict__ fr) {
  constexpr bool F64 = sizeof(R) == 8;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  BfFrameT<R>* f = fr + b;
  // H = (randn + j randn) / sqrt(2) (core/ofdm_core.py:2345-2346): injected or Philox
  double2 H[LTE_BF_MAX_RX][LTE_BF_MAX_TX];
  for (int r = 0; r < num_rx; ++r)
    for (int t = 0; t < num_tx; ++t) {
      const int link = r * num_tx + t;
      double2 h;
      if (inj_h) {
        const R* p = inj_h + (size_t)b * inj_stride + (size_t)link * 2;
        h = make_double2((double)p[0], (double)p[1]);
      } else {
        const u32x4 v = rng4(seed, fid[b], RNG_STREAM_BF + (uint32_t)link, 0u);
        if constexpr (F64) {   // complex / np.sqrt(2): NumPy multiplies by the reciprocal
          const double2 z = gauss2<double>(v.x, v.y);
          h = make_double2(z.x * 0.7071067811865475, z.y * 0.7071067811865475);
        } else {
          const float2 z = box_muller(v.x, v.y);
          h = make_double2(z.x * 0.70710678118654752f, z.y * 0.70710678118654752f);
        }
      }
      H[r][t] = h;
      f->H[r][t] = mkc((R)h.x, (R)h.y);
    }
  // PMI: first codebook vector with the largest ||H w||^2 (LTECodebook.select_best_pmi)
  int pmi = 0;
  double best = -1.0;
  for (int i = 0; i < ncb; ++i) {
    double m = 0.0;
    for (int r = 0; r < num_rx; ++r) {
      double er = 0.0, ei = 0.0;
      for (int t = 0; t < num_tx; ++t) {
        const double hr = H[r][t].x, hi = H[r][t].y;
        const double wr = cb[((size_t)i * num_tx + t) * 2], wi = cb[((size_t)i * num_tx + t) * 2 + 1];
        er += hr * wr - hi * wi;
        ei += hr * wi + hi * wr;
      }
      m += F64 ? abs2_np(make_double2(er, ei)) : er * er + ei * ei;
    }
    if (m > best) { best = m; pmi = i; }
  }
  double wr[LTE_BF_MAX_TX], wi[LTE_BF_MAX_TX];
  if (adaptive) {   // MRT: conj(np.mean(H, axis=0)) / sqrt(sum |.|^2)
    const double inv_rx = 1.0 / (double)num_rx;   // complex / count: the reciprocal (exact for 1, 2, 4, 8)
    double nrm = 0.0;
    for (int t = 0; t < num_tx; ++t) {
      double ar = 0.0, ai = 0.0;
      for (int r = 0; r < num_rx; ++r) { ar += H[r][t].x; ai += H[r][t].y; }
      wr[t] = F64 ? ar * inv_rx : ar / num_rx;
      wi[t] = F64 ? -(ai * inv_rx) : -ai / num_rx;
      nrm += F64 ? abs2_np(make_double2(wr[t], wi[t])) : wr[t] * wr[t] + wi[t] * wi[t];
    }
    const double s = 1.0 / sqrt(nrm);
    for (int t = 0; t < num_tx; ++t) { wr[t] *= s; wi[t] *= s; }
  } else {
    for (int t = 0; t < num_tx; ++t) {
      wr[t] = cb[((size_t)pmi * num_tx + t) * 2];
      wi[t] = cb[((size_t)pmi * num_tx + t) * 2 + 1];
    }
  }
  double pe = 0.0, ph = 0.0;
  for (int r = 0; r < num_rx; ++r) {
    double er = 0.0, ei = 0.0;
    for (int t = 0; t < num_tx; ++t) {
      const double hr = H[r][t].x, hi = H[r][t].y;
      er += hr * wr[t] - hi * wi[t];
      ei += hr * wi[t] + hi * wr[t];
      ph += F64 ? abs2_np(H[r][t]) : hr * hr + hi * hi;
    }
    f->He[r] = mkc((R)er, (R)ei);
    pe += F64 ? abs2_np(make_double2(er, ei)) : er * er + ei * ei;
  }
  for (int t = 0; t < num_tx; ++t) f->W[t] = mkc((R)wr[t], (R)wi[t]);
  f->inv_p = (R)(1.0 / pe);   // comb / np.sum(|He|^2): NumPy multiplies by the reciprocal
  f->pmi = pmi;
  // BeamformingPrecoder.calculate_beamforming_gain: only the adaptive precoder holds W
  f->gain_db = adaptive ? 10.0 * log10(pe / (ph / num_tx)) : 0.0;
}

template <class R, int BPS>
__global__ __launch_bounds__(BWG) void k_bf_data(int B, int n_sym, int Nd, int num_tx, int num_rx,
                                                 const BfFrameT<R>* __restrict__ fr, const R* __restrict__ sigma,
                                                 const uint32_t* __restrict__ pw, int PW, int n_bits,
                                                 const uint64_t* __restrict__ fid, uint64_t seed,
                                                 const R* __restrict__ inj_z, int64_t inj_stride,
                                                 uint32_t* __restrict__ frame_err, cx<R>* __restrict__ cap_syms,
                                                 uint8_t* __restrict__ cap_bits) {
  using V = cx<R>;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t per = (int64_t)n_sym * Nd;
  const bool act = i < (int64_t)B * per;       // tail lanes stay for the wave-level error reduction
  const int b = act ? (int)(i / per) : B - 1;
  const int n = act ? (int)(i - (int64_t)b * per) : 0;     // RE index within the frame (l * Nd + j)
  const BfFrameT<R>* f = fr + b;
  const uint32_t* fb = pw + (size_t)b * PW;
  int idx = 0;
#pragma unroll
  for (int m = 0; m < BPS; ++m) idx = (idx << 1) | (int)getbit(fb, (int64_t)n * BPS + m);
  const V s = qam_point<BPS, R>(idx);
  const R sg = sigma[b];
  const int L = n_sym * Nd;
  V acc = mkc((R)0, (R)0);
  for (int r = 0; r < num_rx; ++r) {
    // y[r] += H[r, t] * x[t], x = W s (W @ d: one product per element)
    V y = mkc((R)0, (R)0);
    for (int t = 0; t < num_tx; ++t) y = cadd(y, cmul(f->H[r][t], cmul(f->W[t], s)));
    V z;
    if (inj_z) {
      const R* zf = inj_z + (size_t)b * inj_stride + (size_t)r * 2 * L;
      z = mkc(zf[n], zf[L + n]);
    } else {
      const u32x4 v = rng4(seed, fid[b], RNG_STREAM_NOISE + (uint32_t)r, (uint32_t)(n >> 1));
      z = (n & 1) ? gauss2<R>(v.z, v.w) : gauss2<R>(v.x, v.y);
    }
    y = mkc(y.x + z.x * sg, y.y + z.y * sg);
    acc = cadd(acc, cmulc(y, f->He[r]));     // conj(He_r) y_r
  }
  const V c = cscale(acc, f->inv_p);
  if (act && cap_syms) cap_syms[(size_t)b * per + n] = c;
  const int hidx = hard_index(c, BPS, (R)qam_norm<BPS>());
  uint32_t errs = 0;
#pragma unroll
  for (int m = 0; m < BPS; ++m) {
    const int64_t pbit = (int64_t)n * BPS + m;
    if (act && pbit < n_bits) {
      const uint32_t bit = (hidx >> (BPS - 1 - m)) & 1;
      errs += bit ^ getbit(fb, pbit);
      if (cap_bits) cap_bits[(size_t)b * n_bits + pbit] = (uint8_t)bit;
    }
  }
  frame_err_add(frame_err, b, errs);
}

template <class R>
int launch_bf(hipStream_t s, int B, int n_sym, int Nd, int bps, int num_tx, int num_rx, int adaptive, int ncb,
              const double* cb, const uint64_t* fid, uint64_t seed, const R* inj_h, int64_t inj_h_stride,
              BfFrameT<R>* fr, const R* sigma, const uint32_t* pw, int PW, int n_bits, const R* inj_z,
              int64_t inj_z_stride, uint32_t* frame_err, cx<R>* cap_syms, uint8_t* cap_bits) {
  if (num_tx < 1 || num_tx > LTE_BF_MAX_TX || num_rx < 1 || num_rx > LTE_BF_MAX_RX) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_bf_setup<R>, dim3((B + BWG - 1) / BWG), dim3(BWG), 0, s, B, num_tx, num_rx, adaptive, ncb, cb,
                     fid, seed, inj_h, inj_h_stride, fr);
  const int64_t n = (int64_t)B * n_sym * Nd;
  const dim3 grid((unsigned)((n + BWG - 1) / BWG));
#define LTE_BFD(B_)                                                                                                \
  hipLaunchKernelGGL((k_bf_data<R, B_>), grid, dim3(BWG), 0, s, B, n_sym, Nd, num_tx, num_rx, fr, sigma, pw, PW,  \
                     n_bits, fid, seed, inj_z, inj_z_stride, frame_err, cap_syms, cap_bits)
  if (bps == 2) LTE_BFD(2); else if (bps == 4) LTE_BFD(4); else LTE_BFD(6);
#undef LTE_BFD
  return (int)hipGetLastError();
}

template int launch_bf<float>(hipStream_t, int, int, int, int, int, int, int, int, const double*, const uint64_t*,
                              uint64_t, const float*, int64_t, BfFrameT<float>*, const float*, const uint32_t*, int,
                              int, const float*, int64_t, uint32_t*, float2*, uint8_t*);
template int launch_bf<double>(hipStream_t, int, int, int, int, int, int, int, int, const double*, const uint64_t*,
                               uint64_t, const double*, int64_t, BfFrameT<double>*, const double*, const uint32_t*,
                               int, int, const double*, int64_t, uint32_t*, double2*, uint8_t*);

}  // namespace lte
