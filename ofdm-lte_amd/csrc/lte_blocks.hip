// Kernels behind the stage entries of the reference's building-block classes
// (lte_capi.hip: lte_qam_map_host64, lte_chest_host64, lte_zf_host64), float64
// with NumPy's operation order and no contraction into FMAs, so the results
// are the reference's to the last bit wherever NumPy's own operations are
// correctly rounded:
//   QAMModulator.bits_to_symbols      core/modulator.py:61-88
//   LTEChannelEstimator.estimate_channel + _interpolate_channel
//                                     core/lte_receiver.py:40-133
//   LTEEqualizerZF.equalize           core/lte_receiver.py:154-180
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include "lte_common.h"
#include "lte_dev.h"
#include "lte_internal.h"

namespace lte {

constexpr int BWG = 256;

// bits [n][BPS] (0 / 1 bytes, MSB first) -> the constellation point of that
// natural-binary index (the chains' qam_point: level * (1 / S), NumPy's
// complex / real divide)
template <int BPS>
__global__ __launch_bounds__(BWG) void k_qam_map_stage(int64_t n, const uint8_t* __restrict__ bits,
                                                       double2* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * BWG + threadIdx.x;
  if (i >= n) return;
  int idx = 0;
#pragma unroll
  for (int m = 0; m < BPS; ++m) idx = (idx << 1) | (bits[i * BPS + m] & 1);
  out[i] = qam_point<BPS, double>(idx);
}

int launch_qam_map(hipStream_t s, int bps, int64_t n, const uint8_t* bits, double2* out) {
  if (n <= 0) return 0;
  const dim3 grid((unsigned)((n + BWG - 1) / BWG));
  if (bps == 2) hipLaunchKernelGGL(k_qam_map_stage<2>, grid, dim3(BWG), 0, s, n, bits, out);
  else if (bps == 4) hipLaunchKernelGGL(k_qam_map_stage<4>, grid, dim3(BWG), 0, s, n, bits, out);
  else if (bps == 6) hipLaunchKernelGGL(k_qam_map_stage<6>, grid, dim3(BWG), 0, s, n, bits, out);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// QAMModulator.symbols_to_bits / LTEReceiver._detect_symbols exactly as the
// reference decides (core/modulator.py:103-110): distances np.abs(c - y) to
// every constellation point, NumPy's complex absolute (its SIMD loop:
// larger * sqrt(fma(smaller / larger, smaller / larger, 1)), bit-identical on
// the FMA hosts the goldens came from, tests/golden/make_golden_r6.py), and
// np.argmin (the first of equal minima).  The chains' per-axis slicer
// (hard_index) agrees everywhere except on exact decision boundaries.
__device__ __forceinline__ double np_cabs(double re, double im) {
  re = fabs(re);
  im = fabs(im);
  const double larger = fmax(re, im), smaller = fmin(im, re);
  const double ratio = larger == 0.0 ? 0.0 : smaller / larger;
  return sqrt(__builtin_fma(ratio, ratio, 1.0)) * larger;
}

template <int BPS>
__global__ __launch_bounds__(BWG) void k_hard_argmin_stage(int64_t n, const double2* __restrict__ y,
                                                           uint8_t* __restrict__ bits) {
  const int64_t i = (int64_t)blockIdx.x * BWG + threadIdx.x;
  if (i >= n) return;
  const double2 v = y[i];
  int best = 0;
  double bd = 0.0;
#pragma unroll 4
  for (int m = 0; m < (1 << BPS); ++m) {
    const double2 c = qam_point<BPS, double>(m);
    const double d = np_cabs(c.x - v.x, c.y - v.y);
    if (m == 0 || d < bd) {
      bd = d;
      best = m;
    }
  }
#pragma unroll
  for (int b = 0; b < BPS; ++b) bits[i * BPS + b] = (uint8_t)((best >> (BPS - 1 - b)) & 1);
}

int launch_hard_argmin(hipStream_t s, int bps, int64_t n, const double2* y, uint8_t* bits) {
  if (n <= 0) return 0;
  const dim3 grid((unsigned)((n + BWG - 1) / BWG));
  if (bps == 2) hipLaunchKernelGGL(k_hard_argmin_stage<2>, grid, dim3(BWG), 0, s, n, y, bits);
  else if (bps == 4) hipLaunchKernelGGL(k_hard_argmin_stage<4>, grid, dim3(BWG), 0, s, n, y, bits);
  else if (bps == 6) hipLaunchKernelGGL(k_hard_argmin_stage<6>, grid, dim3(BWG), 0, s, n, y, bits);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// NumPy's pairwise summation (numpy/_core/src/umath/loops_utils.h.src
// pairwise_sum, which np.add.reduce / np.mean use on a contiguous float64
// array): under 8 terms a plain loop from -0.0, up to 128 eight accumulators
// combined as ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) plus the
// tail, above that sum(first n2) + sum(rest) with n2 = n / 2 rounded down to
// a multiple of 8 -- here as an explicit post-order stack.  v(i) yields term
// i.  (Checked against np.add.reduce for n = 1..300, 1000, 4097: identical.)
template <class F>
__device__ double np_pairwise_sum(int n, F v) {
  struct Node {
    int lo, n;
    bool split;
  };
  Node st[40];
  double vals[40];
  int top = 0, nv = 0;
  st[top++] = Node{0, n, false};
  while (top) {
    const Node nd = st[top - 1];
    if (nd.n <= 128) {
      double r;
      if (nd.n < 8) {
        r = -0.0;
        for (int i = 0; i < nd.n; ++i) r += v(nd.lo + i);
      } else {
        double a[8];
        for (int j = 0; j < 8; ++j) a[j] = v(nd.lo + j);
        int i = 8;
        for (; i < nd.n - (nd.n % 8); i += 8)
          for (int j = 0; j < 8; ++j) a[j] += v(nd.lo + i + j);
        r = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
        for (; i < nd.n; ++i) r += v(nd.lo + i);
      }
      vals[nv++] = r;
      --top;
    } else if (!nd.split) {
      st[top - 1].split = true;
      int n2 = nd.n / 2;
      n2 -= n2 % 8;
      st[top++] = Node{nd.lo + n2, nd.n - n2, false};   // right: evaluated second
      st[top++] = Node{nd.lo, n2, false};               // left: on top, evaluated first
    } else {
      const double r = vals[nv - 2] + vals[nv - 1];
      nv -= 2;
      vals[nv++] = r;
      --top;
    }
  }
  return vals[0];
}

// One block per received grid: the LS estimates Y[p] / X[p] at the pilots
// (NumPy's complex divide, cdiv), their statistics (mean |Y_p|^2 and mean
// |Y_p - X_p|^2, np.abs = hypot, np.mean = pairwise sum / n), then every
// subcarrier from np.linspace between consecutive pilots (step = delta * (1 /
// div), value = j * step + start, the end point = the pilot itself) with the
// edges held.  pidx ascending.
__global__ __launch_bounds__(BWG) void k_chest_stage(int N, int P, const int32_t* __restrict__ pidx,
                                                     const double2* __restrict__ known,
                                                     const double2* __restrict__ Y, double2* __restrict__ H,
                                                     double2* __restrict__ hp_out, double* __restrict__ stats) {
  extern __shared__ double2 hp[];   // [P]
  const int64_t b = blockIdx.x;
  const double2* y = Y + b * N;
  for (int p = threadIdx.x; p < P; p += BWG) {
    const double2 r = cdiv(y[pidx[p]], known[p]);
    hp[p] = r;
    if (hp_out) hp_out[b * P + p] = r;
  }
  __syncthreads();
  if (stats && threadIdx.x == 0) {
    const double pp = np_pairwise_sum(P, [&](int p) {
      const double2 v = y[pidx[p]];
      const double a = hypot(v.x, v.y);
      return a * a;
    });
    const double en = np_pairwise_sum(P, [&](int p) {
      const double2 v = y[pidx[p]], x = known[p];
      const double a = hypot(v.x - x.x, v.y - x.y);
      return a * a;
    });
    stats[2 * b] = pp / (double)P;
    stats[2 * b + 1] = en / (double)P;
  }
  double2* h = H + b * N;
  for (int k = threadIdx.x; k < N; k += BWG) {
    double2 v;
    if (k <= pidx[0]) {
      v = hp[0];
    } else if (k >= pidx[P - 1]) {
      v = hp[P - 1];
    } else {
      int lo = 0, hi = P - 1;   // largest i with pidx[i] <= k
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (pidx[mid] <= k) lo = mid;
        else hi = mid;
      }
      const int j = k - pidx[lo];
      if (j == 0) {
        v = hp[lo];
      } else {
        const double ig = 1.0 / (double)(pidx[lo + 1] - pidx[lo]);
        const double2 v0 = hp[lo], v1 = hp[lo + 1];
        const double sx = (v1.x - v0.x) * ig, sy = (v1.y - v0.y) * ig;
        v = make_double2((double)j * sx + v0.x, (double)j * sy + v0.y);
      }
    }
    h[k] = v;
  }
}

int launch_chest(hipStream_t s, int N, int P, const int32_t* pidx, const double2* known, int64_t batch,
                 const double2* Y, double2* H, double2* hp, double* stats) {
  if (batch <= 0) return 0;
  if (P < 1 || P > 4096 || batch > 0x7FFFFFFF) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_chest_stage, dim3((unsigned)batch), dim3(BWG), (size_t)P * sizeof(double2), s, N, P, pidx,
                     known, Y, H, hp, stats);
  return (int)hipGetLastError();
}

// Y / (H + reg): the real regularisation added to the real part, then
// NumPy's complex divide (cdiv)
__global__ __launch_bounds__(BWG) void k_zf_stage(int64_t n, const double2* __restrict__ Y,
                                                  const double2* __restrict__ H, double reg,
                                                  double2* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * BWG + threadIdx.x;
  if (i >= n) return;
  const double2 h = H[i];
  out[i] = cdiv(Y[i], make_double2(h.x + reg, h.y + 0.0));
}

int launch_zf(hipStream_t s, int64_t n, const double2* Y, const double2* H, double reg, double2* out) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_zf_stage, dim3((unsigned)((n + BWG - 1) / BWG)), dim3(BWG), 0, s, n, Y, H, reg, out);
  return (int)hipGetLastError();
}

// CRC of any length <= 31 by MSB-first long division of the message followed
// by len zero bits, zero initial register (crc.py:89-134, _calculate_crc),
// one lane: the CRCs the chains do not use (CRC-16, crc.py:187-209) -- the
// chains' CRC-24A / 24B run in k_payload / k_crc_count
__global__ void k_crc_serial(int64_t n, const uint8_t* __restrict__ bits, uint32_t poly_low, int len,
                             uint32_t* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint32_t mask = (1u << len) - 1u;
  uint32_t r = 0u;
  for (int64_t i = 0; i < n + len; ++i) {
    const uint32_t b = i < n ? (uint32_t)(bits[i] & 1u) : 0u;
    const uint32_t msb = (r >> (len - 1)) & 1u;
    r = ((r << 1) | b) & mask;
    if (msb) r ^= poly_low;
  }
  out[0] = r;
}

int launch_crc_serial(hipStream_t s, int64_t n, const uint8_t* bits, uint32_t poly_low, int len, uint32_t* out) {
  if (len < 1 || len > 31) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_crc_serial, dim3(1), dim3(64), 0, s, n, bits, poly_low, len, out);
  return (int)hipGetLastError();
}

// RSC constituent encoder (turbo_encoder.py:137-211) of one stream, one lane:
// a_k = u_k ^ s1 ^ s2 is the 'systematic' output, parity a_k ^ s0 ^ s2; the
// termination feeds s1 ^ s2 (so its systematic outputs are 0)
__global__ void k_rsc_stage(int64_t n, const uint8_t* __restrict__ u, int term, uint8_t* __restrict__ sys,
                            uint8_t* __restrict__ par) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t s0 = 0, s1 = 0, s2 = 0;
  const int64_t total = n + (term ? 3 : 0);
  for (int64_t i = 0; i < total; ++i) {
    const uint32_t in = i < n ? (uint32_t)(u[i] & 1u) : (s1 ^ s2);
    const uint32_t fb = in ^ s1 ^ s2;
    sys[i] = (uint8_t)fb;
    par[i] = (uint8_t)(fb ^ s0 ^ s2);
    s2 = s1;
    s1 = s0;
    s0 = fb;
  }
}

int launch_rsc(hipStream_t s, int64_t n, const uint8_t* u, int term, uint8_t* sys, uint8_t* par) {
  hipLaunchKernelGGL(k_rsc_stage, dim3(1), dim3(64), 0, s, n, u, term, sys, par);
  return (int)hipGetLastError();
}

}  // namespace lte
