// Shared device helpers for the gfx950 LTE PHY kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "lte_bm_tables.h"

#define LTE_NEG_BIG (-1.0e30f)

// ---------------------------------------------------------------- precision
// The signal chains compute in R = double (the default: the reference is
// float64 / complex128 throughout) or R = float (opt-in fast mode).  cx<R> is
// the matching complex type (float2 / double2), re_t<V> a complex's real type.
template <class R> struct cx_of;
template <> struct cx_of<float> { using type = float2; };
template <> struct cx_of<double> { using type = double2; };
template <class R> using cx = typename cx_of<R>::type;
template <class V> struct re_of;
template <> struct re_of<float2> { using type = float; };
template <> struct re_of<double2> { using type = double; };
template <class V> using re_t = typename re_of<V>::type;
__host__ __device__ __forceinline__ float2 mkc(float a, float b) { return make_float2(a, b); }
__host__ __device__ __forceinline__ double2 mkc(double a, double b) { return make_double2(a, b); }

// ---------------------------------------------------------------- RNG
// Philox4x32-10 (counter-based, stateless): every random number is a pure
// function of (seed, frame id, stream, index), so results do not depend on
// how frames are sharded over workgroups or GPUs.
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox4x32(u32x4 c, uint32_t k0, uint32_t k1) {
  // each round's two 32x32 -> 64-bit products as one v_mad_u64_u32 apiece
  // (1.23x the draws/s of separate v_mul_lo_u32 + v_mul_hi_u32 halves,
  // scripts/philox_rate_bench.hip)
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    c = {hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

enum : uint32_t {
  RNG_STREAM_BITS = 1u,
  RNG_STREAM_FADE = 0x100u,   // + rx*64 + tx
  RNG_STREAM_NOISE = 0x10000u, // + rx
  RNG_STREAM_MIMO_FADE = 0x20000u,  // + link * n_paths + path, link = rx * num_tx + tx
  RNG_STREAM_MIMO_LINK = 0x30000u,  // + link : link noise (transmit_mimo) / flat link gain (spatial)
  RNG_STREAM_BF = 0x40000u,         // + rx*num_tx + tx : beamforming flat channel H
};

__device__ __forceinline__ u32x4 rng4(uint64_t seed, uint64_t frame, uint32_t stream, uint32_t idx) {
  return philox4x32({idx, stream, (uint32_t)frame, (uint32_t)(frame >> 32)},
                    (uint32_t)seed, (uint32_t)(seed >> 32));
}

// uniform in (0, 1]
__device__ __forceinline__ float u01(uint32_t v) { return ((v >> 8) + 1u) * (1.0f / 16777216.0f); }

// two standard normals from two uniforms (Box-Muller)
__device__ __forceinline__ float2 box_muller(uint32_t a, uint32_t b) {
  const float r = sqrtf(-2.0f * __logf(u01(a)));
  float s, c;
  __sincosf(6.2831853071795864f * u01(b), &s, &c);
  return make_float2(r * c, r * s);
}

// float64 Box-Muller for the f64 chain's synthetic noise: 32-bit uniforms in
// (0, 1), float64 log / sqrt / sincos (the arithmetic type of the chain)
__device__ __forceinline__ double2 box_muller64(uint32_t a, uint32_t b) {
  const double u = ((double)a + 0.5) * 2.3283064365386962890625e-10;   // 2^-32
  const double v = ((double)b + 0.5) * 2.3283064365386962890625e-10;
  const double r = sqrt(-2.0 * log(u));
  double s, c;
  sincospi(2.0 * v, &s, &c);
  return make_double2(r * c, r * s);
}
// Table-driven float64 Box-Muller: the same (a, b) -> (r cos t, r sin t) as
// box_muller64 on the same uniforms, with ln u and the angle's sin / cos from
// correctly rounded float64 tables (lte_bm_tables.h) plus short polynomials
// on |x| < 2^-8: about 40 % of the VALU work of OCML's log and sincospi, and
// within a few float64 ulps of them (scripts/rx_parts_bench.hip measures both).
//  ln u, u = (a + 0.5) 2^-32: u = 2^e m, m in [1, 2); m = c_i (1 + r) with c_i
//  the centre of m's 1/128 bucket, ln u = e ln 2 + ln c_i + log1p(r); for u in
//  [1/2, 1) (e = -1) ln(c_i / 2) + log1p(r) from its own correctly rounded
//  table (BM_LH: -ln 2 + ln c_i cancels there, which cost up to 81 ulp of the
//  radius near u = 1 - 2^-8, tests/test_gpu_philox.py); for u in [1 - 2^-8, 1)
//  log1p(-(1 - u)) directly (keeps the relative precision near 1).
//  angle 2 pi (b + 0.5) 2^-32 = 2 pi (i + 0.5) / 256 + x, |x| < 2 pi 2^-9.
__device__ __forceinline__ double log1p_small(double r) {   // |r| <= 2^-8, error < 2^-60
  return r * (1.0 + r * (-0.5 + r * (0x1.5555555555555p-2 + r * (-0.25 + r * (0.2 + r * (-0x1.5555555555555p-3 +
                                                                                          r * 0x1.2492492492492p-3))))));
}
#ifndef LTE_BM_SELECT   // 0: the three ln u cases as branches (A/B)
#define LTE_BM_SELECT 1
#endif
// Where box_muller64t reads its tables: BmTabC the __constant__ arrays (vector
// gathers through the L1 / L2), BmTabL copies of them in LDS (bm_tables_lds).
struct BmTabC {
  __device__ __forceinline__ double2 sc(int i) const { return BM_SC[i]; }
  __device__ __forceinline__ double2 lg(int i) const { return BM_LG[i]; }
  __device__ __forceinline__ double lh(int i) const { return BM_LH[i]; }
};
struct BmTabL {
  const double2* s;
  const double2* g;
  const double* h;
  __device__ __forceinline__ double2 sc(int i) const { return s[i]; }
  __device__ __forceinline__ double2 lg(int i) const { return g[i]; }
  __device__ __forceinline__ double lh(int i) const { return h[i]; }
};
constexpr int BM_LDS_BYTES = 256 * 16 + 128 * 16 + 128 * 8;   // 7 KB
// copy the tables into lds (BM_LDS_BYTES, 16-B aligned) by nt threads; the
// caller's barrier must follow before the first draw
__device__ __forceinline__ BmTabL bm_tables_lds(void* lds, int tid, int nt) {
  double2* s = reinterpret_cast<double2*>(lds);
  double2* g = s + 256;
  double* h = reinterpret_cast<double*>(g + 128);
  for (int i = tid; i < 256; i += nt) s[i] = BM_SC[i];
  for (int i = tid; i < 128; i += nt) {
    g[i] = BM_LG[i];
    h[i] = BM_LH[i];
  }
  return BmTabL{s, g, h};
}
template <class TB = BmTabC>
__device__ __forceinline__ double ln_u32(uint32_t a, const TB& tb = TB{}) {
  const double x = (double)a + 0.5;   // exact
  const uint64_t bx = (uint64_t)__double_as_longlong(x);
  const int e = (int)(bx >> 52) - 1023 - 32;
  const int i = (int)(bx >> 45) & 127;
  const double m = __longlong_as_double((long long)((bx & 0xFFFFFFFFFFFFFull) | 0x3FF0000000000000ull));
  const double c = 1.0 + ((double)i + 0.5) * 0.0078125;   // exact
  const double2 t = tb.lg(i);
  const bool near1 = a >= 0xFF000000u;
  const double d = ((double)(0xFFFFFFFFu - a) + 0.5) * 0x1p-32;   // 1 - u, exact
  const double r = near1 ? -d : (m - c) * t.x;                    // m - c exact
  const double p = log1p_small(r);
  const double ln2_hi = 0x1.62e42fee00000p-1, ln2_lo = 0x1.a39ef35793c76p-33;
  // the three cases as selects, not branches: a wave's lanes split about
  // evenly between u < 1/2 and u >= 1/2, so branches ran both paths anyway
#if LTE_BM_SELECT
  const double lh = tb.lh(i) + p;
  const double gen = (double)e * ln2_hi + (t.y + ((double)e * ln2_lo + p));
  return near1 ? p : (e == -1 ? lh : gen);
#else
  if (near1) return p;
  if (e == -1) return tb.lh(i) + p;
  return (double)e * ln2_hi + (t.y + ((double)e * ln2_lo + p));
#endif
}
// sqrt for x in [2^-767, 2^1023): the steps of LLVM's correctly rounded
// float64 sqrt expansion for gfx950 (v_rsq_f64 + two Newton-Raphson /
// Goldschmidt corrections), without its range scaling (two ldexp) and its
// zero / inf / nan selects, so the same bits on that range.  The radius
// argument -2 ln u of box_muller64t lies in [2.3e-10, 46].
__device__ __forceinline__ double sqrt_pos(double x) {
  double g = x * __builtin_amdgcn_rsq(x);
  double h = __builtin_amdgcn_rsq(x) * 0.5;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  return __builtin_fma(d, h, g);
}
template <class TB = BmTabC>
__device__ __forceinline__ double2 box_muller64t(uint32_t a, uint32_t b, const TB& tb = TB{}) {
  const double r = sqrt_pos(-2.0 * ln_u32(a, tb));
  const double2 T = tb.sc(b >> 24);
  const double x = ((double)((int)(b & 0xFFFFFFu) - 0x800000) + 0.5) * 0x1p-32 * 0x1.921fb54442d18p+2;
  const double x2 = x * x;
  const double sx = x + x * x2 * (-0x1.5555555555555p-3 + x2 * (0x1.1111111111111p-7 + x2 * -0x1.a01a01a01a01ap-13));
  const double cm1 = x2 * (-0.5 + x2 * (0x1.5555555555555p-5 + x2 * -0x1.6c16c16c16c17p-10));   // cos x - 1
  // the table value plus a small correction, rounded once: |error| <= 2^-53
  // per component (cos x formed as 1 + cm1 first doubled it)
  const double c = T.x + (T.x * cm1 - T.y * sx), s = T.y + (T.y * cm1 + T.x * sx);
  return make_double2(r * c, r * s);
}
template <class R> __device__ __forceinline__ cx<R> gauss2(uint32_t a, uint32_t b);
template <> __device__ __forceinline__ float2 gauss2<float>(uint32_t a, uint32_t b) { return box_muller(a, b); }
template <> __device__ __forceinline__ double2 gauss2<double>(uint32_t a, uint32_t b) { return box_muller64t(a, b); }
// the same draws with the float64 tables read through tb (float32: no tables)
template <class R, class TB> __device__ __forceinline__ cx<R> gauss2t(uint32_t a, uint32_t b, const TB& tb) {
  if constexpr (sizeof(R) == 8) return box_muller64t(a, b, tb);
  else return box_muller(a, b);
}

// ---------------------------------------------------------------- complex
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cmulc(float2 a, float2 b) {  // a * conj(b)
  return make_float2(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y);
}
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 cmulc(double2 a, double2 b) {
  return make_double2(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y);
}
__device__ __forceinline__ double2 cscale(double2 a, double s) { return make_double2(a.x * s, a.y * s); }
// Complex division with Smith's scaling (the algorithm NumPy's complex divide uses).
__device__ __forceinline__ float2 cdiv(float2 a, float2 b) {
  if (fabsf(b.x) >= fabsf(b.y)) {
    if (b.x == 0.0f && b.y == 0.0f) return make_float2(a.x / b.x, a.y / b.x);
    const float rat = b.y / b.x, scl = 1.0f / (b.x + b.y * rat);
    return make_float2((a.x + a.y * rat) * scl, (a.y - a.x * rat) * scl);
  }
  const float rat = b.x / b.y, scl = 1.0f / (b.y + b.x * rat);
  return make_float2((a.x * rat + a.y) * scl, (a.y * rat - a.x) * scl);
}
__device__ __forceinline__ double2 cdiv(double2 a, double2 b) {
  if (fabs(b.x) >= fabs(b.y)) {
    if (b.x == 0.0 && b.y == 0.0) return make_double2(a.x / b.x, a.y / b.x);
    const double rat = b.y / b.x, scl = 1.0 / (b.x + b.y * rat);
    return make_double2((a.x + a.y * rat) * scl, (a.y - a.x * rat) * scl);
  }
  const double rat = b.x / b.y, scl = 1.0 / (b.y + b.x * rat);
  return make_double2((a.x * rat + a.y) * scl, (a.y * rat - a.x) * scl);
}

// ---------------------------------------------------------------- FFT
// Stockham radix-8 complex FFT held in LDS (+ one final radix-4 or radix-2
// pass when log2 N is not a multiple of 3): N = 2048 takes 4 passes.  One
// transform of N points is done by T = N/8 threads (tid in [0,T)), one radix-8
// butterfly per thread per pass, every pass register-staged (read -> barrier
// -> write -> barrier), so several transforms of the same N can share a
// workgroup.  Between passes the data lives in an XOR-swizzled layout
// (fft_sw<V>) that makes the strided Stockham stores and the unit-stride loads
// conflict-free for the element's LDS instructions; the output layout is the
// natural one, the input layout natural or (ISW) swizzled.
// tw[e] = exp(-2*pi*i*e/N), e in [0, N).  V = float2 or double2 (the chain
// precision).
// Unscaled.  N in [128, 2048].  All threads of the workgroup must call it (it
// contains __syncthreads).
template <bool INV, class V>
__device__ __forceinline__ V twid(const V* __restrict__ tw, int e) {
  const V w = tw[e];
  return INV ? mkc(w.x, -w.y) : w;
}

// logical -> physical element index between passes (a bijection on each
// 128-element block).  The bank rules (MI355X_MICROARCH.md, LDS):
// * float2 (8 B): ds_write_b64 serves 16 contiguous lanes per cycle on banks
//   (a/4) mod 32, i.e. element mod 16; ds_read_b64 32 lanes, element mod 32.
//   The radix-8 store 8j + r needs bits 4..6 folded into bits 0..3.
// * double2 (16 B): ds_write_b128 serves 8 contiguous lanes per cycle
//   (element mod 8 must differ), ds_read_b128 the 16-lane groups
//   {0-3, 12-15, 20-27} / {4-11, 16-19, 28-31} (element mod 16).  Folding bits
//   3..5 into bits 0..2 makes the first pass's stride-8 store (lanes j, element
//   8j + r: low bits r ^ (j & 7)) and every unit-stride load conflict-free; the
//   float2 fold above leaves the stride-8 store 2-way and some loads 2-way.
// (scripts/lds_bank_model.py checks both against every pass of N = 128..2048.)
template <class V>
__device__ __forceinline__ int fft_sw(int i) {
  if constexpr (sizeof(V) == 16) return i ^ ((i >> 3) & 7);
  else return i ^ (((i >> 4) & 7) | ((i >> 3) & 8));
}

// x * -j (forward) or x * +j (inverse)
template <bool INV, class V>
__device__ __forceinline__ V mul_mj(V d) {
  return INV ? mkc(-d.y, d.x) : mkc(d.y, -d.x);
}

template <bool INV, class V>
__device__ __forceinline__ void dft4_inplace(V& a0, V& a1, V& a2, V& a3) {
  const V b0 = cadd(a0, a2), b1 = csub(a0, a2), b2 = cadd(a1, a3), b3 = mul_mj<INV>(csub(a1, a3));
  a0 = cadd(b0, b2);
  a2 = csub(b0, b2);
  a1 = cadd(b1, b3);
  a3 = csub(b1, b3);
}

// radix-8 DFT in registers: out[m] = sum_r v[r] W8^(r m)
template <bool INV, class V>
__device__ __forceinline__ void dft8_inplace(V (&v)[8]) {
  using R = re_t<V>;
  dft4_inplace<INV>(v[0], v[2], v[4], v[6]);   // E[m] in v[0,2,4,6]
  dft4_inplace<INV>(v[1], v[3], v[5], v[7]);   // O[m] in v[1,3,5,7]
  const R s = (R)0.70710678118654752440;
  const V o0 = v[1];
  V o1 = v[3], o3 = v[7];
  const V o2 = mul_mj<INV>(v[5]);         // W8^2 = -j (forward)
  if (INV) {                                   // W8^1 = (1+j)/sqrt2, W8^3 = (-1+j)/sqrt2
    o1 = mkc((o1.x - o1.y) * s, (o1.x + o1.y) * s);
    o3 = mkc((-o3.x - o3.y) * s, (o3.x - o3.y) * s);
  } else {                                     // W8^1 = (1-j)/sqrt2, W8^3 = (-1-j)/sqrt2
    o1 = mkc((o1.x + o1.y) * s, (o1.y - o1.x) * s);
    o3 = mkc((o3.y - o3.x) * s, (-o3.x - o3.y) * s);
  }
  const V e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
  v[0] = cadd(e0, o0); v[4] = csub(e0, o0);
  v[1] = cadd(e1, o1); v[5] = csub(e1, o1);
  v[2] = cadd(e2, o2); v[6] = csub(e2, o2);
  v[3] = cadd(e3, o3); v[7] = csub(e3, o3);
}

// NC > 0: a kernel instance for one transform size (NC = N): pass count,
// strides, swizzle predicates and twiddle strides fold and the passes unroll
// (ofdm_tx / rx_data / rx_chest at N = 2048: -2..-15 % time).  NC = 0: runtime N.
// SC: the last pass multiplies its outputs by osc (an output scale folded into
// the final store instead of a separate LDS pass).
// TWR (default for a compile-time N): the twiddles of a butterfly, w^(r ks)
// for r >= 2, formed from w^ks by complex products -- one table load per
// butterfly instead of 7 (radix 8) / 3 (radix 4), a few ulp each; the f64
// N = 2048 transform runs 22 % faster (scripts/rx_parts_bench.hip).
// ISW: the input is in the swizzled layout (written through fft_sw<V> by a
// loader whose natural pattern would conflict, e.g. load_symbol_noisy2's
// stride-2 sample pairs).
template <bool INV, int NC = 0, bool SC = false, bool TWR = (NC > 0), bool ISW = false, class V>
__device__ __forceinline__ void fft_lds(V* buf, int N_, int log2N_, const V* __restrict__ tw, int tid, bool active,
                                        re_t<V> osc = (re_t<V>)1) {
  const int N = NC ? NC : N_;
  const int log2N = NC ? __builtin_ctz(NC) : log2N_;
  const int T = N >> 3;
  const int n8 = log2N / 3, rem = log2N - 3 * n8;
  int Ns = 1, lNs = 0;   // Ns = 8^s
  // the same radix-8 passes twice: unrolled for a compile-time N; as a plain
  // loop otherwise (any other form changes the runtime-N kernels' registers)
  if constexpr (NC > 0) {
#pragma unroll
    for (int s = 0; s < n8; ++s) {
      const bool rsw = s > 0 || ISW, wsw = !(s == n8 - 1 && rem == 0);
      V v[8];
      const int j = tid;
      if (active) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int i = j + r * T;
          v[r] = buf[rsw ? fft_sw<V>(i) : i];
        }
        if (s > 0) {
          const int ks = (j & (Ns - 1)) * (N >> (lNs + 3));   // k * N / (8 Ns)
          if constexpr (TWR) {
            V w[8];
            w[1] = twid<INV>(tw, ks);
            w[2] = cmul(w[1], w[1]);
            w[3] = cmul(w[2], w[1]);
            w[4] = cmul(w[2], w[2]);
            w[5] = cmul(w[4], w[1]);
            w[6] = cmul(w[3], w[3]);
            w[7] = cmul(w[4], w[3]);
#pragma unroll
            for (int r = 1; r < 8; ++r) v[r] = cmul(v[r], w[r]);
          } else {
#pragma unroll
            for (int r = 1; r < 8; ++r) v[r] = cmul(v[r], twid<INV>(tw, r * ks));
          }
        }
        dft8_inplace<INV>(v);
      }
      __syncthreads();
      if (active) {
        const int idx = ((j >> lNs) << (lNs + 3)) + (j & (Ns - 1));
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int i = idx + r * Ns;
          buf[wsw ? fft_sw<V>(i) : i] = (SC && !wsw) ? cscale(v[r], osc) : v[r];
        }
      }
      __syncthreads();
      Ns <<= 3;
      lNs += 3;
    }
  } else {
    for (int s = 0; s < n8; ++s) {
      const bool rsw = s > 0 || ISW, wsw = !(s == n8 - 1 && rem == 0);
      V v[8];
      const int j = tid;
      if (active) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int i = j + r * T;
          v[r] = buf[rsw ? fft_sw<V>(i) : i];
        }
        if (s > 0) {
          const int ks = (j & (Ns - 1)) * (N >> (lNs + 3));   // k * N / (8 Ns)
#pragma unroll
          for (int r = 1; r < 8; ++r) v[r] = cmul(v[r], twid<INV>(tw, r * ks));
        }
        dft8_inplace<INV>(v);
      }
      __syncthreads();
      if (active) {
        const int idx = ((j >> lNs) << (lNs + 3)) + (j & (Ns - 1));
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int i = idx + r * Ns;
          buf[wsw ? fft_sw<V>(i) : i] = (SC && !wsw) ? cscale(v[r], osc) : v[r];
        }
      }
      __syncthreads();
      Ns <<= 3;
      lNs += 3;
    }
  }
  if (rem == 2) {   // final radix-4 pass (Ns == N/4): two butterflies per thread
    const int q4 = N >> 2;
    V v[2][4];
    if (active) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int j = tid + q * T;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[q][r] = buf[fft_sw<V>(j + r * q4)];
        if constexpr (TWR) {
          const V w1 = twid<INV>(tw, j), w2 = cmul(w1, w1), w3 = cmul(w2, w1);
          v[q][1] = cmul(v[q][1], w1);
          v[q][2] = cmul(v[q][2], w2);
          v[q][3] = cmul(v[q][3], w3);
        } else {
#pragma unroll
          for (int r = 1; r < 4; ++r) v[q][r] = cmul(v[q][r], twid<INV>(tw, j * r));
        }
        dft4_inplace<INV>(v[q][0], v[q][1], v[q][2], v[q][3]);
      }
    }
    __syncthreads();
    if (active) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int j = tid + q * T;
#pragma unroll
        for (int r = 0; r < 4; ++r) buf[j + r * q4] = SC ? cscale(v[q][r], osc) : v[q][r];
      }
    }
    __syncthreads();
  } else if (rem == 1) {   // final radix-2 pass (Ns == N/2): four butterflies per thread
    const int h = N >> 1;
    V v[4][2];
    if (active) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = tid + q * T;
        const V a = buf[fft_sw<V>(j)], b = cmul(buf[fft_sw<V>(j + h)], twid<INV>(tw, j));
        v[q][0] = cadd(a, b);
        v[q][1] = csub(a, b);
      }
    }
    __syncthreads();
    if (active) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = tid + q * T;
        buf[j] = SC ? cscale(v[q][0], osc) : v[q][0];
        buf[j + h] = SC ? cscale(v[q][1], osc) : v[q][1];
      }
    }
    __syncthreads();
  }
}

// Two transforms of the same compile-time size NC in one sweep (buffers a and
// b, e.g. the two TX grids of an Alamouti symbol): the passes of fft_lds<INV,
// NC, SC, TWR = true> on both, sharing each butterfly's twiddles and the
// barriers (half of them, and twice the independent work between them).
// Outputs identical to two fft_lds calls (the same operations per element).
template <bool INV, int NC, bool SC = false, class V>
__device__ __forceinline__ void fft2_lds(V* a, V* b, const V* __restrict__ tw, int tid, bool active,
                                         re_t<V> osc = (re_t<V>)1) {
  static_assert(NC >= 128, "compile-time N only");
  constexpr int N = NC, log2N = __builtin_ctz(NC), T = N >> 3;
  constexpr int n8 = log2N / 3, rem = log2N - 3 * n8;
  V* bufs[2] = {a, b};
  int Ns = 1, lNs = 0;
#pragma unroll
  for (int s = 0; s < n8; ++s) {
    const bool rsw = s > 0, wsw = !(s == n8 - 1 && rem == 0);
    V v[2][8];
    const int j = tid;
    if (active) {
      V w[8];
      if (s > 0) {
        const int ks = (j & (Ns - 1)) * (N >> (lNs + 3));
        w[1] = twid<INV>(tw, ks);
        w[2] = cmul(w[1], w[1]);
        w[3] = cmul(w[2], w[1]);
        w[4] = cmul(w[2], w[2]);
        w[5] = cmul(w[4], w[1]);
        w[6] = cmul(w[3], w[3]);
        w[7] = cmul(w[4], w[3]);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int i = j + r * T;
          v[u][r] = bufs[u][rsw ? fft_sw<V>(i) : i];
        }
        if (s > 0) {
#pragma unroll
          for (int r = 1; r < 8; ++r) v[u][r] = cmul(v[u][r], w[r]);
        }
        dft8_inplace<INV>(v[u]);
      }
    }
    __syncthreads();
    if (active) {
      const int idx = ((j >> lNs) << (lNs + 3)) + (j & (Ns - 1));
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int i = idx + r * Ns;
          bufs[u][wsw ? fft_sw<V>(i) : i] = (SC && !wsw) ? cscale(v[u][r], osc) : v[u][r];
        }
    }
    __syncthreads();
    Ns <<= 3;
    lNs += 3;
  }
  if constexpr (rem == 2) {   // final radix-4 pass: two butterflies per thread and buffer
    constexpr int q4 = N >> 2;
    V v[2][2][4];
    if (active) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int j = tid + q * T;
        const V w1 = twid<INV>(tw, j), w2 = cmul(w1, w1), w3 = cmul(w2, w1);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[u][q][r] = bufs[u][fft_sw<V>(j + r * q4)];
          v[u][q][1] = cmul(v[u][q][1], w1);
          v[u][q][2] = cmul(v[u][q][2], w2);
          v[u][q][3] = cmul(v[u][q][3], w3);
          dft4_inplace<INV>(v[u][q][0], v[u][q][1], v[u][q][2], v[u][q][3]);
        }
      }
    }
    __syncthreads();
    if (active) {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int j = tid + q * T;
#pragma unroll
          for (int r = 0; r < 4; ++r) bufs[u][j + r * q4] = SC ? cscale(v[u][q][r], osc) : v[u][q][r];
        }
    }
    __syncthreads();
  } else if constexpr (rem == 1) {   // final radix-2 pass
    constexpr int h = N >> 1;
    V v[2][4][2];
    if (active) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = tid + q * T;
        const V w = twid<INV>(tw, j);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const V x0 = bufs[u][fft_sw<V>(j)], x1 = cmul(bufs[u][fft_sw<V>(j + h)], w);
          v[u][q][0] = cadd(x0, x1);
          v[u][q][1] = csub(x0, x1);
        }
      }
    }
    __syncthreads();
    if (active) {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int j = tid + q * T;
          bufs[u][j] = SC ? cscale(v[u][q][0], osc) : v[u][q][0];
          bufs[u][j + h] = SC ? cscale(v[u][q][1], osc) : v[u][q][1];
        }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- CRC-24 algebra
// The LTE CRCs (crc.py:89-184: zero initial register, no reflection, no final
// XOR) are linear over GF(2): crc(M) = M(x) x^24 mod P.  A message split into
// blocks B_0 .. B_{n-1} of lengths l_i therefore has
//   crc(M) = sum_i crc(B_i) * x^(l_{i+1} + ... + l_{n-1})  mod P,
// which lets lanes (or waves) form the CRCs of their blocks independently and
// combine them with a few multiplications.  Appending z zero bits multiplies the
// CRC by x^z, so a message zero-padded to a convenient length is corrected by
// x^(-z) (x is invertible mod P: both LTE polynomials have a constant term).
// poly = P without its x^24 term; all values are 24-bit.
__host__ __device__ __forceinline__ uint32_t gf24_mul(uint32_t a, uint32_t b, uint32_t poly) {
  uint32_t r = 0u;
#pragma unroll
  for (int i = 23; i >= 0; --i) {
    r = ((r << 1) & 0xFFFFFFu) ^ ((r & 0x800000u) ? poly : 0u);   // r * x mod P
    r ^= ((a >> i) & 1u) ? b : 0u;
  }
  return r;
}
// x^e mod P (e >= 0); inv: x^(-e) mod P
__host__ __device__ inline uint32_t gf24_xpow(uint64_t e, uint32_t poly, bool inv = false) {
  uint32_t base = inv ? (((poly ^ 1u) >> 1) | 0x800000u) : 2u;   // x^-1 = (P + 1) / x
  uint32_t r = 1u;
  while (e) {
    if (e & 1u) r = gf24_mul(r, base, poly);
    base = gf24_mul(base, base, poly);
    e >>= 1;
  }
  return r;
}
// one byte of CRC register update through a 256-entry table (crc24_byte_table)
__host__ __device__ __forceinline__ uint32_t crc24_table_entry(uint32_t i, uint32_t poly) {
  uint32_t r = i << 16;
  for (int k = 0; k < 8; ++k) r = (r & 0x800000u) ? (((r << 1) ^ poly) & 0xFFFFFFu) : ((r << 1) & 0xFFFFFFu);
  return r & 0xFFFFFFu;
}
// Slice-by-4 tables T[k][b] = b x^(8k) x^24 mod P (k = 0: the byte table), so
// 32 message bits x update the register c in one step of four independent
// lookups: with v = (c << 8) ^ x, c' = T3[v >> 24] ^ T2[v >> 16] ^ T1[v >> 8] ^
// T0[v] (bytes).  Fill: every thread of the block calls it, then a barrier.
__device__ __forceinline__ void crc24_slice4_fill(uint32_t* T, uint32_t poly) {
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    uint32_t c = crc24_table_entry((uint32_t)i, poly);
    T[i] = c;
#pragma unroll
    for (int k = 1; k < 4; ++k) {   // one more zero byte: c x^8 mod P
      c = ((c << 8) & 0xFFFFFFu) ^ crc24_table_entry(c >> 16, poly);
      T[k * 256 + i] = c;
    }
  }
}
__device__ __forceinline__ uint32_t crc24_slice4(const uint32_t* T, uint32_t c, uint32_t x) {
  const uint32_t v = (c << 8) ^ x;
  return T[768 + (v >> 24)] ^ T[512 + ((v >> 16) & 0xFFu)] ^ T[256 + ((v >> 8) & 0xFFu)] ^ T[v & 0xFFu];
}

// ---------------------------------------------------------------- bits
// Packed bit streams are MSB-first: bit i of a stream lives in word i>>5 at
// bit position 31-(i&31).
__device__ __forceinline__ uint32_t getbit(const uint32_t* __restrict__ w, int64_t i) {
  return (w[i >> 5] >> (31 - (i & 31))) & 1u;
}
// bits [i, i + NB) of an MSB-first stream (NB <= 32), bit i in the result's
// bit NB - 1: one or two word loads instead of NB single-bit loads.  Word
// (i >> 5) + 1 is read only when the bits reach into it and it starts before
// lim (the stream's bit count); bits at or past lim read as 0.
template <int NB>
__device__ __forceinline__ uint32_t getbits(const uint32_t* __restrict__ w, int64_t i, int64_t lim) {
  const int64_t wi = i >> 5;
  const int sh = (int)(i & 31);
  uint64_t v = (uint64_t)w[wi] << 32;
  if (sh + NB > 32 && ((wi + 1) << 5) < lim) v |= w[wi + 1];
  uint32_t r = (uint32_t)(v >> (64 - sh - NB)) & (uint32_t)((1ull << NB) - 1);
  if (i + NB > lim) {
    const int valid = lim > i ? (int)(lim - i) : 0;
    r &= ~(uint32_t)((1ull << (NB - valid)) - 1);
  }
  return r;
}
// mask of the first min(max(lim - i, 0), NB) of NB bits (MSB-first, as getbits)
template <int NB>
__device__ __forceinline__ uint32_t bits_valid(int64_t i, int64_t lim) {
  if (i + NB <= lim) return (uint32_t)((1ull << NB) - 1);
  const int valid = lim > i ? (int)(lim - i) : 0;
  return (uint32_t)((1ull << NB) - 1) & ~(uint32_t)((1ull << (NB - valid)) - 1);
}
