// Wave-private float64 FFT of N = 2048 points (gfx950).
//
// One wave64 owns one transform: 32 complex values per lane in registers, no
// workgroup barrier.  N = 2048 = 32 x 64 (Cooley-Tukey, n = 64 m + l,
// k = k1 + 32 k2):
//   1. lane l holds x[64 m + l] in v[m]; a 32-point DFT over m in registers
//      (4 x radix-8 after 8 x radix-4, constant twiddles), then v[k1] *=
//      W_2048^(l k1);
//   2. the 64-point DFT over l = l' + 32 h starts with its radix-2 step across
//      the lane pair (l', l' + 32): v_permlane32_swap of register pairs
//      (2i, 2i + 1) puts both operands of k1 = 2i + h in lane l' + 32 h, which
//      forms a = x0 + x1 and b = (x0 - x1) W_64^l';
//   3. one wave-local transpose through LDS (real parts, then imaginary parts:
//      2048 doubles in rows padded to 33, 16.5 KB per wave, every ds_write_b64
//      / ds_read_b64 conflict-free) gives lane c = k1 + 32 p the 32 values of
//      its 32-point DFT over l';
//   4. a 32-point DFT over l' in registers: lane c, register q = X[64 q + c].
// Input and output are both in the "lane l, register m <-> element 64 m + l"
// layout, so HBM loads and stores of a natural-order symbol are unit-stride
// (1 KB per wave instruction).
//
// Forward: W = exp(-2 pi i / N); INV: the conjugate twiddles (unscaled).
// tw: the plan's table tw[e] = exp(-2 pi i e / 2048), e in [0, 2048).
// lds: wfft::LDS_DOUBLES doubles (16.5 KB) private to the calling wave.  All 64 lanes must call.
#pragma once
#include "lte_common.h"

namespace wfft {

// cos(2 pi e / 32), e = 0..8, correctly rounded (scripts: Decimal series)
__device__ constexpr double C32[9] = {
    0x1.0000000000000p+0,  0x1.f6297cff75cb0p-1, 0x1.d906bcf328d46p-1, 0x1.a9b66290ea1a3p-1, 0x1.6a09e667f3bcdp-1,
    0x1.1c73b39ae68c8p-1,  0x1.87de2a6aea963p-2, 0x1.8f8b83c69a60bp-3, 0.0};

// v * W_32^E (forward: W = exp(-2 pi i / 32)), E in [0, 32): trivial cases
// without multiplies (e = 0, 8, 16, 24), the rest one complex multiply by a
// constant
template <bool INV, int E>
__device__ __forceinline__ double2 tw32(double2 v) {
  constexpr int e = E & 31;
  if constexpr (e == 0) return v;
  else if constexpr (e == 16) return make_double2(-v.x, -v.y);
  else if constexpr (e == 8) return mul_mj<INV>(v);                    // -j (forward)
  else if constexpr (e == 24) return mul_mj<!INV>(v);                  // +j (forward)
  else {
    // cos(2 pi e / 32), sin(2 pi e / 32) from the first-octant table
    constexpr int q = e >> 3, r = e & 7;   // quadrant, offset
    constexpr double c0 = C32[r], s0 = C32[8 - r];
    // rotate (c0, s0) by q quarter turns: (c, s) of angle 2 pi e / 32
    constexpr double c = q == 0 ? c0 : q == 1 ? -s0 : q == 2 ? -c0 : s0;
    constexpr double s = q == 0 ? s0 : q == 1 ? c0 : q == 2 ? -s0 : -c0;
    // forward multiplies by (c - j s), inverse by (c + j s)
    constexpr double wi = INV ? s : -s;
    return make_double2(v.x * c - v.y * wi, v.x * wi + v.y * c);
  }
}

// 32-point DFT in registers, natural order in and out: v[k] = sum_m v[m] W32^(m k).
// m = 8 a + b, k = c + 4 d: eight DFT-4s over a, twiddles W32^(b c), four
// DFT-8s over b.
template <bool INV>
__device__ __forceinline__ void dft32(double2 (&v)[32]) {
  double2 y[4][8];
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    double2 a0 = v[b], a1 = v[8 + b], a2 = v[16 + b], a3 = v[24 + b];
    dft4_inplace<INV>(a0, a1, a2, a3);
    y[0][b] = a0;
    y[1][b] = a1;
    y[2][b] = a2;
    y[3][b] = a3;
  }
  // twiddles W32^(b c): compile-time exponents
#define WF_TW(c, b) y[c][b] = tw32<INV, (b) * (c)>(y[c][b])
  WF_TW(1, 1); WF_TW(1, 2); WF_TW(1, 3); WF_TW(1, 4); WF_TW(1, 5); WF_TW(1, 6); WF_TW(1, 7);
  WF_TW(2, 1); WF_TW(2, 2); WF_TW(2, 3); WF_TW(2, 4); WF_TW(2, 5); WF_TW(2, 6); WF_TW(2, 7);
  WF_TW(3, 1); WF_TW(3, 2); WF_TW(3, 3); WF_TW(3, 4); WF_TW(3, 5); WF_TW(3, 6); WF_TW(3, 7);
#undef WF_TW
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    dft8_inplace<INV>(y[c]);
#pragma unroll
    for (int d = 0; d < 8; ++d) v[c + 4 * d] = y[c][d];
  }
}

// lanes 32-63 of a <-> lanes 0-31 of b (v_permlane32_swap, one per dword)
__device__ __forceinline__ void swap_halves(double& a, double& b) {
  const uint64_t ua = (uint64_t)__double_as_longlong(a), ub = (uint64_t)__double_as_longlong(b);
  const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)ua, (uint32_t)ub, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(ua >> 32), (uint32_t)(ub >> 32), false, false);
  a = __longlong_as_double((long long)(((uint64_t)hi[0] << 32) | lo[0]));
  b = __longlong_as_double((long long)(((uint64_t)hi[1] << 32) | lo[1]));
}

// the compiler must not move LDS accesses across a wave-local exchange point;
// the hardware keeps one wave's LDS instructions in order
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// LDS slot of (row c, column col): rows padded to 33 doubles, so the step-3
// stores (16 contiguous lanes: one row, 16 consecutive columns) and loads (32
// lanes: 32 consecutive rows, one column) are conflict-free for ds_write_b64 /
// ds_read_b64 (MI355X_MICROARCH.md LDS table), and every access of a lane is
// its base address plus a compile-time offset
constexpr int TROW = 33;
constexpr int LDS_DOUBLES = 64 * TROW;   // per wave: 16.5 KB
__device__ __forceinline__ int tslot(int c, int col) { return c * TROW + col; }

template <bool INV>
__device__ __forceinline__ void fft2048(double2 (&v)[32], double* __restrict__ lds, const double2* __restrict__ tw,
                                        int lane) {
  // 1. 32-point DFTs over m, then W_2048^(l k1) (k1 = a + 8 b: tw[l a] tw[8 l b],
  //    each factor a correctly rounded table value)
  dft32<INV>(v);
  {
    double2 wa[8], wb[4];
#pragma unroll
    for (int a = 1; a < 8; ++a) wa[a] = twid<INV>(tw, lane * a);
#pragma unroll
    for (int b = 1; b < 4; ++b) wb[b] = twid<INV>(tw, 8 * lane * b);
#pragma unroll
    for (int k = 1; k < 32; ++k) {
      const int a = k & 7, b = k >> 3;
      const double2 w = b == 0 ? wa[a] : (a == 0 ? wb[b] : cmul(wa[a], wb[b]));
      v[k] = cmul(v[k], w);
    }
  }
  // 2. radix-2 across the lane pair (l', l' + 32)
  {
    const int lp = lane & 31;
    const double2 w = twid<INV>(tw, 32 * lp);   // W_64^l'
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      swap_halves(v[2 * i].x, v[2 * i + 1].x);
      swap_halves(v[2 * i].y, v[2 * i + 1].y);
      const double2 x0 = v[2 * i], x1 = v[2 * i + 1];
      v[2 * i] = cadd(x0, x1);
      v[2 * i + 1] = cmul(csub(x0, x1), w);
    }
  }
  // 3. transpose: lane (l', h), register 2 i + p holds (k1 = 2 i + h, p, l')
  //    -> row c = k1 + 32 p, column l'; lane c reads its row
  {
    const int lp = lane & 31, h = lane >> 5;
    const int c_me = lane;
#pragma unroll
    for (int part = 0; part < 2; ++part) {
#pragma unroll
      for (int r = 0; r < 32; ++r) {
        const int c = (r & ~1) + h + 32 * (r & 1);
        lds[tslot(c, lp)] = part ? v[r].y : v[r].x;
      }
      wave_lds_fence();
#pragma unroll
      for (int col = 0; col < 32; ++col) {
        const double t = lds[tslot(c_me, col)];
        if (part) v[col].y = t;
        else v[col].x = t;
      }
      wave_lds_fence();
    }
  }
  // 4. 32-point DFTs over l': lane c, register q = X[64 q + c]
  dft32<INV>(v);
}

}  // namespace wfft
