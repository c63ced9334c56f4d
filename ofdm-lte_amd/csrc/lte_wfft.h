// Wave-private float64 FFTs of N = 2048 and N = 1024 points (gfx950).
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


// ---------------------------------------------------------------------------
// N = 1024 = 16 x 64 (config 3's 10 MHz), the same scheme with 16 values per
// lane (n = 64 m + l, k = k1 + 16 k2):
//   1. lane l holds x[64 m + l] in v[m]; a 16-point DFT over m in registers,
//      then v[k1] *= W_1024^(l k1) (k1 = a + 4 b: tw[l a] tw[4 l b]);
//   2. the 64-point DFT over l = l' + 16 a0 + 32 a1 (k2 = c0 + 2 c1 + 4 d)
//      starts with two radix-2 steps across lanes:
//      * over a1: v_permlane32_swap of register pairs (2i, 2i + 1) as in
//        fft2048 -- lane (l' + 16 a0, h) then holds k1 = 2i + h in register
//        2i + c0; times W_4^(a0 c0) (-j forward on the a0 = 1, c0 = 1 values);
//      * over a0: v_permlane16_swap of register pairs (4j + c0, 4j + 2 + c0)
//        -- lane (l', a0', h) then holds k1 = 4j + 2 a0' + h in register
//        4j + c, c = c0 + 2 c1;
//      then times W_64^(l' c);
//   3. one wave-local transpose through LDS (real parts, then imaginary parts;
//      rows padded to 17 doubles, 8.5 KB per wave): lane k1 + 16 c gets the 16
//      values of its 16-point DFT over l';
//   4. a 16-point DFT over l' in registers: lane c, register d = X[64 d + c].
// tw: the plan's table tw[e] = exp(-2 pi i e / 1024), e in [0, 1024).
// lds: wfft::LDS_DOUBLES_1024 doubles private to the calling wave.

// 16-point DFT in registers, natural order in and out (m = 4 a + b,
// k = c + 4 d: four DFT-4s over a, twiddles W16^(b c) = W32^(2 b c), four
// DFT-4s over b)
template <bool INV>
__device__ __forceinline__ void dft16(double2 (&v)[16]) {
  double2 y[4][4];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    double2 a0 = v[b], a1 = v[4 + b], a2 = v[8 + b], a3 = v[12 + b];
    dft4_inplace<INV>(a0, a1, a2, a3);
    y[0][b] = a0;
    y[1][b] = a1;
    y[2][b] = a2;
    y[3][b] = a3;
  }
#define WF16_TW(c, b) y[c][b] = tw32<INV, 2 * (b) * (c)>(y[c][b])
  WF16_TW(1, 1); WF16_TW(1, 2); WF16_TW(1, 3);
  WF16_TW(2, 1); WF16_TW(2, 2); WF16_TW(2, 3);
  WF16_TW(3, 1); WF16_TW(3, 2); WF16_TW(3, 3);
#undef WF16_TW
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    dft4_inplace<INV>(y[c][0], y[c][1], y[c][2], y[c][3]);
#pragma unroll
    for (int d = 0; d < 4; ++d) v[c + 4 * d] = y[c][d];
  }
}

// rows 1 and 3 (lanes 16-31, 48-63) of a <-> rows 0 and 2 of b (v_permlane16_swap)
__device__ __forceinline__ void swap_rows(double& a, double& b) {
  const uint64_t ua = (uint64_t)__double_as_longlong(a), ub = (uint64_t)__double_as_longlong(b);
  const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)ua, (uint32_t)ub, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(ua >> 32), (uint32_t)(ub >> 32), false, false);
  a = __longlong_as_double((long long)(((uint64_t)hi[0] << 32) | lo[0]));
  b = __longlong_as_double((long long)(((uint64_t)hi[1] << 32) | lo[1]));
}

constexpr int TROW16 = 17;
constexpr int LDS_DOUBLES_1024 = 64 * TROW16;   // per wave: 8.5 KB

template <bool INV>
__device__ __forceinline__ void fft1024(double2 (&v)[16], double* __restrict__ lds, const double2* __restrict__ tw,
                                        int lane) {
  // 1. 16-point DFTs over m, then W_1024^(l k1) (k1 = a + 4 b: tw[l a] tw[4 l b],
  //    six table loads in flight instead of fifteen)
  dft16<INV>(v);
  {
    double2 wa[4], wb[4];
#pragma unroll
    for (int a = 1; a < 4; ++a) wa[a] = twid<INV>(tw, lane * a);
#pragma unroll
    for (int b = 1; b < 4; ++b) wb[b] = twid<INV>(tw, 4 * lane * b);
#pragma unroll
    for (int k = 1; k < 16; ++k) {
      const int a = k & 3, b = k >> 2;
      const double2 w = b == 0 ? wa[a] : (a == 0 ? wb[b] : cmul(wa[a], wb[b]));
      v[k] = cmul(v[k], w);
    }
  }
  // 2. radix-2 over a1 (lane halves), W_4^(a0 c0), radix-2 over a0 (row pairs)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    swap_halves(v[2 * i].x, v[2 * i + 1].x);
    swap_halves(v[2 * i].y, v[2 * i + 1].y);
    const double2 x0 = v[2 * i], x1 = v[2 * i + 1];
    v[2 * i] = cadd(x0, x1);
    v[2 * i + 1] = csub(x0, x1);
  }
  if (lane & 16) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[2 * i + 1] = mul_mj<INV>(v[2 * i + 1]);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int c0 = 0; c0 < 2; ++c0) {
      const int r = 4 * j + c0, r2 = r + 2;
      swap_rows(v[r].x, v[r2].x);
      swap_rows(v[r].y, v[r2].y);
      const double2 x0 = v[r], x1 = v[r2];
      v[r] = cadd(x0, x1);
      v[r2] = csub(x0, x1);
    }
  {
    const int lp = lane & 15;
    const double2 w1 = twid<INV>(tw, 16 * lp), w2 = twid<INV>(tw, 32 * lp), w3 = twid<INV>(tw, 48 * lp);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int c = r & 3;
      if (c) v[r] = cmul(v[r], c == 1 ? w1 : (c == 2 ? w2 : w3));
    }
  }
  // 3. transpose: lane (l', a0', h), register 4 j + c -> row k1 + 16 c, column l'
  {
    const int lp = lane & 15, kb = ((lane >> 4) & 1) * 2 + (lane >> 5);
#pragma unroll
    for (int part = 0; part < 2; ++part) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = 4 * (r >> 2) + kb + 16 * (r & 3);
        lds[row * TROW16 + lp] = part ? v[r].y : v[r].x;
      }
      wave_lds_fence();
#pragma unroll
      for (int col = 0; col < 16; ++col) {
        const double t = lds[lane * TROW16 + col];
        if (part) v[col].y = t;
        else v[col].x = t;
      }
      wave_lds_fence();
    }
  }
  // 4. 16-point DFTs over l': lane c, register d = X[64 d + c]
  dft16<INV>(v);
}

}  // namespace wfft
