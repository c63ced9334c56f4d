// Turbo decoder (max-log BCJR, 8-state RSC) for gfx950.
//
// Replaces turbo_decode / LogMAPDecoder (core/channel_coding/turbo_decoder.py:
// 118-450).  Design (DESIGN.md §5 k_turbo):
//  * one lane = one code block; a wave = 64 code blocks of the same K taken
//    from 64 consecutive frames.  All state (8 alpha/beta metrics, window of
//    recomputed alphas) lives in VGPRs -> no cross-lane traffic at all.
//  * batch-innermost layout [row][64 lanes] per (CB slot r, frame group g):
//    every load/store of a step is one 256-B (f32) / 512-B (f64) coalesced
//    row; the QPP index pi(k) is wave-uniform (computed incrementally on the
//    scalar unit) so the interleaved accesses of decoder 2 are whole rows too.
//  * full-length recursion exactly as the reference (no sliding-window
//    approximation): the forward pass stores alpha checkpoints every SW steps,
//    the backward pass recomputes each window from its checkpoint.
//  * two element types (TurboT below):
//    - double (the default, the reference's precision): the reference's
//      unnormalised recursion in the reference's operation order -- alpha /
//      beta start at delta_0 / -inf, gamma = (+-Ls/2 +- Lp/2) +- La/2, the
//      a-posteriori terms (alpha + gamma) + beta (turbo_decoder.py:214-276),
//      every add a separately rounded f64 add -- so decisions and extrinsics
//      are bit-identical to the float64 reference (and to oracle/
//      coding_oracle.c or_turbo_decode, which restates it op for op).
//    - float (opt-in fast mode): metrics normalised to state 0 every step,
//      -1e30 sentinels, a-posteriori terms alpha + (beta + gamma); bit-exact
//      with its C model (coding_oracle.c or_turbo_decode_f32), not with the
//      reference.
#include "lte_common.h"
#include "lte_internal.h"

// the exact log-MAP instance (k_turbo64_logmap, an exactness mode, not a hot
// path) is too large for the requested full unrolls; it runs correctly rolled
#pragma clang diagnostic ignored "-Wpass-failed"

#ifndef LTE_TURBO_SUB
#define LTE_TURBO_SUB 2
#endif
#ifndef LTE_TURBO_HALVES
#define LTE_TURBO_HALVES 2
#endif
#ifndef LTE_TURBO64_SUB
#define LTE_TURBO64_SUB 3   // f64: 24-step super-windows (A/B on MI355X: 2 / 3 / 4 -> 352 / 341 / 377 ms)
#endif
#ifndef LTE_TURBO64_FWD_PF
#define LTE_TURBO64_FWD_PF 0
#endif
#ifndef LTE_TURBO64_HALVES
#define LTE_TURBO64_HALVES 2
#endif

namespace lte {

template <class T> struct TurboT;
template <> struct TurboT<float> {
  static constexpr bool NORM = true;             // normalise to state 0 every step
  static constexpr int CK = TURBO_CK_ROWS_F32;   // checkpointed states 1..7 (state 0 is 0)
  static constexpr int TSUB = LTE_TURBO_SUB;     // 8-step sub-windows per checkpoint
  static constexpr int HALVES = LTE_TURBO_HALVES;
  static constexpr bool FWD_PF = false;
  __device__ static constexpr float neg() { return LTE_NEG_BIG; }
};
template <> struct TurboT<double> {
  static constexpr bool NORM = false;            // the reference's unnormalised metrics
  static constexpr int CK = TURBO_CK_ROWS_F64;   // all 8 states
  static constexpr int TSUB = LTE_TURBO64_SUB;
  static constexpr int HALVES = LTE_TURBO64_HALVES;
  static constexpr bool FWD_PF = LTE_TURBO64_FWD_PF;
  __device__ static constexpr double neg() { return -__builtin_inf(); }
};

__device__ __forceinline__ float vmax(float a, float b) { return fmaxf(a, b); }
__device__ __forceinline__ double vmax(double a, double b) { return fmax(a, b); }

// max* of the recursions: LM = false max-log-MAP (max), LM = true the exact
// log-MAP of set_decoder_mode(False): log_sum_exp (turbo_decoder.py:64-88) --
// -inf operands return the other one, else max + log1p(exp(-|a - b|)) in the
// reference's branch order (float64 only).
template <bool LM, class T>
__device__ __forceinline__ T mstar(T a, T b) {
  if constexpr (!LM) {
    return vmax(a, b);
  } else {
    if (a == -__builtin_inf()) return b;
    if (b == -__builtin_inf()) return a;
    return a > b ? a + log1p(exp(b - a)) : b + log1p(exp(a - b));
  }
}

// gamma for (fb, par, u); c = {g(0,0,0), g(0,0,1), g(0,1,0), g(0,1,1)}.  The
// other four are exact negations (turbo_decoder.py:305-333 sums +/-L/2 terms,
// and round-to-nearest is symmetric: fl(-x - y) = -fl(x + y)).
template <class T>
__device__ __forceinline__ T gsel(const T c[4], int fb, int par, int u) {
  return fb == 0 ? c[par * 2 + u] : -c[(1 - par) * 2 + (1 - u)];
}

// Decoder rows hold LLR/2 (the dematch / host entry points scale by 0.5,
// exact): those halves ARE the +-L/2 metric terms (turbo_decoder.py:316-331
// divides by 2.0), so gamma needs no multiplies and alpha, beta and the
// a-posteriori L are unchanged (LLR units).  gamma = (sys + par) + apr as the
// reference sums it (:333).  The extrinsic is stored halved as (L/2 - La/2) -
// Ls/2, exactly half of (L - La) - Ls (:270; scaling by 2 commutes with
// rounding).
template <class T>
__device__ __forceinline__ void gam(T hs, T hp, T ha, T c[4]) {
  const T sp = hs + hp, sm = hs - hp;
  c[0] = sp + ha;
  c[1] = sp - ha;
  c[2] = sm + ha;
  c[3] = sm - ha;
}

// forward recursion (turbo_decoder.py:227-235: alpha + gamma, max over the
// two predecessors) + the f32 mode's normalisation.
// State s = 4*s0 + 2*s1 + s2; next = 4*fb + 2*s0 + s1, fb = u^s1^s2,
// par = fb^s0^s2.  Predecessors of ns=(f,a,b): (a,b,0) with u=f^b, par=f^a and
// (a,b,1) with u=f^b^1, par=f^a^1.
template <class T, bool LM = false>
__device__ __forceinline__ void fwd(const T a[8], const T c[4], T o[8]) {
#pragma unroll
  for (int ns = 0; ns < 8; ++ns) {
    const int f = ns >> 2, s0 = (ns >> 1) & 1, s1 = ns & 1;
    const T v0 = a[4 * s0 + 2 * s1] + gsel(c, f, f ^ s0, f ^ s1);
    const T v1 = a[4 * s0 + 2 * s1 + 1] + gsel(c, f, f ^ s0 ^ 1, f ^ s1 ^ 1);
    o[ns] = mstar<LM>(v0, v1);
  }
  if constexpr (TurboT<T>::NORM) {
    const T n0 = o[0];
    o[0] = (T)0;
#pragma unroll
    for (int s = 1; s < 8; ++s) o[s] -= n0;
  }
}

// backward recursion only (trellis-termination steps, turbo_decoder.py:
// 238-245): beta(s) = max(beta[next(s,0)] + g(s,0), beta[next(s,1)] + g(s,1)),
// g(s,1) = -g(s,0), next(s,1) = next(s,0) ^ 4.
template <class T, bool LM = false>
__device__ __forceinline__ void bonly(T b[8], const T c[4]) {
  T bn[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int s0 = s >> 2, s1 = (s >> 1) & 1, s2 = s & 1;
    const int fb = s1 ^ s2, par = fb ^ s0 ^ s2, ns = 4 * fb + 2 * s0 + s1;
    const T g = gsel(c, fb, par, 0);
    bn[s] = mstar<LM>(b[ns] + g, b[ns ^ 4] - g);
  }
  if constexpr (TurboT<T>::NORM) {
    const T n0 = bn[0];
    b[0] = (T)0;
#pragma unroll
    for (int s = 1; s < 8; ++s) b[s] = bn[s] - n0;
  } else {
#pragma unroll
    for (int s = 0; s < 8; ++s) b[s] = bn[s];
  }
}

// One backward step streamed over the states: the beta update and the
// a-posteriori LLR max_s(u=0 terms) - max_s(u=1 terms) (turbo_decoder.py:
// 250-266) in one loop.  f64: each term is (alpha + gamma) + beta, the
// reference's order (:257); f32: alpha + (beta + gamma), its C model's order.
// Returns L and advances beta in place.
template <class T, bool LM = false>
__device__ __forceinline__ T bstep(T b[8], const T c[4], const T a[8]) {
  T bn[8], m0 = (T)0, m1 = (T)0;
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int s0 = s >> 2, s1 = (s >> 1) & 1, s2 = s & 1;
    const int fb = s1 ^ s2, par = fb ^ s0 ^ s2, ns = 4 * fb + 2 * s0 + s1;
    const T g = gsel(c, fb, par, 0);
    const T t0 = b[ns] + g, t1 = b[ns ^ 4] - g;
    T u0, u1;
    if constexpr (TurboT<T>::NORM) {
      u0 = a[s] + t0;
      u1 = a[s] + t1;
    } else {
      u0 = (a[s] + g) + b[ns];
      u1 = (a[s] - g) + b[ns ^ 4];
    }
    if (s == 0) {
      m0 = u0;
      m1 = u1;
    } else {
      m0 = mstar<LM>(m0, u0);
      m1 = mstar<LM>(m1, u1);
    }
    bn[s] = mstar<LM>(t0, t1);
  }
  if constexpr (TurboT<T>::NORM) {
    const T n0 = bn[0];
    b[0] = (T)0;
#pragma unroll
    for (int s = 1; s < 8; ++s) b[s] = bn[s] - n0;
  } else {
#pragma unroll
    for (int s = 0; s < 8; ++s) b[s] = bn[s];
  }
  return m0 - m1;
}

__device__ __forceinline__ int modadd(int a, int b, int K) { a += b; return a >= K ? a - K : a; }
__device__ __forceinline__ int modsub(int a, int b, int K) { a -= b; return a < 0 ? a + K : a; }

constexpr int RS = TURBO_RS;   // row stride (elements): 64 lanes
constexpr int TW = 8;          // steps per sub-window (recomputed in halves)

// Buffer-resource row accessor: the 128-bit descriptor (SGPRs) covers one
// wave's block; a row is addressed by a scalar byte offset (soffset) and the
// lane by one shared 32-bit VGPR (voffset = sizeof(T)*lane).  T8/T20 of the
// CDNA guide: no per-load 64-bit vector addresses, no waterfall loops.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* pu = (void*)(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(pu, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

// Cache-policy bits of the decoder's row loads / stores (buffer "aux"; gfx950:
// 1 = sc0, 2 = nt, 16 = sc1).  nt helps only together with the wave-chunked
// layout (TURBO_CH; scripts/turbo_shape_bench.hip).  Same-box A/B
// of k_turbo64 at 65 536 frames: sc0|nt 320-324 ms, nt 322-324, none 339-346
// (chunk 64), nt / sc1|nt / sc0 without chunking no better than none.
#ifndef LTE_TURBO_CPOL
#define LTE_TURBO_CPOL 3
#endif

// RSB: bytes between consecutive rows (TURBO_CH groups of 64 lanes for the
// decoder's block arrays); CP: cache-policy bits
template <class T, int RSB = RS * (int)sizeof(T), int CP = 0>
struct RowPtr {
  __amdgpu_buffer_rsrc_t r;
  int row0;   // first row of this sub-array inside the block
  int voff;   // sizeof(T) * lane (+ the group's slot within its chunk)
  int rstr = 1;   // row stride of the sub-array (2: interleaved LS / LE)
  __device__ __forceinline__ T ld(int row) const {
    const int so = (row0 + row * rstr) * RSB;
    if constexpr (sizeof(T) == 8) {
      return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, voff, so, CP));
    } else {
      return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(r, voff, so, CP));
    }
  }
  __device__ __forceinline__ void st(int row, T v) const {
    const int so = (row0 + row * rstr) * RSB;
    if constexpr (sizeof(T) == 8) {
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), r, voff, so, CP);
    } else {
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, voff, so, CP);
    }
  }
};

// One half-iteration (one constituent decoder pass) for the code block of this lane.
// All pointers are wave-uniform (scalar) bases; `lane` is the only per-lane
// offset, so every access is a buffer load/store with a scalar row offset and
// one shared VGPR lane offset.
// Forward: alpha over the whole block, checkpoint every SW = 8 * TSUB steps
// (f32: states 1..7; f64: all 8).  Backward, per super-window of SW steps:
// load its inputs once into VGPRs, recompute the alphas at each 8-step
// sub-window start from the checkpoint (kept in VGPRs), then sweep the
// sub-windows top-down; each sub-window recomputes its alphas in HALVES
// pieces (the upper piece first from a recomputed start, then the lower), so
// only 8 / HALVES alpha vectors are ever live.  Recomputed alphas are
// bit-identical to the forward pass (same operations, same order).  HBM rows
// per step: 3 input loads x 2 passes + 1 extrinsic store + 2 CK/SW checkpoint
// rows (f32 TSUB = 2: 7.875 rows of 4 B; f64 TSUB = 3: 7.67 rows of 8 B).
// MODE TM_FINAL: the decoder-1 a-posteriori pass that ends a decode; it also
// packs the hard decisions L < 0 MSB-first into `bo` (words [kw][64 lanes]),
// storing each word as the backward sweep reaches its bit 0 (no re-read pass).
template <class T, int MODE, bool LM = false, int CH = TURBO_CH>
__device__ __forceinline__ void half_pass(T* __restrict__ wbase, T* __restrict__ wck, int slot, int lane, int K,
                                          int f1, int f2, bool first, uint32_t* __restrict__ bo = nullptr) {
  using TT = TurboT<T>;
  using DRow = RowPtr<T, RS * CH * (int)sizeof(T), LTE_TURBO_CPOL>;   // the block arrays' rows (CH groups side by side)
  constexpr int TSUB = TT::TSUB, SW = TW * TSUB, CK = TT::CK, CK0 = 8 - CK;   // CK0: first stored state
  constexpr int TH = TW / TT::HALVES;
  // wbase / wck: the group's chunk; slot: the group's place in it (turbo_elem)
  const int vo = (slot * RS + lane) * (int)sizeof(T);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(wbase, (uint32_t)(turbo_rows(K) * CH * RS * sizeof(T)));
  // rows of step k < K: base + k * stride (lte_internal.h trow_*); tails separately
  constexpr int IST = LTE_TURBO_ILV == 3 ? 4 : LTE_TURBO_ILV == 2 ? 3 : LTE_TURBO_ILV == 1 ? 2 : 1;
  constexpr int DEC = (MODE == TM_DEC2) ? 2 : 1;
  const DRow LS{rb, 0, vo, IST};
  const DRow LS1T{rb, (int)trow_ls(K, K), vo};   // decoder 1's systematic tail
  const DRow LP{rb, (int)trow_lp(K, DEC, 0), vo, LTE_TURBO_ILV == 3 ? 4 : (DEC == 1 && LTE_TURBO_ILV == 2) ? 3 : 1};
  const DRow LPT{rb, (int)trow_lp(K, DEC, K), vo};   // parity tail
  const DRow LS2T{rb, (int)trow_ls2t(K, 0), vo};
  const DRow LE{rb, (int)trow_le(K, 0), vo, IST};
  const DRow ck{make_rsrc(wck, (uint32_t)(turbo_nwin(K) * CK * CH * RS * sizeof(T))), 0, vo};
  const int nsub = K / TW;   // every LTE K is a multiple of 8
  const int tf2 = (2 * f2) % K;
  const bool use_la = !first;
  RowPtr<uint32_t> bout{};
  uint32_t acc = 0;
  if (MODE == TM_FINAL) bout = RowPtr<uint32_t>{make_rsrc(bo, (uint32_t)(turbo_kw(K) * RS * 4)), 0, lane * 4};

  // ---------------- forward pass (alpha[0] = delta_0, turbo_decoder.py:214-218)
  T a[8];
  a[0] = (T)0;
#pragma unroll
  for (int s = 1; s < 8; ++s) a[s] = TT::neg();
  int pi = 0, d = (f1 + f2) % K;
  // window w's inputs (pi / d advance in window order)
  auto ldwin = [&](int w, T (&ls)[TW], T (&lp)[TW], T (&la)[TW]) {
#pragma unroll
    for (int j = 0; j < TW; ++j) {
      const int k = w * TW + j;
      const int p = (MODE == TM_DEC2) ? pi : k;
      ls[j] = LS.ld(p);
      lp[j] = LP.ld(k);
      la[j] = use_la ? LE.ld(p) : (T)0;
      if (MODE == TM_DEC2) { pi = modadd(pi, d, K); d = modadd(d, tf2, K); }
    }
  };
  auto stepwin = [&](int w, const T (&ls)[TW], const T (&lp)[TW], const T (&la)[TW]) {
    if (w % TSUB == 0) {
#pragma unroll
      for (int s = CK0; s < 8; ++s) ck.st((w / TSUB) * CK + s - CK0, a[s]);
    }
#pragma unroll
    for (int j = 0; j < TW; ++j) {
      T c[4], o[8];
      gam(ls[j], lp[j], la[j], c);
      fwd<T, LM>(a, c, o);
#pragma unroll
      for (int s = 0; s < 8; ++s) a[s] = o[s];
    }
  };
  if constexpr (TT::FWD_PF) {
    // software-pipelined: window w + 1's loads are in flight while window w
    // is computed (one resident wave per SIMD has no other wave to overlap)
    T x0[TW], y0[TW], z0[TW], x1[TW], y1[TW], z1[TW];
    ldwin(0, x0, y0, z0);
#pragma unroll 1
    for (int w = 0; w < nsub; w += 2) {
      if (w + 1 < nsub) ldwin(w + 1, x1, y1, z1);
      stepwin(w, x0, y0, z0);
      if (w + 1 < nsub) {
        if (w + 2 < nsub) ldwin(w + 2, x0, y0, z0);
        stepwin(w + 1, x1, y1, z1);
      }
    }
  } else {
#pragma unroll 1
    for (int w = 0; w < nsub; ++w) {
      T ls[TW], lp[TW], la[TW];
      ldwin(w, ls, lp, la);
      stepwin(w, ls, lp, la);
    }
  }

  // ---------------- backward pass (beta[K+3] = delta_0, :220-221)
  T b[8];
  b[0] = (T)0;
#pragma unroll
  for (int s = 1; s < 8; ++s) b[s] = TT::neg();
  // trellis-termination steps k = K+2, K+1, K (only beta is needed there;
  // their a priori is 0, turbo_decoder.py:406, 428)
#pragma unroll
  for (int j = 2; j >= 0; --j) {
    const T ls = (MODE == TM_DEC2) ? LS2T.ld(j) : LS1T.ld(j);
    const T lp = LPT.ld(j);
    T c[4];
    gam(ls, lp, (T)0, c);
    bonly<T, LM>(b, c);
  }
  // pi/d are now at k = K (decoder 2); each super-window steps them back to
  // its start, walks forward while loading and back again while storing
  const int nsw = (nsub + TSUB - 1) / TSUB;
#pragma unroll 1
  for (int q = nsw - 1; q >= 0; --q) {
    const int ns = min(TSUB, nsub - q * TSUB);   // sub-windows here (wave-uniform)
    const int k0 = q * SW;
    if (MODE == TM_DEC2) {
#pragma unroll 1
      for (int j = 0; j < ns * TW; ++j) { d = modsub(d, tf2, K); pi = modsub(pi, d, K); }
    }
    T ls[SW], lp[SW], la[SW];
    int pp = pi, dd = d;
#pragma unroll
    for (int m = 0; m < TSUB; ++m) {
      if (m < ns) {
#pragma unroll
        for (int j = 0; j < TW; ++j) {
          const int i = m * TW + j, k = k0 + i;
          const int p = (MODE == TM_DEC2) ? pp : k;
          ls[i] = LS.ld(p);
          lp[i] = LP.ld(k);
          la[i] = use_la ? LE.ld(p) : (T)0;
          if (MODE == TM_DEC2) { pp = modadd(pp, dd, K); dd = modadd(dd, tf2, K); }
        }
      }
    }
    // alpha at every sub-window start: the checkpoint, then forward
    T cks[TSUB][8];
    if (CK0) cks[0][0] = (T)0;
#pragma unroll
    for (int s = CK0; s < 8; ++s) cks[0][s] = ck.ld(q * CK + s - CK0);
#pragma unroll
    for (int m = 1; m < TSUB; ++m) {
#pragma unroll
      for (int s = 0; s < 8; ++s) cks[m][s] = cks[m - 1][s];
      if (m < ns) {
#pragma unroll
        for (int j = 0; j < TW; ++j) {
          const int i = (m - 1) * TW + j;
          T c[4], o[8];
          gam(ls[i], lp[i], la[i], c);
          fwd<T, LM>(cks[m], c, o);
#pragma unroll
          for (int s = 0; s < 8; ++s) cks[m][s] = o[s];
        }
      }
    }
#pragma unroll
    for (int m = TSUB - 1; m >= 0; --m) {
      if (m >= ns) continue;
#pragma unroll
      for (int h = TT::HALVES - 1; h >= 0; --h) {
        // each recompute repeats a chain already run (the lower half: the one
        // the upper half ran from the sub-window start; the upper half: the
        // one that produced the next sub-window's start); hide that from CSE
        // so it is recomputed (cheap VALU) instead of holding alpha vectors live
#pragma unroll
        for (int s = CK0; s < 8; ++s) asm volatile("" : "+v"(cks[m][s]));
#pragma unroll
        for (int j = 0; j < (TSUB > 1 ? TW : TH); ++j)
          asm volatile("" : "+v"(ls[m * TW + j]), "+v"(lp[m * TW + j]), "+v"(la[m * TW + j]));
        // A[j] = alpha before step k0 + m*TW + h*TH + j
        T A[TH][8];
#pragma unroll
        for (int s = 0; s < 8; ++s) A[0][s] = cks[m][s];
        if (h > 0) {
#pragma unroll
          for (int j = 0; j < h * TH; ++j) {
            const int i = m * TW + j;
            T c[4], o[8];
            gam(ls[i], lp[i], la[i], c);
            fwd<T, LM>(A[0], c, o);
#pragma unroll
            for (int s = 0; s < 8; ++s) A[0][s] = o[s];
          }
        }
#pragma unroll
        for (int j = 0; j < TH - 1; ++j) {
          const int i = m * TW + h * TH + j;
          T c[4];
          gam(ls[i], lp[i], la[i], c);
          fwd<T, LM>(A[j], c, A[j + 1]);
        }
        // gamma is 6 VALU ops: recompute it below rather than keep the
        // recompute's gamma vectors live next to the inputs
#pragma unroll
        for (int j = 0; j < TH; ++j) {
          const int i = m * TW + h * TH + j;
          asm volatile("" : "+v"(ls[i]), "+v"(lp[i]), "+v"(la[i]));
        }
#pragma unroll
        for (int j = TH - 1; j >= 0; --j) {
          const int i = m * TW + h * TH + j;
          const int k = k0 + i;
          T c[4];
          gam(ls[i], lp[i], la[i], c);
          const T L = bstep<T, LM>(b, c, A[j]);
          if (MODE == TM_DEC1) {
            LE.st(k, ((T)0.5 * L - la[i]) - ls[i]);
          } else if (MODE == TM_DEC2) {
            dd = modsub(dd, tf2, K);
            pp = modsub(pp, dd, K);   // pp = pi(k)
            LE.st(pp, ((T)0.5 * L - la[i]) - ls[i]);
          } else if (MODE == TM_APP) {  // a-posteriori LLR in place of the extrinsic row
            LE.st(k, L);
          } else {  // TM_FINAL
            // L is still stored: without a per-step store into the block the
            // compiler schedules this pass with ~40 more VGPRs
            LE.st(k, L);
            acc |= (L < (T)0 ? 1u : 0u) << (31 - (k & 31));
          }
        }
      }
      if (MODE == TM_FINAL) {   // words start on sub-window boundaries (32 = 4 * TW)
        const int k = k0 + m * TW;
        if ((k & 31) == 0) {
          bout.st(k >> 5, acc);
          acc = 0;
        }
      }
    }
    if (MODE == TM_DEC2) { pi = pp; d = dd; }   // back at k0
  }
}

// One launch decodes every code-block slot of the batch: wave w -> job r
// (CB slot, i.e. one K) and frame group g.  256-thread blocks = 4 independent
// waves (no LDS, no barriers).
template <class T, bool LM = false, int CH = TURBO_CH>
__device__ __forceinline__ void turbo_body(const TurboJobs& jobs, int iters, int mode) {
  const int wg = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (wg >= jobs.prefix[jobs.n]) return;
  int r = 0;
  while (wg >= jobs.prefix[r + 1]) ++r;
  const TurboJob jb = jobs.j[r];
  const int g = wg - jobs.prefix[r];
  const int K = jb.K;
  // the group's chunk of the block arrays (turbo_elem: [chunk][row][CH][64])
  const int slot = g % CH;
  T* base = reinterpret_cast<T*>(jb.blk) + turbo_elem<CH>(turbo_rows(K), g - slot, 0);
  T* ck = reinterpret_cast<T*>(jb.ck) + turbo_elem<CH>(turbo_nwin(K) * TurboT<T>::CK, g - slot, 0);
  uint32_t* bo = jb.bits + (size_t)g * turbo_kw(K) * RS;
  if (mode == TM_APP) {
    half_pass<T, TM_APP, LM, CH>(base, ck, slot, lane, K, jb.f1, jb.f2, false);
    return;
  }
  for (int it = 0; it < iters; ++it) {
    half_pass<T, TM_DEC1, LM, CH>(base, ck, slot, lane, K, jb.f1, jb.f2, it == 0);
    half_pass<T, TM_DEC2, LM, CH>(base, ck, slot, lane, K, jb.f1, jb.f2, false);
  }
  // final pass = decoder 1 a-posteriori LLRs (turbo_decoder.py:440-447) and
  // the hard decisions L < 0 (:276), packed MSB-first
  half_pass<T, TM_FINAL, LM, CH>(base, ck, slot, lane, K, jb.f1, jb.f2, iters == 0, bo);
}

// f32 fast mode: 134 VGPRs = 3 waves per SIMD; LTE_TURBO32_WAVES = 2 / 1 caps
// the resident waves with reserved AGPRs (A/B knob, as k_turbo64)
#ifndef LTE_TURBO32_WAVES
#define LTE_TURBO32_WAVES 3
#endif
// CH: the chunk width of the jobs' block arrays (TURBO_CH, or 1 for arrays of
// fewer groups: turbo_chunk)
template <int CH>
__global__ __launch_bounds__(256, LTE_TURBO32_WAVES == 3 ? 2 : 1) void k_turbo(TurboJobs jobs, int iters, int mode) {
#if LTE_TURBO32_WAVES == 2
  asm volatile("" ::: "a47");
#elif LTE_TURBO32_WAVES == 1
  asm volatile("" ::: "a127");
#endif
  turbo_body<float, false, CH>(jobs, iters, mode);
}

// f64: one wave per SIMD (LTE_TURBO64_ONE_WAVE, default on; 0: up to 256
// VGPRs, two waves).  The decoder streams HBM slightly faster with one
// resident wave per SIMD than with two (A/B on one MI355X: 358 / 359 ms vs
// 367 / 368 ms per 65 536 frames); the cap is set by reserving 32 AGPRs.
#ifndef LTE_TURBO64_ONE_WAVE
#define LTE_TURBO64_ONE_WAVE 1
#endif
template <int CH>
__global__ __launch_bounds__(256, LTE_TURBO64_ONE_WAVE ? 1 : 2) void k_turbo64(TurboJobs jobs, int iters, int mode) {
#if LTE_TURBO64_ONE_WAVE
  asm volatile("" ::: "a31");
#endif
  turbo_body<double, false, CH>(jobs, iters, mode);
}

// f64 exact log-MAP (set_decoder_mode(False)); not a hot path
template <int CH>
__global__ __launch_bounds__(256, 1) void k_turbo64_logmap(TurboJobs jobs, int iters, int mode) {
  turbo_body<double, true, CH>(jobs, iters, mode);
}

// decoder arithmetic of the f64 entry points and chains: max-log-MAP (the
// reference's default, USE_MAX_LOG_MAP = True) or exact log-MAP
static int g_logmap = 0;
void set_logmap(int on) { g_logmap = on ? 1 : 0; }
int logmap_on() { return g_logmap; }

int launch_turbo_jobs(hipStream_t s, const TurboJob* jobs, int n, int iters, int mode, int f64) {
  for (int o = 0; o < n; o += TURBO_MAX_JOBS) {
    TurboJobs J{};
    J.n = n - o < TURBO_MAX_JOBS ? n - o : TURBO_MAX_JOBS;
    J.prefix[0] = 0;
    for (int i = 0; i < J.n; ++i) {
      J.j[i] = jobs[o + i];
      J.prefix[i + 1] = J.prefix[i] + jobs[o + i].G;
    }
    const int waves = J.prefix[J.n];
    if (waves == 0) continue;
    const int ch = J.j[0].ch;
    for (int i = 1; i < J.n; ++i)
      if (J.j[i].ch != ch) return (int)hipErrorInvalidValue;   // one chunk width per launch
    const dim3 grid((waves + 3) / 4);
    if (ch == TURBO_CH) {
      if (f64 && g_logmap) hipLaunchKernelGGL(k_turbo64_logmap<TURBO_CH>, grid, dim3(256), 0, s, J, iters, mode);
      else if (f64) hipLaunchKernelGGL(k_turbo64<TURBO_CH>, grid, dim3(256), 0, s, J, iters, mode);
      else hipLaunchKernelGGL(k_turbo<TURBO_CH>, grid, dim3(256), 0, s, J, iters, mode);
    } else if (ch == 1) {
      if (f64 && g_logmap) hipLaunchKernelGGL(k_turbo64_logmap<1>, grid, dim3(256), 0, s, J, iters, mode);
      else if (f64) hipLaunchKernelGGL(k_turbo64<1>, grid, dim3(256), 0, s, J, iters, mode);
      else hipLaunchKernelGGL(k_turbo<1>, grid, dim3(256), 0, s, J, iters, mode);
    } else {
      return (int)hipErrorInvalidValue;
    }
    const int e = (int)hipGetLastError();
    if (e) return e;
  }
  return 0;
}

int launch_turbo(hipStream_t s, void* blk, void* ckpt, uint32_t* bits, int K, int f1, int f2, int iters, int G,
                 int mode, int f64, int ch) {
  TurboJob j{blk, ckpt, bits, K, f1, f2, G, ch};
  return launch_turbo_jobs(s, &j, 1, iters, mode, f64);
}

// ---------------------------------------------------------------------------
// Single max-log BCJR pass of any length n in float64, a-posteriori output for
// every step: LogMAPDecoder.decode (turbo_decoder.py:181-278) as the drop-in
// LogMAPDecoder class calls it (tail steps included, any a priori).  One lane
// per code block; alpha of every step kept in a scratch [n][8][lanes] (f64,
// the reference's unnormalised metrics), then the backward sweep.  Not a hot
// path (the chain runs k_turbo64); the reference's operation order.
template <bool LM>
__global__ __launch_bounds__(64) void k_bcjr64(const double* __restrict__ ls, const double* __restrict__ lp,
                                               const double* __restrict__ la, int n, int ncb,
                                               double* __restrict__ alpha, double* __restrict__ app) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (c >= ncb) return;
  const double* S = ls + (size_t)c * n;
  const double* P = lp + (size_t)c * n;
  const double* A = la + (size_t)c * n;
  double* al = alpha + (size_t)c * 8;   // step k at al[k * ncb * 8]
  const size_t st = (size_t)ncb * 8;
  double a[8];
  a[0] = 0.0;
  for (int s = 1; s < 8; ++s) a[s] = -__builtin_inf();
  for (int k = 0; k < n; ++k) {
    for (int s = 0; s < 8; ++s) al[k * st + s] = a[s];
    double cc[4], o[8];
    gam(0.5 * S[k], 0.5 * P[k], 0.5 * A[k], cc);   // x / 2.0 == 0.5 * x (exact)
    fwd<double, LM>(a, cc, o);
    for (int s = 0; s < 8; ++s) a[s] = o[s];
  }
  double b[8];
  b[0] = 0.0;
  for (int s = 1; s < 8; ++s) b[s] = -__builtin_inf();
  for (int k = n - 1; k >= 0; --k) {
    double cc[4], ak[8];
    gam(0.5 * S[k], 0.5 * P[k], 0.5 * A[k], cc);
    for (int s = 0; s < 8; ++s) ak[s] = al[k * st + s];
    app[(size_t)c * n + k] = bstep<double, LM>(b, cc, ak);
  }
}

int launch_bcjr64(hipStream_t s, const double* ls, const double* lp, const double* la, int n, int ncb,
                  double* alpha_scratch, double* app) {
  if (n < 1 || ncb < 1) return (int)hipErrorInvalidValue;
  if (g_logmap)
    hipLaunchKernelGGL(k_bcjr64<true>, dim3((ncb + 63) / 64), dim3(64), 0, s, ls, lp, la, n, ncb, alpha_scratch, app);
  else
    hipLaunchKernelGGL(k_bcjr64<false>, dim3((ncb + 63) / 64), dim3(64), 0, s, ls, lp, la, n, ncb, alpha_scratch, app);
  return (int)hipGetLastError();
}

}  // namespace lte
