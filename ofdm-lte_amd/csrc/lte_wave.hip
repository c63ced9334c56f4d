// Wave-private signal kernels (gfx950): one wave64 owns one frame's OFDM
// symbols and transforms them with wfft::fft2048 (registers + a wave-local LDS
// transpose, no block barrier).  Same stage outputs as the block kernels of
// lte_kernels.hip they replace where they apply.
#include <cstdlib>
#include "lte_common.h"
#include "lte_internal.h"
#include "lte_dev.h"
#include "lte_wfft.h"

namespace lte {

template <class V>
__device__ __forceinline__ V* dyn_lds() {
  extern __shared__ double2 lte_dyn_lds[];
  return reinterpret_cast<V*>(lte_dyn_lds);
}

// The fused SISO receiver's equaliser pieces (lte_kernels.hip: abs2_ref, ZfCoef,
// chest_interp), restated here for the wave kernels: the same expressions.
// (Kept apart from the block kernels' copies on purpose: defined in a shared
// header they changed how the compiler contracted other expressions of those
// kernels, by an ulp, which exact f32 path-equality tests caught.)
namespace wrx {
// |h|^2 as the reference forms it: f64 np.abs(h) ** 2 (hypot, then squared);
// f32 h.x^2 + h.y^2
template <class V>
__device__ __forceinline__ re_t<V> abs2_ref(V h) {
  if constexpr (sizeof(re_t<V>) == 8) {
    const double a = hypot(h.x, h.y);
    return a * a;
  } else {
    return h.x * h.x + h.y * h.y;
  }
}


template <class R> struct ZfCoef;
template <> struct ZfCoef<double> {   // cdiv(y, h) (Smith, lte_common.h) with the h-only terms precomputed
  double rat, sre, sim;
  bool swp;
  __device__ __forceinline__ void set(double2 h) {
    swp = !(fabs(h.x) >= fabs(h.y));
    if (!swp) {
      rat = (h.x == 0.0 && h.y == 0.0) ? 0.0 : h.y / h.x;   // h = 0: a / 0 as cdiv
      sre = sim = (h.x == 0.0 && h.y == 0.0) ? 1.0 / h.x : 1.0 / (h.x + h.y * rat);
    } else {
      rat = h.x / h.y;
      sre = 1.0 / (h.y + h.x * rat);
      sim = -sre;
    }
  }
  // !swp: ((a.x + a.y rat) s, (a.y - a.x rat) s); swp: ((a.x rat + a.y) s, (a.y rat - a.x) s)
  __device__ __forceinline__ double2 apply(double2 a) const {
    const double u = swp ? a.x : a.y, v = swp ? a.y : a.x;
    return make_double2((v + u * rat) * sre, (u - v * rat) * sim);
  }
};
template <> struct ZfCoef<float> {    // zf_div(y, h): y conj(h) / |h|^2
  float2 h;
  float r;
  __device__ __forceinline__ void set(float2 hh) {
    h = hh;
    r = 1.0f / (hh.x * hh.x + hh.y * hh.y);
  }
  __device__ __forceinline__ float2 apply(float2 y) const {
    return make_float2((y.x * h.x + y.y * h.y) * r, (y.y * h.x - y.x * h.y) * r);
  }
};

// linear interpolation of the pilot LS estimates hp at subcarrier k with edge
// hold (lte_receiver.py:114-133), as k_rx_chest forms it
template <class R>
__device__ __forceinline__ cx<R> chest_interp(const Grid& g, const cx<R>* hp, int k) {
  using V = cx<R>;
  const int sidx = g.seg[k];
  if (sidx < 0) return hp[0];
  if (sidx >= g.Np - 1) return hp[g.Np - 1];
  const V v0 = hp[sidx], v1 = hp[sidx + 1];
  const R fk = (R)(k - g.pilot_idx[sidx]);
  const R ig = GridT<R>::inv_gap(g)[sidx];
  return mkc(fk * ((v1.x - v0.x) * ig) + v0.x, fk * ((v1.y - v0.y) * ig) + v0.y);
}

// the fused SIMO receiver's per-RE interpolation (lte_kernels.hip interp_seg:
// chest_interp with the segment, offset and 1 / gap precomputed per RE)
template <class R>
__device__ __forceinline__ cx<R> interp_seg(const cx<R>* hp, int np, int sidx, R fk, R ig) {
  if (sidx < 0) return hp[0];
  if (sidx >= np - 1) return hp[np - 1];
  const cx<R> v0 = hp[sidx], v1 = hp[sidx + 1];
  return mkc(fk * ((v1.x - v0.x) * ig) + v0.x, fk * ((v1.y - v0.y) * ig) + v0.y);
}
}  // namespace wrx

// One OFDM symbol's N = 64 M received samples after its CP (stream offset
// off) into wfft's register layout (lane l, register m = sample 64 m + l: 1 KB
// per wave load instruction) plus sigma times the noise as load_symbol_noisy2
// draws it: injected [2][L] draws, or one rng4 per sample pair on stream
// RNG_STREAM_NOISE + rx, lanes 2t / 2t + 1 computing the pair counters of
// registers m / m + 1 and trading halves with one DPP swap.  Half a symbol at
// a time, a rolled loop draws into the wave's LDS scratch zs (M / 2 KB) and
// each register then adds its draw (unrolled over the registers, the 16 Philox
// + 32 Box-Muller chains of N = 2048 took the kernel past 512 registers).
#ifndef WSN_UNROLL   // the draw loop's unroll (1: rolled)
#define WSN_UNROLL 1
#endif
template <int M, class TB>
__device__ __forceinline__ void wave_symbol_noisy(double2 (&v)[M], const double2* __restrict__ yf, int off, int lane,
                                                  double sigma, uint64_t seed, uint64_t fr, int rx,
                                                  const double* __restrict__ zf, int L, double* scratch,
                                                  const TB& bmt) {
  constexpr int MH = M / 2;
  const bool odd = lane & 1;
#pragma unroll
  for (int m = 0; m < M; ++m) v[m] = yf[off + 64 * m + lane];
  double2* zs = reinterpret_cast<double2*>(scratch);   // [M / 2][64]
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (zf) {
#pragma unroll 1
      for (int mm = 0; mm < MH; ++mm) {
        const int n = off + 64 * (MH * h + mm) + lane;
        zs[64 * mm + lane] = make_double2(zf[n], zf[L + n]);
      }
    } else {
#pragma unroll WSN_UNROLL
      for (int mm = 0; mm < MH; mm += 2) {
        // even lanes: the pair counter of register m; odd lanes: of register m + 1
        const int m = MH * h + mm;
        const uint32_t ctr = (uint32_t)((off + 64 * m + (odd ? 64 : 0) + lane) >> 1);
        const u32x4 r = rng4(seed, fr, RNG_STREAM_NOISE + (uint32_t)rx, ctr);
        const uint32_t t0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)(odd ? r.x : r.z), 0xB1, 0xF, 0xF, true);
        const uint32_t t1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)(odd ? r.y : r.w), 0xB1, 0xF, 0xF, true);
        zs[64 * mm + lane] = gauss2t<double>(odd ? t0 : r.x, odd ? t1 : r.y, bmt);
        zs[64 * (mm + 1) + lane] = gauss2t<double>(odd ? r.z : t0, odd ? r.w : t1, bmt);
      }
    }
    wfft::wave_lds_fence();
#pragma unroll
    for (int i = 0; i < MH; ++i) {
      const double2 z = zs[64 * i + lane];
      v[MH * h + i] = make_double2(v[MH * h + i].x + sigma * z.x, v[MH * h + i].y + sigma * z.y);
    }
    wfft::wave_lds_fence();
  }
}

// Wave-private fused SISO receiver (float64, N = 2048, coded chain with the
// demap in k_dematch_zn): one wave64 per frame walks its 14 n_sym symbols with
// no block barrier.  Per symbol: the 2048 samples after the CP land in
// registers in wfft's layout (lane l, register m = sample 64 m + l: 1 KB per
// wave load instruction), plus the Philox noise -- one rng4 per sample pair as
// load_symbol_noisy2 draws it, lanes 2t / 2t + 1 computing the counters of
// registers m / m + 1 and trading halves with one DPP swap -- then
// wfft::fft2048 (registers + one wave-local LDS transpose) leaves lane c,
// register q = X[64 q + c].  Grid::kinfo names each bin's role.  At the first
// symbol of a 14-symbol group the pilot lanes form the LS estimates into the
// wave's LDS scratch (the transpose buffer, free between transforms), and each
// data RE's equaliser terms (ZfCoef: rat and sre, the swap flag as bit q of a
// per-lane mask) and sigma^2_eff (nvo) are formed once per group, exactly as
// k_rx_frame forms them (same chest_interp / ZfCoef / abs2_ref code, so the
// same bits for the same FFT output).  The (rat, sre) pairs wait in the
// group's last symbol's slot of the output zo -- Nd x 16 B, exactly its size
// -- read back by the same lane each symbol and overwritten by that symbol's
// own outputs (read before write, same lane and address), so the wave's LDS
// is the transpose buffer alone (16.5 KB): two waves per SIMD.  The
// transform's rounding differs from fft_lds's (both within a few 1e-14 of the
// exact DFT: profiles/r6_wfft_microbench_wpe*.jsonl).
#ifndef RXW_WPE   // register budget: waves per SIMD the compiler schedules for (LDS allows 1)
#define RXW_WPE 2
#endif
constexpr int RXW_WAVES = 4;
#ifndef TXW_WAVES   // frames (waves) per block of k_ofdm_txf_w
#define TXW_WAVES 4
#endif
#ifndef TXW_OUNROLL
#define TXW_OUNROLL 2
#endif
#ifndef TXW_WPE
#define TXW_WPE 2
#endif
__global__ __launch_bounds__(64 * RXW_WAVES) __attribute__((amdgpu_waves_per_eu(RXW_WPE, RXW_WPE)))
void k_rx_frame_w(Grid g, int rayleigh, int B, const double2* __restrict__ y, int64_t y_frame_stride,
                  const double* __restrict__ npow, const double* __restrict__ snr_lin, const uint64_t* __restrict__ fid,
                  uint64_t seed, const double* __restrict__ inj_z, int64_t inj_stride, double2* __restrict__ zo,
                  double* __restrict__ nvo, double2* __restrict__ cap_syms, double2* __restrict__ H,
                  double* __restrict__ pstats) {
  constexpr int N = 2048;
  using G = GridT<double>;
  LTE_BM_LDS_DECL(double);
  const auto bmt = bm_stage<double>(lte_bmt);
  const int lane0 = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.x * RXW_WAVES + w;
  double* tl = reinterpret_cast<double*>(dyn_lds<double2>()) + (size_t)w * wfft::LDS_DOUBLES;
  __syncthreads();   // the Box-Muller tables (the only block barrier)
  if (b >= B) return;
  const double sigma = sqrt(npow[b] / 2.0);
  const double s2 = 1.0 / snr_lin[b];
  const uint64_t fr = fid[b];
  const double* zf = inj_z ? inj_z + (size_t)b * inj_stride : nullptr;
  const double2* yf = y + (size_t)b * y_frame_stride;
  const size_t fre = (size_t)b * g.n_sym * g.Nd;
  const double sc = rx_scale<double>(N);
  uint32_t swpm = 0;
  double2* cf = zo + fre;   // the current group's (rat, sre) by data ordinal
  for (int l = 0; l < g.n_sym; ++l) {
    // lane made opaque per symbol: the twiddle / address arithmetic derived
    // from it is recomputed each symbol instead of hoisted and held live (spills)
    int lane = lane0;
    asm volatile("" : "+v"(lane));
    const int off = l * (N + g.cp) + g.cp;
    double2 v[32];
    wave_symbol_noisy(v, yf, off, lane, sigma, seed, fr, 0, zf, g.L, tl, bmt);
    // and again before the transform, so its twiddle loads are not hoisted
    // above the noise (48 more registers live across it)
    int lane_f = lane;
    asm volatile("" : "+v"(lane_f));
    wfft::fft2048<false>(v, tl, G::tw(g), lane_f);
    if (l % 14 == 0) {   // group estimate from its first symbol (lte_receiver.py:360-411)
      const int grp = l / 14;
      double2* hp = reinterpret_cast<double2*>(tl);   // [Np] LS estimates, then [Np] scaled pilots
      double2* yp = hp + g.Np;
#pragma unroll
      for (int q = 0; q < 32; ++q) {
        const int kq = g.kinfo[64 * q + lane];
        if (kq <= -2) yp[-kq - 2] = cscale(v[q], sc);
      }
      wfft::wave_lds_fence();
      for (int p = lane; p < g.Np; p += 64) hp[p] = cdiv(yp[p], G::pilots(g)[p]);
      wfft::wave_lds_fence();
      if (H) {
        double2* Hf = H + ((size_t)b * g.n_grp + grp) * N;
        for (int k = lane; k < N; k += 64) Hf[k] = wrx::chest_interp<double>(g, hp, k);
      }
      // rolled (kinfo re-read): the interpolation and ZfCoef code once, not per register
      swpm = 0;
      cf = zo + fre + (size_t)min(l + 13, g.n_sym - 1) * g.Nd;   // the group's last symbol's slot
      const size_t nvg = ((size_t)b * g.n_grp + grp) * g.Nd;
#pragma unroll 1
      for (int q = 0; q < 32; ++q) {
        const int k = 64 * q + lane, j = g.kinfo[k];
        if (j < 0) continue;
        const double2 h = wrx::chest_interp<double>(g, hp, k);
        wrx::ZfCoef<double> zc;
        zc.set(make_double2(h.x + 1e-6, h.y));
        cf[j] = make_double2(zc.rat, zc.sre);
        swpm |= (uint32_t)zc.swp << q;
        const double den = wrx::abs2_ref(h);
        nvo[nvg + j] = rayleigh ? fmax(s2 / fmin(fmax(den, 1e-6), 1e6), s2 / 4.0) : s2;
      }
      if (pstats && lane == 0) {
        double pp = 0.0, en = 0.0;
        for (int p = 0; p < g.Np; ++p) {
          const double2 Yp = yp[p], X = G::pilots(g)[p];
          pp += Yp.x * Yp.x + Yp.y * Yp.y;
          const double2 d = csub(Yp, X);
          en += d.x * d.x + d.y * d.y;
        }
        double* st = pstats + ((size_t)b * g.n_grp + grp) * 2;
        st[0] = pp / (double)g.Np;
        st[1] = en / (double)g.Np;
      }
      wfft::wave_lds_fence();   // the scratch is the next transform's
    }
    // the bins' roles re-read per symbol (L1-resident 8 KB table; held in
    // registers they were widened to 64-bit addresses and spilled)
    const size_t fl = fre + (size_t)l * g.Nd;
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      const int j = g.kinfo[64 * q + lane];
      if (j >= 0) {
        const double2 c = cf[j];
        wrx::ZfCoef<double> zc;
        zc.rat = c.x;
        zc.sre = c.y;
        zc.swp = (swpm >> q) & 1u;
        zc.sim = zc.swp ? -c.y : c.y;
        const double2 z = zc.apply(cscale(v[q], sc));
        zo[fl + j] = z;
        if (cap_syms) cap_syms[fl + j] = z;
      }
    }
  }
}

bool rx_frame_w_supported(const Grid& g, int chain, int f64) {
  return f64 && g.N == 2048 && chain == LTE_CHAIN_CODED && g.kinfo && g.pilots64 && g.cp % 2 == 0 && g.Np >= 1 &&
         32 * g.Np <= wfft::LDS_DOUBLES * 8;
}

// ---------------------------------------------------------------------------
// Wave-private coded OFDM TX + static-tap channel (float64, N = 2048): one
// wave64 per frame walks its symbols, the k_ofdm_txf outputs without a block
// barrier.  Per symbol: lane c, register q builds bin k = 64 q + c (Grid::kinfo:
// the data RE's BPS coded bits through tx_map -> qam_point, a pilot, or 0),
// wfft::fft2048<INV> and the output scale sqrt(N) / N give x[64 q + c]; the
// taps' cyclic reach (every delay <= 64 <= CP, so output sample n of the
// received stream is sum_p c_p x[(n - d_p) mod N] for the N samples after the
// CP and, again, for the CP samples past max_delay) reads x through the wave's
// LDS window, half a symbol (17 registers' samples) at a time; the symbol
// power sums |y|^2 over those samples (k_chan_fix adds the first max_delay).
// STAGE: the frame's coded stream staged in the wave's LDS once (else the bit
// gathers go through L1 / L2).
constexpr int TXW_XS = 17 * 64 * 16;   // bytes: the tap window (>= the transpose buffer)
static_assert(TXW_XS >= wfft::LDS_DOUBLES * 8, "the tap window doubles as the transpose buffer");
template <int BPS, int NP, bool STAGE>
__global__ __launch_bounds__(64 * TXW_WAVES) __attribute__((amdgpu_waves_per_eu(TXW_WPE, TXW_WPE)))
void k_ofdm_txf_w(Grid g, const uint32_t* __restrict__ enc, int enc_words, const int32_t* __restrict__ tx_map, int B,
                  double2* __restrict__ cap_syms, TxChannelT<double> ch) {
  constexpr int N = 2048;
  using G = GridT<double>;
  const int lane0 = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.x * TXW_WAVES + w;
  if (b >= B) return;   // no block barrier anywhere in this kernel
  const int ew = STAGE ? (enc_words + 3) & ~3 : 0;
  char* wl = reinterpret_cast<char*>(dyn_lds<double2>()) + (size_t)w * (TXW_XS + 4 * (size_t)ew);
  double2* xs = reinterpret_cast<double2*>(wl);
  const uint32_t* es;
  if constexpr (STAGE) {
    uint32_t* e = reinterpret_cast<uint32_t*>(wl + TXW_XS);
    const uint32_t* fe = enc + (size_t)b * enc_words;
    for (int i = lane0; i < enc_words; i += 64) e[i] = fe[i];
    wfft::wave_lds_fence();
    es = e;
  } else {
    es = enc + (size_t)b * enc_words;
  }
  const double sc = tx_scale<double>(N);
  const int cp = g.cp, S = N + cp, D = ch.max_delay;
  double2 cf[NP];
  int dl[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    cf[p] = ch.coef[(size_t)b * NP + p];   // SISO: one RX
    dl[p] = ch.delays[p];
  }
  for (int l = 0; l < g.n_sym; ++l) {
    int lane = lane0;   // opaque per symbol (see k_rx_frame_w)
    asm volatile("" : "+v"(lane));
    double2 v[32];
    const size_t sym0 = ((size_t)b * g.n_sym + l) * g.Nd;
    // the bins half a symbol at a time: a rolled loop forms them into the
    // wave's LDS window, then the registers read them (unrolled over the
    // registers, every bin's tx_map / coded-bit loads were hoisted together)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll 1
      for (int i = 0; i < 16; ++i) {
        const int r = g.kinfo[64 * (16 * h + i) + lane];
        double2 x = make_double2(0.0, 0.0);
        if (r >= 0) {
          const int32_t* src = tx_map + ((int64_t)l * g.Nd + r) * BPS;
          int idx = 0;
          bool zero = false;
#pragma unroll
          for (int m = 0; m < BPS; m += 2) {
            const int2 t = *reinterpret_cast<const int2*>(src + m);
            zero |= t.x == -2 || t.y == -2;
            idx = (idx << 2) | (int)((t.x >= 0 ? getbit(es, t.x) : 0u) << 1) | (int)(t.y >= 0 ? getbit(es, t.y) : 0u);
          }
          x = zero ? make_double2(0.0, 0.0) : qam_point<BPS, double>(idx);
          if (cap_syms) cap_syms[sym0 + r] = x;
        } else if (r <= -2) {
          x = G::pilots(g)[-r - 2];
        }
        xs[64 * i + lane] = x;
      }
      wfft::wave_lds_fence();
#pragma unroll
      for (int i = 0; i < 16; ++i) v[16 * h + i] = xs[64 * i + lane];
      wfft::wave_lds_fence();
    }
    int lane_f = lane;
    asm volatile("" : "+v"(lane_f));
    wfft::fft2048<true>(v, reinterpret_cast<double*>(xs), G::tw(g), lane_f);
#pragma unroll
    for (int q = 0; q < 32; ++q) v[q] = cscale(v[q], sc);
    if (D > 0) {   // the TX samples at both ends of the CP-extended symbol (k_chan_fix reads them)
      double2* xh = ch.xh + ((size_t)b * g.n_sym + l) * 2 * D;
#pragma unroll
      for (int q = 0; q < 32; ++q) {
        const int n = 64 * q + lane;
        if (n >= N - cp && n < N - cp + D) xh[n - (N - cp)] = v[q];
        if (n >= N - D) xh[n - (N - 2 * D)] = v[q];
      }
    }
    double2* yo = ch.y + (size_t)b * g.L + (size_t)l * S + cp;
    double pw = 0.0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      // window rows i = 0..16 hold registers 16 h - 1 + i (mod 32): samples
      // 64 (16 h - 1) ... 64 (16 h + 16) - 1 of the cyclic symbol
      wfft::wave_lds_fence();
#pragma unroll
      for (int i = 0; i < 17; ++i) xs[64 * i + lane] = v[(16 * h + 31 + i) & 31];
      wfft::wave_lds_fence();
      // outputs from the window only (not the registers): partly rolled, so the
      // window loads of all 16 outputs are not hoisted together
#pragma unroll TXW_OUNROLL
      for (int i = 0; i < 16; ++i) {
        const int q = 16 * h + i, n = 64 * q + lane;
        double2 y = make_double2(0.0, 0.0);
#pragma unroll
        for (int p = 0; p < NP; ++p) y = cadd(y, cmul(cf[p], xs[64 * (i + 1) + lane - dl[p]]));
        yo[n] = y;
        const double e = y.x * y.x + y.y * y.y;
        pw += e;
        if (n >= N - cp + D) pw += e;   // the CP sample m = n - N + cp carries the same value
      }
    }
    for (int o = 32; o > 0; o >>= 1) pw += __shfl_xor(pw, o);
    if (lane == 0) ch.pow_part[(size_t)b * g.n_sym + l] = pw;
  }
}

bool txf_w_supported(const Grid& g, int f64, int n_paths, int max_delay, int num_rx, int tv) {
  return f64 && g.N == 2048 && g.kinfo && g.pilots64 && num_rx == 1 && !tv && n_paths == 4 && max_delay <= 64 &&
         max_delay <= g.cp && (g.bps == 2 || g.bps == 4 || g.bps == 6);
}

// ---------------------------------------------------------------------------
// Wave-private multi-antenna RX FFT + CRS pilot estimates (float64, N = 2048;
// k_rx_fft_mimo<.., HPO>'s outputs): one wave64 per (frame, RX antenna) walks
// the frame's symbols.  Per symbol wave_symbol_noisy + wfft::fft2048; the
// n_dsc data SCs go to Y[b][l][rx][n_dsc] from the registers (Grid::kinfo's
// data ordinal); on estimation symbols (SFBC: first of each group, spatial:
// every symbol) the scaled spectrum passes through the wave's LDS scratch
// half a symbol at a time and each TX's LS pilot estimates
// (mimo_channel_estimator_periodic.py:195-273) go to H[b][rx][e][tx][maxP].
constexpr int RXMW_WAVES = 4;
#ifndef RXMW_WPE   // register budget (LDS allows two waves per SIMD)
#define RXMW_WPE 2
#endif
__global__ __launch_bounds__(64 * RXMW_WAVES) __attribute__((amdgpu_waves_per_eu(RXMW_WPE, RXMW_WPE)))
void k_rx_fft_mimo_w(Grid g, MimoGrid m, int B, const double2* __restrict__ y, const double* __restrict__ npow,
                     const uint64_t* __restrict__ fid, uint64_t seed, const double* __restrict__ inj_z,
                     int64_t inj_stride, double2* __restrict__ Y, double2* __restrict__ H) {
  constexpr int N = 2048;
  using G = GridT<double>;
  LTE_BM_LDS_DECL(double);
  const auto bmt = bm_stage<double>(lte_bmt);
  const int lane0 = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int gs = blockIdx.x * RXMW_WAVES + w;
  const int b = gs / m.num_rx, rx = gs - b * m.num_rx;
  double* tl = reinterpret_cast<double*>(dyn_lds<double2>()) + (size_t)w * wfft::LDS_DOUBLES;
  __syncthreads();   // the Box-Muller tables (the only block barrier)
  if (b >= B) return;
  const size_t br = (size_t)b * m.num_rx + rx;
  const double sigma = sqrt(npow[br] * 0.5);
  const uint64_t fr = fid[b];
  const double* zf = inj_z ? inj_z + (size_t)b * inj_stride + (size_t)rx * 2 * g.L : nullptr;
  const double2* yf = y + br * g.L;
  const double sc = rx_scale<double>(N);
  const double2* pv = MGT<double>::pval(m);
  for (int l = 0; l < g.n_sym; ++l) {
    int lane = lane0;   // opaque per symbol (see k_rx_frame_w)
    asm volatile("" : "+v"(lane));
    const int off = l * (N + g.cp) + g.cp;
    double2 v[32];
    wave_symbol_noisy(v, yf, off, lane, sigma, seed, fr, rx, zf, g.L, tl, bmt);
    int lane_f = lane;
    asm volatile("" : "+v"(lane_f));
    wfft::fft2048<false>(v, tl, G::tw(g), lane_f);
#pragma unroll
    for (int q = 0; q < 32; ++q) v[q] = cscale(v[q], sc);
    const bool est = m.mode == MIMO_SFBC ? (l % 14) == 0 : true;
    if (est) {
      const int e = m.mode == MIMO_SFBC ? l / 14 : l;
      double2* xs = reinterpret_cast<double2*>(tl);   // [1024]: bins 1024 h ... 1024 h + 1023
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < 16; ++i) xs[64 * i + lane] = v[16 * h + i];
        wfft::wave_lds_fence();
        for (int t = 0; t < m.num_tx; ++t) {
          double2* Ho = H + ((br * m.n_est + e) * m.num_tx + t) * m.maxP;
          for (int p = lane; p < m.np_tx[t]; p += 64) {
            const int pos = m.ppos[t * m.maxP + p];
            if ((pos >> 10) == h) Ho[p] = cdiv(xs[pos & 1023], pv[t * m.maxP + p]);
          }
        }
        wfft::wave_lds_fence();
      }
    }
    double2* Yo = Y + (((size_t)b * g.n_sym + l) * m.num_rx + rx) * m.n_dsc;
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      const int j = g.kinfo[64 * q + lane];
      if (j >= 0 && j < m.n_dsc) Yo[j] = v[q];
    }
  }
}

bool rx_fft_mimo_w_supported(const Grid& g, const MimoGrid& m, int f64, int h_pilots) {
  return f64 && h_pilots && g.N == 2048 && g.kinfo && m.pval64 && g.cp % 2 == 0;
}

// ---------------------------------------------------------------------------
// Wave-private fused SIMO MRC receiver (float64, N = 1024, uncoded: config 3;
// k_rx_frame_simo2's outputs): one frame per 256-thread block, wave w owns RX
// antenna w (num_rx <= 4).  Per symbol, two phases split by the block's only
// two barriers:
//   1. each RX wave loads its stream's 1024 samples after the CP plus the
//      Philox noise (wave_symbol_noisy, the same draws) and transforms them
//      with wfft::fft1024 (registers + one wave-local LDS transpose); the
//      scaled data bins go to its row of yb by data ordinal (Grid::kinfo) and,
//      on a group's first symbol, its pilot bins' LS estimates to hpa;
//   2. every thread takes up to two data REs and folds the RX in order into
//      the MRC sums exactly as k_rx_frame_simo2 does (interp_seg, abs2_ref,
//      cmulc), then the hard decision and bit errors.
// A wave's yb row doubles as its noise / transpose scratch (free once phase 2
// has read it), so the block's LDS is 4 x 544 x 16 B + the estimates + the
// per-RE interpolation terms + the Box-Muller tables (53 KB at 10 MHz): three
// blocks per CU.
#ifndef SIMOW_WPE
#define SIMOW_WPE 3
#endif
constexpr int SIMOW_WAVES = 4;
constexpr int SIMOW_ROW_MIN = (wfft::LDS_DOUBLES_1024 + 1) / 2;   // double2 slots a row needs as scratch
static_assert(SIMOW_ROW_MIN * 16 >= 8 * 64 * 16, "a row holds the noise scratch (8 registers x 64 lanes)");
template <int BPS>
__global__ __launch_bounds__(64 * SIMOW_WAVES) __attribute__((amdgpu_waves_per_eu(SIMOW_WPE, SIMOW_WPE)))
void k_rx_frame_simo_w(Grid g, int B, int num_rx, int yrow, const double2* __restrict__ y, int64_t y_rx_stride,
                       int64_t y_frame_stride, const double* __restrict__ npow, const uint64_t* __restrict__ fid,
                       uint64_t seed, const double* __restrict__ inj_z, int64_t inj_stride,
                       const uint32_t* __restrict__ pw, int PW, int n_bits, uint32_t* __restrict__ frame_err,
                       double2* __restrict__ cap_syms, uint8_t* __restrict__ cap_bits) {
  constexpr int N = 1024, WGS = 64 * SIMOW_WAVES, QM = 2;
  using G = GridT<double>;
  LTE_BM_LDS_DECL(double);
  const auto bmt = bm_stage<double>(lte_bmt);
  const int tid0 = threadIdx.x, lane0 = tid0 & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid0 >> 6);
  const int b = blockIdx.x;
  double2* yb = dyn_lds<double2>();                 // [SIMOW_WAVES][yrow] scaled data bins
  double2* hpa = yb + (size_t)SIMOW_WAVES * yrow;    // [num_rx][Np] LS pilot estimates of the group
  int2* rtab = reinterpret_cast<int2*>(hpa + (size_t)num_rx * g.Np);   // [QM WGS] phase 2's per-RE terms
  double* igl = reinterpret_cast<double*>(rtab + QM * WGS);            // [Np] 1 / pilot gap
  double* tl = reinterpret_cast<double*>(yb + (size_t)w * yrow);
  const double sc = rx_scale<double>(N);
  constexpr double QS = qam_norm<BPS>();
  const uint64_t fr = fid[b];
  const uint32_t* fb = pw + (size_t)b * PW;
  const size_t fre = (size_t)b * g.n_sym * g.Nd;
  // phase 1's RX
  const bool has_rx = w < num_rx;
  const int rx = has_rx ? w : 0;
  const double sigma = sqrt(npow[(size_t)b * num_rx + rx] / 2.0);
  const double* zf = inj_z ? inj_z + (size_t)b * inj_stride + (size_t)rx * 2 * g.L : nullptr;
  const double2* yr = y + (size_t)b * y_frame_stride + rx * y_rx_stride;
  // phase 2's REs: chest_interp's per-subcarrier terms, staged in LDS once
  // (held in registers across phase 1 they pushed the transform into spills;
  // re-read from the tables per symbol they put a dependent load chain on the
  // critical path): x = data SC | (segment + 1) << 16, y = offset from the
  // segment's left pilot
  double den[QM];   // the sum over RX of |h|^2, per group
#pragma unroll
  for (int q = 0; q < QM; ++q) {
    den[q] = 0.0;
    const int j = tid0 + q * WGS;
    if (j < g.Nd) {
      const int kpos = g.data_idx[j], sg = g.seg[kpos];
      const int sc_ = sg < 0 ? 0 : (sg >= g.Np - 1 ? g.Np - 1 : sg);
      rtab[j] = make_int2(kpos | ((sg + 1) << 16), kpos - g.pilot_idx[sc_]);
    }
  }
  for (int p = tid0; p < g.Np; p += WGS) igl[p] = G::inv_gap(g)[p];
  uint32_t errs = 0;
  __syncthreads();   // the Box-Muller tables, rtab, igl
  for (int l = 0; l < g.n_sym; ++l) {
    const bool est = l % 14 == 0;
    if (has_rx) {
      int lane = lane0;   // opaque per symbol (see k_rx_frame_w)
      asm volatile("" : "+v"(lane));
      const int off = l * (N + g.cp) + g.cp;
      double2 v[16];
      wave_symbol_noisy(v, yr, off, lane, sigma, seed, fr, rx, zf, g.L, tl, bmt);
      int lane_f = lane;
      asm volatile("" : "+v"(lane_f));
      wfft::fft1024<false>(v, tl, G::tw(g), lane_f);
      double2* hp = hpa + rx * g.Np;
      double2* yw = yb + (size_t)w * yrow;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int j = g.kinfo[64 * q + lane];
        const double2 x = cscale(v[q], sc);
        if (j >= 0) yw[j] = x;
        else if (est && j <= -2) hp[-j - 2] = cdiv(x, G::pilots(g)[-j - 2]);   // lte_receiver.py:360-411
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < QM; ++q) {
      const int j = tid0 + q * WGS;
      if (j >= g.Nd) continue;
      const int2 rt = rtab[j];
      const int sg = (rt.x >> 16) - 1;
      const int sc_ = sg < 0 ? 0 : (sg >= g.Np - 1 ? g.Np - 1 : sg);
      const double fk = (double)rt.y, ig = igl[sc_];
      if (est) den[q] = 0.0;
      double2 num = make_double2(0.0, 0.0);
      for (int u = 0; u < num_rx; ++u) {   // the RX in order
        const double2 h = wrx::interp_seg<double>(hpa + u * g.Np, g.Np, sg, fk, ig);
        if (est) den[q] += wrx::abs2_ref(h);
        num = cadd(num, cmulc(yb[(size_t)u * yrow + j], h));
      }
      const int re = l * g.Nd + j;
      const double rr = 1.0 / (den[q] + 1e-10);
      const double2 z = make_double2(num.x * rr, num.y * rr);
      if (cap_syms) cap_syms[fre + re] = z;
      const int idx = hard_index(z, BPS, QS);
      const int64_t pb0 = (int64_t)re * BPS;
      errs += __popc(((uint32_t)idx ^ getbits<BPS>(fb, pb0, n_bits)) & bits_valid<BPS>(pb0, n_bits));
      if (cap_bits) {
#pragma unroll
        for (int m = 0; m < BPS; ++m)
          if (pb0 + m < n_bits) cap_bits[(size_t)b * n_bits + pb0 + m] = (uint8_t)((idx >> (BPS - 1 - m)) & 1);
      }
    }
    __syncthreads();   // every read of yb / hpa done before the next symbol's phase 1
  }
  frame_err_add(frame_err, b, errs);
}

bool rx_simo_w_supported(const Grid& g, int num_rx, int f64, bool H, bool pstats, bool xin) {
  return f64 && g.N == 1024 && g.kinfo && g.pilots64 && g.cp % 2 == 0 && num_rx >= 1 && num_rx <= SIMOW_WAVES &&
         num_rx <= RXS_MAXRX && !H && !pstats && !xin && g.Nd <= 2 * 64 * SIMOW_WAVES && g.Np >= 1 &&
         (g.bps == 2 || g.bps == 4 || g.bps == 6);
}

// ---------------------------------------------------------------------------
// Wave-private uncoded OFDM TX + static-tap SIMO channel (float64, N = 1024:
// config 3; k_ofdm_tx<.., CH = 1>'s outputs): one wave64 per (frame, OFDM
// symbol), no block barrier.  Lane c, register q builds bin k = 64 q + c from
// Grid::kinfo (a data RE's BPS payload bits -> qam_point, a pilot, or 0);
// wfft::fft1024<INV> and the output scale give x[64 q + c], which is staged in
// the wave's LDS (the transform's scratch before) so that every RX's taps read
// their cyclic shifts: received sample n = sum_p c_rp x[(n - d_p) mod N]
// (every delay <= CP), the same terms in the same order as tx_channel.
// Each RX's N samples after the CP go out as 1 KB wave stores; its power
// partial is the sum of |y|^2 over those samples plus the CP samples past
// max_delay (cyclically the last cp - max_delay samples again), by one wave
// reduction (tx_channel sums the same values in another order).
// TXSW_HALF (max_delay <= 64, cp <= 512, <= 4 RX): the taps read x through a
// 9-register window (9 KB) half a symbol at a time instead of the whole symbol
// staged (16 KB), for four waves per SIMD (120 VGPRs) instead of two and a
// half (profiles/r6_simo_tx_wave/: 14.1 against 15.5 ms per 65 536 frames).
// TXSW_FRAME (with TXSW_HALF): one wave per frame walking its symbols, which
// keeps the previous symbol's last register and so also forms each symbol's
// first max_delay channel-output samples' power (their taps reach into the
// previous symbol: k_chan_fix's work, which then does not run) from a tenth
// window slot.
#ifndef TXSW_HALF
#define TXSW_HALF 1
#endif
#ifndef TXSW_FRAME
#define TXSW_FRAME 1
#endif
static_assert(!TXSW_FRAME || TXSW_HALF, "the per-frame form uses the window");
constexpr int TXSW_WAVES = 2;
constexpr int TXSW_XS = TXSW_HALF ? (9 + TXSW_FRAME) * 64 : 1024;   // double2 per wave
static_assert(TXSW_XS * 2 >= wfft::LDS_DOUBLES_1024, "the window doubles as the transpose buffer");
#ifndef TXSW_UNROLL
#if TXSW_HALF
#define TXSW_UNROLL 1
#else
#define TXSW_UNROLL 4
#endif
#endif
#ifndef TXSW_WPE
#define TXSW_WPE (TXSW_HALF ? 4 : 2)
#endif
template <int BPS, int NP>
__global__ __launch_bounds__(64 * TXSW_WAVES) __attribute__((amdgpu_waves_per_eu(TXSW_WPE, TXSW_WPE)))
void k_ofdm_tx_simo_w(Grid g, const uint32_t* __restrict__ pw, int PW, int B, double2* __restrict__ cap_syms,
                      TxChannelT<double> ch) {
  constexpr int N = 1024;
  using G = GridT<double>;
  const int lane0 = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int gs = blockIdx.x * TXSW_WAVES + w;
#if TXSW_FRAME
  const int b = gs;
  if (b >= B) return;   // uniform per wave; no block barrier below
  double2 tailp = make_double2(0.0, 0.0);   // the previous symbol's x[960 + lane]
  for (int l = 0; l < g.n_sym; ++l) {
#else
  const int b = gs / g.n_sym, l = gs - b * g.n_sym;
  if (b >= B) return;   // uniform per wave; no block barrier below
#endif
  double2* xs = dyn_lds<double2>() + (size_t)w * TXSW_XS;
  int lane = lane0;
  asm volatile("" : "+v"(lane));
  // 1. the bins (QAMModulator.bits_to_symbols, ResourceMapper.map_symbols)
  const uint32_t* fb = pw + (size_t)b * PW;
  const size_t cre = ((size_t)b * g.n_sym + l) * g.Nd;
  double2 v[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int kq = g.kinfo[64 * q + lane];
    double2 x = make_double2(0.0, 0.0);
    if (kq >= 0) {
      const int idx = (int)getbits<BPS>(fb, ((int64_t)l * g.Nd + kq) * BPS, INT64_MAX);
      x = qam_point<BPS, double>(idx);
      if (cap_syms) cap_syms[cre + kq] = x;
    } else if (kq <= -2) {
      x = G::pilots(g)[-kq - 2];
    }
    v[q] = x;
  }
  // 2. ifft * sqrt(N) (modulator.py:242-248), staged for the taps
  int lane_f = lane;
  asm volatile("" : "+v"(lane_f));
  wfft::fft1024<true>(v, reinterpret_cast<double*>(xs), G::tw(g), lane_f);
  const double sc = tx_scale<double>(N);
  const int cp = g.cp, S = N + cp, D = ch.max_delay;
  constexpr int PM = NP ? NP : TXCH_MAXP;
  const int np = NP ? NP : ch.n_paths;
  const int tail = N - cp + D;   // samples n >= tail repeat as the CP samples past max_delay
#if TXSW_HALF
#pragma unroll
  for (int q = 0; q < 16; ++q) v[q] = cscale(v[q], sc);
  if (!TXSW_FRAME && D > 0) {   // the TX samples at both ends of the extended symbol (k_chan_fix), from the registers
    double2* xh = ch.xh + ((size_t)b * g.n_sym + l) * 2 * D;
#pragma unroll
    for (int q = 8; q < 16; ++q) {   // (cp <= 512)
      const int n = 64 * q + lane_f;
      if (n >= N - cp && n < N - cp + D) xh[n - (N - cp)] = v[q];
      if (n >= N - D) xh[n - N + 2 * D] = v[q];
    }
  }
  // 3. every RX's taps (transmit_simo, core/ofdm_core.py:361-412), half a
  //    symbol at a time: window slot s holds register (8 h - 1 + s) mod 16, so
  //    output n = 512 h + 64 q + lane reads x[n - d] at slot q + 1 - d / 64
  double pwr[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int sl = 0; sl < 9; ++sl) xs[64 * sl + lane_f] = v[(8 * h - 1 + sl) & 15];
#if TXSW_FRAME
    if (h == 1) xs[64 * 9 + lane_f] = tailp;
#endif
    wfft::wave_lds_fence();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (r >= ch.num_rx) break;
      const size_t br = (size_t)b * ch.num_rx + r;
      double2 cf[PM];
      int dl[PM];
#pragma unroll
      for (int p = 0; p < PM; ++p) {
        cf[p] = p < np ? ch.coef[br * np + p] : make_double2(0.0, 0.0);
        dl[p] = ch.delays[p];
      }
      double2* yo = ch.y + br * g.L + (size_t)l * S + cp;
      double pr = 0.0;
#pragma unroll TXSW_UNROLL
      for (int q = 0; q < 8; ++q) {
        const int n = 512 * h + 64 * q + lane_f;
        double2 y = make_double2(0.0, 0.0);
#pragma unroll
        for (int p = 0; p < PM; ++p)
          if (p < np) y = cadd(y, cmul(cf[p], xs[64 * q + lane_f + 64 - dl[p]]));
        yo[n] = y;
        const double e = y.x * y.x + y.y * y.y;
        pr += e;
        if (n >= tail) pr += e;
      }
#if TXSW_FRAME
      if (h == 1 && lane_f < D) {
        // extended-symbol sample m = lane < max_delay: x_ext[m - d] is this
        // symbol's x[N - cp + m - d] (slot index 576 - cp + m - d) or, before
        // it, the previous symbol's x[N + m - d] (slot 9; zero for symbol 0)
        const int m = lane_f;
        double2 y = make_double2(0.0, 0.0);
#pragma unroll
        for (int p = 0; p < PM; ++p)
          if (p < np) {
            const int k = m - dl[p];
            const double2 xv = k >= 0 ? xs[576 - cp + k] : (l > 0 ? xs[64 * 10 + k] : make_double2(0.0, 0.0));
            y = cadd(y, cmul(cf[p], xv));
          }
        pr += y.x * y.x + y.y * y.y;
      }
#endif
      pwr[r] += pr;
    }
    wfft::wave_lds_fence();   // the window is restaged
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (r >= ch.num_rx) break;
    double t = pwr[r];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
    if (lane_f == 0) ch.pow_part[((size_t)b * ch.num_rx + r) * g.n_sym + l] = t;
  }
#if TXSW_FRAME
  tailp = v[15];
  }   // symbols
#endif
#else
#pragma unroll
  for (int q = 0; q < 16; ++q) xs[64 * q + lane_f] = cscale(v[q], sc);
  wfft::wave_lds_fence();
  if (D > 0) {   // the TX samples at both ends of the extended symbol (k_chan_fix)
    double2* xh = ch.xh + ((size_t)b * g.n_sym + l) * 2 * D;
    for (int i = lane_f; i < 2 * D; i += 64) {
      const int j = i < D ? i : S - 2 * D + i;
      xh[i] = xs[(j - cp) & (N - 1)];
    }
  }
  // 3. every RX's taps (transmit_simo, core/ofdm_core.py:361-412)
  for (int r = 0; r < ch.num_rx; ++r) {
    const size_t br = (size_t)b * ch.num_rx + r;
    double2 cf[PM];
    int dl[PM];
#pragma unroll
    for (int p = 0; p < PM; ++p) {
      cf[p] = p < np ? ch.coef[br * np + p] : make_double2(0.0, 0.0);
      dl[p] = ch.delays[p];
    }
    double2* yo = ch.y + br * g.L + (size_t)l * S + cp;
    double pwr = 0.0;
    // partly rolled: fully unrolled, the 16 x NP shifted reads were all hoisted (spills)
#pragma unroll TXSW_UNROLL
    for (int q = 0; q < 16; ++q) {
      const int n = 64 * q + lane_f;
      double2 y = make_double2(0.0, 0.0);
#pragma unroll
      for (int p = 0; p < PM; ++p)
        if (p < np) y = cadd(y, cmul(cf[p], xs[(n - dl[p]) & (N - 1)]));
      yo[n] = y;
      const double e = y.x * y.x + y.y * y.y;
      pwr += e;
      if (n >= tail) pwr += e;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) pwr += __shfl_xor(pwr, o);
    if (lane_f == 0) ch.pow_part[br * g.n_sym + l] = pwr;
  }
#endif
}

bool tx_simo_w_supported(const Grid& g, int f64, int coded, int sc_fdm, const TxChannelT<double>& ch) {
  return f64 && !coded && !sc_fdm && g.N == 1024 && g.kinfo && g.pilots64 && !ch.tcoef && !ch.x_out &&
         ch.n_paths >= 1 && ch.n_paths <= TXCH_MAXP && ch.max_delay >= 0 && ch.max_delay <= g.cp && g.cp < 1024 &&
         ch.num_rx >= 1 && (g.bps == 2 || g.bps == 4 || g.bps == 6) &&
         (!TXSW_HALF || (ch.max_delay <= 64 && g.cp <= 512 && ch.num_rx <= 4));
}
// the wave TX also forms the head samples' power (TXSW_FRAME): k_chan_fix must not run
bool tx_simo_w_fuses_fix(const Grid& g, int coded, int sc_fdm, const TxChannelT<double>& ch) {
  return TXSW_FRAME && simo_tx_wave_enabled() && tx_simo_w_supported(g, 1, coded, sc_fdm, ch);
}

// Which wave-private kernels run by default (same-box A/B, profiles/r6_wave_ab.md):
// the config-5 RX (k_rx_fft_mimo_w) beats its block kernel; the config-2 RX and
// TX do not (2 waves per SIMD at most with a symbol in registers, against 3 for
// the block kernels; the noise, the coded-bit gathers and the taps, not the
// FFT, set their time), so they are opt-in.  Env LTE_RX_WAVE / LTE_TX_WAVE /
// LTE_MIMO_RX_WAVE = 0 / 1 override.
#ifndef LTE_RX_WAVE
#define LTE_RX_WAVE 0
#endif
#ifndef LTE_MIMO_RX_WAVE
#define LTE_MIMO_RX_WAVE 1
#endif
static int env_or(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}
int rx_wave_enabled() { return env_or("LTE_RX_WAVE", LTE_RX_WAVE); }
int mimo_rx_wave_enabled() { return env_or("LTE_MIMO_RX_WAVE", LTE_MIMO_RX_WAVE); }
#ifndef LTE_SIMO_RX_WAVE
#define LTE_SIMO_RX_WAVE 1
#endif
int simo_rx_wave_enabled() { return env_or("LTE_SIMO_RX_WAVE", LTE_SIMO_RX_WAVE); }
#ifndef LTE_SIMO_TX_WAVE
#define LTE_SIMO_TX_WAVE 1
#endif
int simo_tx_wave_enabled() { return env_or("LTE_SIMO_TX_WAVE", LTE_SIMO_TX_WAVE); }

template <int BPS, int NP>
static void tx_simo_w_go(hipStream_t s, unsigned blocks, const Grid& g, const uint32_t* pw, int PW, int B,
                         double2* cap_syms, const TxChannelT<double>& ch) {
  hipLaunchKernelGGL((k_ofdm_tx_simo_w<BPS, NP>), dim3(blocks), dim3(64 * TXSW_WAVES),
                     (size_t)TXSW_WAVES * TXSW_XS * sizeof(double2), s, g, pw, PW, B, cap_syms, ch);
}
template <int BPS>
static void tx_simo_w_np(hipStream_t s, unsigned blocks, const Grid& g, const uint32_t* pw, int PW, int B,
                         double2* cap_syms, const TxChannelT<double>& ch) {
  if (ch.n_paths == 6) tx_simo_w_go<BPS, 6>(s, blocks, g, pw, PW, B, cap_syms, ch);
  else if (ch.n_paths == 4) tx_simo_w_go<BPS, 4>(s, blocks, g, pw, PW, B, cap_syms, ch);
  else tx_simo_w_go<BPS, 0>(s, blocks, g, pw, PW, B, cap_syms, ch);
}
int launch_ofdm_tx_simo_w(hipStream_t s, const Grid& g, const uint32_t* pw, int PW, int B, double2* cap_syms,
                          const TxChannelT<double>& ch) {
  if (!tx_simo_w_supported(g, 1, 0, 0, ch)) return (int)hipErrorInvalidValue;
  const int64_t waves = TXSW_FRAME ? (int64_t)B : (int64_t)B * g.n_sym;
  if (waves > 0x7FFFFFFF - TXSW_WAVES) return (int)hipErrorInvalidValue;
  const unsigned blocks = (unsigned)((waves + TXSW_WAVES - 1) / TXSW_WAVES);
  if (g.bps == 2) tx_simo_w_np<2>(s, blocks, g, pw, PW, B, cap_syms, ch);
  else if (g.bps == 4) tx_simo_w_np<4>(s, blocks, g, pw, PW, B, cap_syms, ch);
  else tx_simo_w_np<6>(s, blocks, g, pw, PW, B, cap_syms, ch);
  return (int)hipGetLastError();
}

int launch_rx_frame_simo_w(hipStream_t s, const Grid& g, int B, int num_rx, const double2* y, int64_t y_rx_stride,
                           int64_t y_frame_stride, const double* npow, const uint64_t* fid, uint64_t seed,
                           const double* inj_z, int64_t inj_stride, const uint32_t* pw, int PW, int n_bits,
                           uint32_t* frame_err, double2* cap_syms, uint8_t* cap_bits) {
  if (!rx_simo_w_supported(g, num_rx, 1, false, false, false)) return (int)hipErrorInvalidValue;
  const int yrow = g.Nd > SIMOW_ROW_MIN ? g.Nd : SIMOW_ROW_MIN;
  const size_t shm = ((size_t)SIMOW_WAVES * yrow + (size_t)num_rx * g.Np) * sizeof(double2) +
                     (size_t)2 * 64 * SIMOW_WAVES * sizeof(int2) + (size_t)g.Np * sizeof(double);
#define LTE_SIMOW(BPS_)                                                                                             \
  hipLaunchKernelGGL(k_rx_frame_simo_w<BPS_>, dim3(B), dim3(64 * SIMOW_WAVES), shm, s, g, B, num_rx, yrow, y,       \
                     y_rx_stride, y_frame_stride, npow, fid, seed, inj_z, inj_stride, pw, PW, n_bits, frame_err,    \
                     cap_syms, cap_bits)
  if (g.bps == 2) LTE_SIMOW(2);
  else if (g.bps == 4) LTE_SIMOW(4);
  else LTE_SIMOW(6);
#undef LTE_SIMOW
  return (int)hipGetLastError();
}

int launch_rx_frame_w(hipStream_t s, const Grid& g, int rayleigh, int B, const double2* y, int64_t y_frame_stride,
                      const double* npow, const double* snr_lin, const uint64_t* fid, uint64_t seed,
                      const double* inj_z, int64_t inj_stride, double* zo, double* nv_out, double2* cap_syms,
                      double2* H, double* pstats) {
  if (!rx_frame_w_supported(g, LTE_CHAIN_CODED, 1) || !nv_out) return (int)hipErrorInvalidValue;
  const size_t shm = (size_t)RXW_WAVES * wfft::LDS_DOUBLES * sizeof(double);
  (void)hipFuncSetAttribute((const void*)k_rx_frame_w, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  hipLaunchKernelGGL(k_rx_frame_w, dim3((B + RXW_WAVES - 1) / RXW_WAVES), dim3(64 * RXW_WAVES), shm, s, g, rayleigh,
                     B, y, y_frame_stride, npow, snr_lin, fid, seed, inj_z, inj_stride,
                     reinterpret_cast<double2*>(zo), nv_out, cap_syms, H, pstats);
  return (int)hipGetLastError();
}

#ifndef LTE_TX_WAVE
#define LTE_TX_WAVE 0
#endif
#ifndef TXW_STAGE_DEFAULT   // 1: the coded streams staged in the wave's LDS (LTE_TXW_STAGE overrides)
#define TXW_STAGE_DEFAULT 0
#endif
int tx_wave_enabled() { return env_or("LTE_TX_WAVE", LTE_TX_WAVE); }

template <int BPS, bool STAGE>
static int txf_w_go(hipStream_t s, const Grid& g, const uint32_t* enc, int enc_words, const int32_t* tx_map, int B,
                    double2* cap_syms, const TxChannelT<double>& ch) {
  const size_t shm = (size_t)TXW_WAVES * (TXW_XS + (STAGE ? 4 * (size_t)((enc_words + 3) & ~3) : 0));
  if (shm > 160 * 1024) return (int)hipErrorInvalidValue;
  auto k = k_ofdm_txf_w<BPS, 4, STAGE>;
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  hipLaunchKernelGGL(k, dim3((B + TXW_WAVES - 1) / TXW_WAVES), dim3(64 * TXW_WAVES), shm, s, g, enc, enc_words,
                     tx_map, B, cap_syms, ch);
  return (int)hipGetLastError();
}

int launch_ofdm_txf_w(hipStream_t s, const Grid& g, const uint32_t* enc, int enc_words, const int32_t* tx_map, int B,
                      double2* cap_syms, const TxChannelT<double>& ch) {
  if (!txf_w_supported(g, 1, ch.n_paths, ch.max_delay, ch.num_rx, ch.tcoef != nullptr)) return (int)hipErrorInvalidValue;
  const char* e = std::getenv("LTE_TXW_STAGE");
  const bool stage = e ? std::atoi(e) != 0 : TXW_STAGE_DEFAULT;
  if (stage) {
    if (g.bps == 2) return txf_w_go<2, true>(s, g, enc, enc_words, tx_map, B, cap_syms, ch);
    if (g.bps == 4) return txf_w_go<4, true>(s, g, enc, enc_words, tx_map, B, cap_syms, ch);
    return txf_w_go<6, true>(s, g, enc, enc_words, tx_map, B, cap_syms, ch);
  }
  if (g.bps == 2) return txf_w_go<2, false>(s, g, enc, enc_words, tx_map, B, cap_syms, ch);
  if (g.bps == 4) return txf_w_go<4, false>(s, g, enc, enc_words, tx_map, B, cap_syms, ch);
  return txf_w_go<6, false>(s, g, enc, enc_words, tx_map, B, cap_syms, ch);
}

int launch_rx_fft_mimo_w(hipStream_t s, const Grid& g, const MimoGrid& m, int B, const double2* y, const double* npow,
                         const uint64_t* fid, uint64_t seed, const double* inj_z, int64_t inj_stride, double2* Y,
                         double2* H) {
  if (!rx_fft_mimo_w_supported(g, m, 1, 1)) return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)B * m.num_rx;
  if (total > 0x7FFFFFFF - RXMW_WAVES) return (int)hipErrorInvalidValue;
  const size_t shm = (size_t)RXMW_WAVES * wfft::LDS_DOUBLES * sizeof(double);
  hipLaunchKernelGGL(k_rx_fft_mimo_w, dim3((unsigned)((total + RXMW_WAVES - 1) / RXMW_WAVES)), dim3(64 * RXMW_WAVES),
                     shm, s, g, m, B, y, npow, fid, seed, inj_z, inj_stride, Y, H);
  return (int)hipGetLastError();
}

}  // namespace lte
