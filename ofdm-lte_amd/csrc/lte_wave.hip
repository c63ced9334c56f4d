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
// data RE's equaliser terms (ZfCoef: rat, sre in LDS by data ordinal, the swap
// flag as bit q of a per-lane mask) and sigma^2_eff (nvo) are formed once per
// group, exactly as k_rx_frame forms them (same chest_interp / ZfCoef / abs2_ref
// code, so the same bits for the same FFT output).  The transform's rounding
// differs from fft_lds's (both within a few 1e-14 of the exact DFT:
// profiles/r6_wfft_microbench_wpe*.jsonl).
// LDS per wave: the transpose buffer (16.5 KB) + Nd x 16 B coefficients (16 KB
// at 20 MHz), so one wave per SIMD (four per CU); the full register file (512
// VGPRs + AGPRs) is the wave's.
#ifndef RXW_EXP   // register-pressure probes (wrong outputs): 1 no noise, 2 no FFT
#define RXW_EXP 0
#endif
#ifndef RXW_WPE   // register budget: waves per SIMD the compiler schedules for (LDS allows 1)
#define RXW_WPE 2
#endif
constexpr int RXW_WAVES = 4;
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
  double* tl = reinterpret_cast<double*>(dyn_lds<double2>()) + (size_t)w * (wfft::LDS_DOUBLES + 2 * g.Nd);
  double2* cf = reinterpret_cast<double2*>(tl + wfft::LDS_DOUBLES);
  __syncthreads();   // the Box-Muller tables (the only block barrier)
  if (b >= B) return;
  const double sigma = sqrt(npow[b] / 2.0);
  const double s2 = 1.0 / snr_lin[b];
  const uint64_t fr = fid[b];
  const double* zf = inj_z ? inj_z + (size_t)b * inj_stride : nullptr;
  const double2* yf = y + (size_t)b * y_frame_stride;
  const size_t fre = (size_t)b * g.n_sym * g.Nd;
  const double sc = rx_scale<double>(N);
  const bool odd = lane0 & 1;
  uint32_t swpm = 0;
  for (int l = 0; l < g.n_sym; ++l) {
    // lane made opaque per symbol: the twiddle / address arithmetic derived
    // from it is recomputed each symbol instead of hoisted and held live (spills)
    int lane = lane0;
    asm volatile("" : "+v"(lane));
    const int off = l * (N + g.cp) + g.cp;
    double2 v[32];
#pragma unroll
    for (int m = 0; m < 32; ++m) v[m] = yf[off + 64 * m + lane];
    // The noise, half a symbol at a time (registers 16 h .. 16 h + 15): a
    // rolled loop draws it into the wave's LDS scratch, then each register adds
    // its draw.  (Unrolled over the registers, the 16 Philox + 32 Box-Muller
    // chains took the kernel past 512 registers.)
    double2* zs = reinterpret_cast<double2*>(tl);   // [16][64]
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (zf) {
#pragma unroll 1
        for (int mm = 0; mm < 16; ++mm) {
          const int n = off + 64 * (16 * h + mm) + lane;
          zs[64 * mm + lane] = make_double2(zf[n], zf[g.L + n]);
        }
      } else {
#pragma unroll 1
        for (int mm = 0; mm < 16; mm += 2) {
          // even lanes: the pair counter of register m; odd lanes: of register m + 1
          const int m = 16 * h + mm;
          const uint32_t ctr = (uint32_t)((off + 64 * m + (odd ? 64 : 0) + lane) >> 1);
          const u32x4 r = rng4(seed, fr, RNG_STREAM_NOISE, ctr);
          const uint32_t t0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)(odd ? r.x : r.z), 0xB1, 0xF, 0xF, true);
          const uint32_t t1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)(odd ? r.y : r.w), 0xB1, 0xF, 0xF, true);
          zs[64 * mm + lane] = gauss2t<double>(odd ? t0 : r.x, odd ? t1 : r.y, bmt);
          zs[64 * (mm + 1) + lane] = gauss2t<double>(odd ? r.z : t0, odd ? r.w : t1, bmt);
        }
      }
      wfft::wave_lds_fence();
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const double2 z = zs[64 * i + lane];
        v[16 * h + i] = make_double2(v[16 * h + i].x + sigma * z.x, v[16 * h + i].y + sigma * z.y);
      }
      wfft::wave_lds_fence();
    }
#if RXW_EXP & 32
    for (int m = 0; m < 32; ++m) zo[fre + (size_t)l * 2048 + 64 * m + lane] = v[m];
    continue;
#endif
    // and again before the transform, so its twiddle loads are not hoisted
    // above the noise (48 more registers live across it)
    int lane_f = lane;
    asm volatile("" : "+v"(lane_f));
    if (!(RXW_EXP & 2)) wfft::fft2048<false>(v, tl, G::tw(g), lane_f);
    if (!(RXW_EXP & 16) && l % 14 == 0) {   // group estimate from its first symbol (lte_receiver.py:360-411)
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
        for (int k = lane; k < N; k += 64) Hf[k] = chest_interp<double>(g, hp, k);
      }
      // rolled (kinfo re-read): the interpolation and ZfCoef code once, not per register
      swpm = 0;
      const size_t nvg = ((size_t)b * g.n_grp + grp) * g.Nd;
#pragma unroll 1
      for (int q = 0; q < 32; ++q) {
        const int k = 64 * q + lane, j = g.kinfo[k];
        if (j < 0) continue;
        const double2 h = chest_interp<double>(g, hp, k);
        ZfCoef<double> zc;
        zc.set(make_double2(h.x + 1e-6, h.y));
        cf[j] = make_double2(zc.rat, zc.sre);
        swpm |= (uint32_t)zc.swp << q;
        const double den = abs2_ref(h);
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
      wfft::wave_lds_fence();   // coefficients visible; the scratch is the next transform's
    }
    // the bins' roles re-read per symbol (L1-resident 8 KB table; held in
    // registers they were widened to 64-bit addresses and spilled)
    const size_t fl = fre + (size_t)l * g.Nd;
#pragma unroll
    for (int q = 0; q < ((RXW_EXP & 8) ? 0 : 32); ++q) {
      const int j = g.kinfo[64 * q + lane];
      if (j >= 0) {
        const double2 c = cf[j];
        ZfCoef<double> zc;
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

#ifndef LTE_RX_WAVE   // 1: k_rx_frame_w where it applies (env LTE_RX_WAVE=0 / 1 overrides)
#define LTE_RX_WAVE 1
#endif
int rx_wave_enabled() {
  const char* e = std::getenv("LTE_RX_WAVE");
  return e ? std::atoi(e) : LTE_RX_WAVE;
}

int launch_rx_frame_w(hipStream_t s, const Grid& g, int rayleigh, int B, const double2* y, int64_t y_frame_stride,
                      const double* npow, const double* snr_lin, const uint64_t* fid, uint64_t seed,
                      const double* inj_z, int64_t inj_stride, double* zo, double* nv_out, double2* cap_syms,
                      double2* H, double* pstats) {
  if (!rx_frame_w_supported(g, LTE_CHAIN_CODED, 1) || !nv_out) return (int)hipErrorInvalidValue;
  const size_t shm = (size_t)RXW_WAVES * (wfft::LDS_DOUBLES * sizeof(double) + (size_t)g.Nd * sizeof(double2));
  if (shm + BM_LDS_BYTES > 160 * 1024) return (int)hipErrorInvalidValue;
  (void)hipFuncSetAttribute((const void*)k_rx_frame_w, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  hipLaunchKernelGGL(k_rx_frame_w, dim3((B + RXW_WAVES - 1) / RXW_WAVES), dim3(64 * RXW_WAVES), shm, s, g, rayleigh,
                     B, y, y_frame_stride, npow, snr_lin, fid, seed, inj_z, inj_stride,
                     reinterpret_cast<double2*>(zo), nv_out, cap_syms, H, pstats);
  return (int)hipGetLastError();
}

}  // namespace lte
