// Microbenchmark: the wave-private float64 2048- / 1024-point FFTs
// (csrc/lte_wfft.h) against the workgroup LDS FFT of the block kernels (fft_lds
// in csrc/lte_common.h, N / 8 threads per transform, a barrier per pass).
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../ofdm-lte_amd/csrc [-DWN=1024] wfft_bench.hip -o wfft_bench
//   ./wfft_bench [M transforms] [REP]
//
// Two modes per kernel: HBM (load, one transform, store) and compute (load,
// REP transforms on the same data, store).  Checks both kernels against each
// other and against a long-double DFT of a few transforms.  One JSON line per
// measurement.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "lte_wfft.h"

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

#ifndef WN
#define WN 2048
#endif
constexpr int N = WN, TL = N / 8, LOG2N = N == 2048 ? 11 : 10, MR = N / 64;
constexpr int WLDS = N == 2048 ? wfft::LDS_DOUBLES : wfft::LDS_DOUBLES_1024;
static_assert(N == 2048 || N == 1024, "wfft sizes");

template <bool INV, int REP>
__global__ __launch_bounds__(TL) void k_lds(const double2* __restrict__ in, double2* __restrict__ out,
                                             const double2* __restrict__ tw, int M) {
  extern __shared__ double2 buf[];
  const int t = blockIdx.x;
  if (t >= M) return;   // uniform per block
  const double2* x = in + (size_t)t * N;
#pragma unroll
  for (int r = 0; r < 8; ++r) buf[threadIdx.x + TL * r] = x[threadIdx.x + TL * r];
  __syncthreads();
#pragma unroll 1
  for (int rep = 0; rep < REP; ++rep) fft_lds<INV, N, false, true, false>(buf, N, LOG2N, tw, threadIdx.x, true);
  double2* y = out + (size_t)t * N;
#pragma unroll
  for (int r = 0; r < 8; ++r) y[threadIdx.x + TL * r] = buf[threadIdx.x + TL * r];
}

#ifndef WPE
#define WPE 2
#endif
template <bool INV, int REP, int W>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void k_wave(const double2* __restrict__ in, double2* __restrict__ out,
                                                 const double2* __restrict__ tw, int M) {
  extern __shared__ double lds_d[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int t = blockIdx.x * W + w;
  if (t >= M) return;   // uniform per wave; no barrier below
  double* lds = lds_d + w * WLDS;
  const double2* x = in + (size_t)t * N;
  double2 v[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) v[m] = x[64 * m + lane];
#pragma unroll 1
  for (int rep = 0; rep < REP; ++rep) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    if constexpr (N == 2048) wfft::fft2048<INV>(v, lds, tw, ln);
    else wfft::fft1024<INV>(v, lds, tw, ln);
  }
  double2* y = out + (size_t)t * N;
#pragma unroll
  for (int q = 0; q < MR; ++q) y[64 * q + lane] = v[q];
}

static double lcg(uint64_t& s) {
  s = s * 6364136223846793005ull + 1442695040888963407ull;
  return ((double)(s >> 11) / 9007199254740992.0) * 2.0 - 1.0;
}

template <class F>
static float timeit(F f, int iters) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 131072;
  const size_t n = (size_t)M * N;
  std::vector<double2> h(n), tw(N);
  uint64_t s = 12345;
  for (size_t i = 0; i < n; ++i) h[i] = make_double2(lcg(s), lcg(s));
  for (int e = 0; e < N; ++e) {
    const long double a = -2.0L * 3.14159265358979323846264338327950288L * e / N;
    tw[e] = make_double2((double)cosl(a), (double)sinl(a));
  }
  double2 *d_in, *d_a, *d_b, *d_tw;
  CK(hipMalloc(&d_in, n * 16));
  CK(hipMalloc(&d_a, n * 16));
  CK(hipMalloc(&d_b, n * 16));
  CK(hipMalloc(&d_tw, N * 16));
  CK(hipMemcpy(d_in, h.data(), n * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_tw, tw.data(), N * 16, hipMemcpyHostToDevice));

  auto run_lds = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(M), dim3(TL), N * 16, 0, d_in, d_a, d_tw, M); };
  auto run_wave = [&](auto kern, int W) {
    hipLaunchKernelGGL(kern, dim3((M + W - 1) / W), dim3(64 * W), W * WLDS * 8, 0, d_in, d_b, d_tw, M);
  };
  // correctness (forward and inverse, REP = 1)
  for (int inv = 0; inv < 2; ++inv) {
    if (inv) {
      run_lds(k_lds<true, 1>);
      run_wave(k_wave<true, 1, 4>, 4);
    } else {
      run_lds(k_lds<false, 1>);
      run_wave(k_wave<false, 1, 4>, 4);
    }
    CK(hipDeviceSynchronize());
    std::vector<double2> A(n), B(n);
    CK(hipMemcpy(A.data(), d_a, n * 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(B.data(), d_b, n * 16, hipMemcpyDeviceToHost));
    double dmax = 0, amax = 0;
    for (size_t i = 0; i < n; ++i) {
      dmax = fmax(dmax, fabs(A[i].x - B[i].x));
      dmax = fmax(dmax, fabs(A[i].y - B[i].y));
      amax = fmax(amax, fabs(A[i].x));
    }
    double ea = 0, eb = 0, xmax = 0;
    const int picks[3] = {0, M / 2, M - 1};
    for (int pi = 0; pi < 3; ++pi) {
      const size_t base = (size_t)picks[pi] * N;
      for (int k = 0; k < N; ++k) {
        long double re = 0, im = 0;
        for (int j = 0; j < N; ++j) {
          const long double a = (inv ? 2.0L : -2.0L) * 3.14159265358979323846264338327950288L *
                                (long double)((int64_t)j * k % N) / N;
          const long double c = cosl(a), sn = sinl(a);
          re += h[base + j].x * c - h[base + j].y * sn;
          im += h[base + j].x * sn + h[base + j].y * c;
        }
        ea = fmax(ea, (double)fabsl(A[base + k].x - re));
        ea = fmax(ea, (double)fabsl(A[base + k].y - im));
        eb = fmax(eb, (double)fabsl(B[base + k].x - re));
        eb = fmax(eb, (double)fabsl(B[base + k].y - im));
        xmax = fmax(xmax, (double)fabsl(re));
      }
    }
    printf("{\"N\": %d, \"check\": \"%s\", \"max_abs_lds_vs_wave\": %.3e, \"max_abs_out\": %.3e, "
           "\"err_lds_vs_ldouble\": %.3e, \"err_wave_vs_ldouble\": %.3e, \"ref_max\": %.3e}\n",
           N, inv ? "inverse" : "forward", dmax, amax, ea, eb, xmax);
  }
  // timing
  const double bytes = 2.0 * n * 16;
  auto line = [&](const char* k, int rep, float ms) {
    printf("{\"kernel\": \"%s\", \"N\": %d, \"M\": %d, \"rep\": %d, \"ms\": %.4f, \"GBps\": %.1f, \"ns_per_fft\": %.3f}\n", k, N, M,
           rep, ms, bytes / ms / 1e6, ms * 1e6 / ((double)M * rep));
  };
  line("lds", 1, timeit([&] { run_lds(k_lds<false, 1>); }, 10));
  line("wave_w4", 1, timeit([&] { run_wave(k_wave<false, 1, 4>, 4); }, 10));
  line("wave_w1", 1, timeit([&] { run_wave(k_wave<false, 1, 1>, 1); }, 10));
  line("wave_w2", 1, timeit([&] { run_wave(k_wave<false, 1, 2>, 2); }, 10));
  line("lds", 8, timeit([&] { run_lds(k_lds<false, 8>); }, 5));
  line("wave_w4", 8, timeit([&] { run_wave(k_wave<false, 8, 4>, 4); }, 5));
  line("wave_w1", 8, timeit([&] { run_wave(k_wave<false, 8, 1>, 1); }, 5));
  line("wave_w2", 8, timeit([&] { run_wave(k_wave<false, 8, 2>, 2); }, 5));
  CK(hipFree(d_in));
  CK(hipFree(d_a));
  CK(hipFree(d_b));
  CK(hipFree(d_tw));
  return 0;
}
