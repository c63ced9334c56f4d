// Cost breakdown of the receiver front end's float64 work on MI355X, each
// part run over the work of 65 536 config-2 subframes (14 x 2048 noisy
// samples, 14 N = 2048 FFTs, 13 986 ZF divisions per subframe):
//   philox        Philox4x32-10 only (one call per pair of samples)
//   bm64_ocml     Philox + float64 Box-Muller with OCML log / sqrt / sincospi
//   bm64_table    Philox + the table-driven float64 Box-Muller (lte_common.h)
//   fft64 / fft32 the LDS radix-8 FFT (fft_lds<false, 2048>), one per block
//   cdiv64        NumPy's complex division (Smith) per RE
// and the accuracy of the table-driven Box-Muller against the OCML one.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I ofdm-lte_amd/csrc -o scripts/rx_parts_bench scripts/rx_parts_bench.hip
#include "lte_common.h"
#include <cmath>
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <vector>

constexpr int FRAMES = 65536, NSYM = 14, N = 2048;
constexpr long long PAIRS = (long long)FRAMES * NSYM * N / 2;
constexpr int PPT = 56;   // pairs per thread
constexpr long long THREADS = PAIRS / PPT;

template <int V>
__global__ __launch_bounds__(256) void k_noise(double* out, uint64_t seed) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  double acc = 0.0;
  uint32_t xacc = 0;
  for (int i = 0; i < PPT; ++i) {
    const u32x4 r = rng4(seed, (uint64_t)blockIdx.x, RNG_STREAM_NOISE, (uint32_t)(i * 256 + threadIdx.x));
    if (V == 0) {
      xacc ^= r.x ^ r.y ^ r.z ^ r.w;
    } else if (V == 1) {
      const double2 a = box_muller64(r.x, r.y), b = box_muller64(r.z, r.w);
      acc += (a.x + a.y) + (b.x + b.y);
    } else {
      const double2 a = box_muller64t(r.x, r.y), b = box_muller64t(r.z, r.w);
      acc += (a.x + a.y) + (b.x + b.y);
    }
  }
  out[t] = acc + (double)xacc;
}

template <class R, bool TWR = false, int REP = 1>
__global__ __launch_bounds__(256) void k_fft(const cx<R>* __restrict__ tw, double* out) {
  extern __shared__ double2 lds_raw[];
  cx<R>* buf = reinterpret_cast<cx<R>*>(lds_raw);
  const int tid0 = threadIdx.x;
  double acc = 0.0;
  for (int rep = 0; rep < REP; ++rep) {   // REP FFTs per block in sequence (the per-frame kernels' shape)
    int tid = tid0;
    asm volatile("" : "+v"(tid));
    for (int k = tid; k < N; k += 256) buf[k] = mkc((R)(k ^ (blockIdx.x + rep)), (R)(k - (int)blockIdx.x));
    __syncthreads();
    fft_lds<false, N, false, TWR>(buf, N, 11, tw, tid, true);
    acc += (double)buf[tid].x;
    __syncthreads();
  }
  out[(size_t)blockIdx.x * 256 + tid0] = acc;
}

__global__ __launch_bounds__(256) void k_cdiv(const double2* __restrict__ h, double* out, int per) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  double acc = 0.0;
  for (int i = 0; i < per; ++i) {
    const double2 y = make_double2(1.0 + i, 0.5 * t);
    const double2 z = cdiv(y, h[(threadIdx.x + i) & 1023]);
    acc += z.x + z.y;
  }
  out[t] = acc;
}

// accuracy: both Box-Mullers on the same Philox words
__global__ void k_acc(double* err, int n) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= n) return;
  const u32x4 r = rng4(7, 3, RNG_STREAM_NOISE, (uint32_t)t);
  // include the extremes of the uniform range
  uint32_t a = r.x, b = r.y;
  if (t < 64) a = (uint32_t)t;
  else if (t < 128) a = 0xFFFFFFFFu - (uint32_t)(t - 64);
  if (t >= 128 && t < 1152) b = (uint32_t)(t - 128) << 22;
  const double2 p = box_muller64(a, b), q = box_muller64t(a, b);
  const double sc = fmax(1.0, fmax(fabs(p.x), fabs(p.y)));
  err[t] = fmax(fabs(p.x - q.x), fabs(p.y - q.y)) / sc;
}

static float timeit(void (*fn)(void*), void* arg) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  fn(arg);
  if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); std::exit(1); }
  (void)hipEventRecord(e0);
  fn(arg);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

struct Ctx {
  double* out;
  double2* tw64;
  float2* tw32;
  double2* h;
};

int main() {
  Ctx c;
  // the largest grid: the FFT kernels' FRAMES * NSYM / 8 blocks x 256 outputs
  const size_t nout = std::max<size_t>((size_t)THREADS, (size_t)FRAMES * NSYM / 8 * 256);
  if (hipMalloc(&c.out, nout * sizeof(double)) != hipSuccess) return 1;
  (void)hipMalloc(&c.tw64, N * sizeof(double2));
  (void)hipMalloc(&c.tw32, N * sizeof(float2));
  (void)hipMalloc(&c.h, 1024 * sizeof(double2));
  std::vector<double2> tw(N);
  std::vector<float2> twf(N);
  for (int e = 0; e < N; ++e) {
    tw[e] = make_double2(std::cos(-2 * M_PI * e / N), std::sin(-2 * M_PI * e / N));
    twf[e] = make_float2((float)tw[e].x, (float)tw[e].y);
  }
  std::vector<double2> hh(1024);
  for (int i = 0; i < 1024; ++i) hh[i] = make_double2(std::cos(i * 0.37) * (1 + i % 7), std::sin(i * 0.61) * (1 + i % 5));
  (void)hipMemcpy(c.tw64, tw.data(), N * sizeof(double2), hipMemcpyHostToDevice);
  (void)hipMemcpy(c.tw32, twf.data(), N * sizeof(float2), hipMemcpyHostToDevice);
  (void)hipMemcpy(c.h, hh.data(), 1024 * sizeof(double2), hipMemcpyHostToDevice);
  const unsigned nb = (unsigned)(THREADS / 256);
  auto p0 = [](void* a) { hipLaunchKernelGGL(k_noise<0>, dim3((unsigned)(THREADS / 256)), dim3(256), 0, 0, ((Ctx*)a)->out, 0x5EEDull); };
  auto p1 = [](void* a) { hipLaunchKernelGGL(k_noise<1>, dim3((unsigned)(THREADS / 256)), dim3(256), 0, 0, ((Ctx*)a)->out, 0x5EEDull); };
  auto p2 = [](void* a) { hipLaunchKernelGGL(k_noise<2>, dim3((unsigned)(THREADS / 256)), dim3(256), 0, 0, ((Ctx*)a)->out, 0x5EEDull); };
  auto f64 = [](void* a) {
    hipLaunchKernelGGL(k_fft<double>, dim3(FRAMES * NSYM / 8), dim3(256), N * sizeof(double2), 0, ((Ctx*)a)->tw64, ((Ctx*)a)->out);
  };
  auto f32 = [](void* a) {
    hipLaunchKernelGGL(k_fft<float>, dim3(FRAMES * NSYM / 8), dim3(256), N * sizeof(float2), 0, ((Ctx*)a)->tw32, ((Ctx*)a)->out);
  };
  auto f64t = [](void* a) {
    hipLaunchKernelGGL((k_fft<double, true>), dim3(FRAMES * NSYM / 8), dim3(256), N * sizeof(double2), 0, ((Ctx*)a)->tw64, ((Ctx*)a)->out);
  };
  auto f64r = [](void* a) {   // 14 FFTs per block (one frame's symbols)
    hipLaunchKernelGGL((k_fft<double, false, 14>), dim3(FRAMES / 8), dim3(256), N * sizeof(double2), 0, ((Ctx*)a)->tw64, ((Ctx*)a)->out);
  };
  auto f64rt = [](void* a) {
    hipLaunchKernelGGL((k_fft<double, true, 14>), dim3(FRAMES / 8), dim3(256), N * sizeof(double2), 0, ((Ctx*)a)->tw64, ((Ctx*)a)->out);
  };
  auto cd = [](void* a) {
    hipLaunchKernelGGL(k_cdiv, dim3(FRAMES * 14 / 256), dim3(256), 0, 0, ((Ctx*)a)->h, ((Ctx*)a)->out, 999 / 8);
  };
  (void)nb;
  const float t0 = timeit(p0, &c), t1 = timeit(p1, &c), t2 = timeit(p2, &c);
  // FFTs: 1/8 of the subframes' FFTs timed, scaled by 8
  const float t3 = 8 * timeit(f64, &c), t4 = 8 * timeit(f32, &c);
  const float t3t = 8 * timeit(f64t, &c), t3r = 8 * timeit(f64r, &c), t3rt = 8 * timeit(f64rt, &c);
  // divisions: FRAMES*14/256 blocks * 256 threads * 124 = 1/8 of 13 986 per subframe, scaled by 8
  const float t5 = 8 * timeit(cd, &c);
  printf("{\"part\": \"philox\", \"ms_per_65536_subframes\": %.3f}\n", t0);
  printf("{\"part\": \"bm64_ocml\", \"ms_per_65536_subframes\": %.3f}\n", t1);
  printf("{\"part\": \"bm64_table\", \"ms_per_65536_subframes\": %.3f}\n", t2);
  printf("{\"part\": \"fft64\", \"ms_per_65536_subframes\": %.3f}\n", t3);
  printf("{\"part\": \"fft32\", \"ms_per_65536_subframes\": %.3f}\n", t4);
  printf("{\"part\": \"fft64_twr\", \"ms_per_65536_subframes\": %.3f}\n", t3t);
  printf("{\"part\": \"fft64_14_per_block\", \"ms_per_65536_subframes\": %.3f}\n", t3r);
  printf("{\"part\": \"fft64_14_per_block_twr\", \"ms_per_65536_subframes\": %.3f}\n", t3rt);
  printf("{\"part\": \"cdiv64\", \"ms_per_65536_subframes\": %.3f}\n", t5);
  const int n = 1 << 22;
  hipLaunchKernelGGL(k_acc, dim3(n / 256), dim3(256), 0, 0, c.out, n);
  std::vector<double> err(n);
  (void)hipMemcpy(err.data(), c.out, n * sizeof(double), hipMemcpyDeviceToHost);
  double mx = 0;
  for (double e : err) mx = std::fmax(mx, e);
  printf("{\"bm64_table_max_err_vs_ocml\": %.3e, \"samples\": %d}\n", mx, n);
  return 0;
}
