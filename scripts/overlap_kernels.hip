// Probe: do an HBM-streaming kernel at one wave per SIMD (the decoder's
// occupancy: >256 registers) and an f64 VALU kernel (the front end's shape:
// 256 threads, 32 KB LDS, <=128 VGPRs) run concurrently on two streams?
// Build: hipcc --offload-arch=gfx950 -O3 scripts/overlap_kernels.hip -o scripts/overlap_kernels
// Run:   ./scripts/overlap_kernels [rows] [blocks_v] [iters] [passes]   (prints ms for D, V, D||V)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#ifndef DW
#define DW 1.0
#endif
#ifndef NACC
#define NACC 136
#endif
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

// decoder-like: each lane streams its own rows (stride 64 doubles per row
// group), a long dependent chain in registers, one wave per SIMD
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void k_stream(const double* __restrict__ in, double* __restrict__ out, int rows, int passes) {
  const size_t lane = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t nl = (size_t)gridDim.x * 256;
  double acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = 0.0;
  for (int ps = 0; ps < passes; ++ps)
  for (int r = 0; r < rows; r += 64) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      double v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = __builtin_nontemporal_load(in + (size_t)(r + 8 * u + j) * nl + lane);
#pragma unroll
      for (int i = u * (NACC / 8); i < (u + 1) * (NACC / 8); ++i)
        acc[i] = fmax(acc[i] + v[i & 7], acc[(i + 1) % NACC] - v[(i + 3) & 7]) * DW;
    }
    __builtin_nontemporal_store(acc[r & 63], out + (size_t)(r >> 6) * nl + lane);
  }
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[lane] = s;
}

// front-end-like: f64 FMA chains with LDS exchanges and barriers
__global__ __launch_bounds__(256) void k_valu(double* __restrict__ out, int iters) {
  __shared__ double buf[4096];
  const int t = threadIdx.x;
  double a = t * 1e-3 + blockIdx.x, b = 1.0 - t * 1e-4;
  for (int i = 0; i < 16; ++i) buf[t + 256 * i] = a + i;
  __syncthreads();
  for (int it = 0; it < iters; ++it) {
#pragma unroll 8
    for (int k = 0; k < 64; ++k) { a = fma(a, b, 1e-9); b = fma(b, a, -1e-9); }
    buf[(t * 17 + it) & 4095] += a;
    __syncthreads();
    a += buf[(t * 33 + it) & 4095] * 1e-12;
  }
  out[(size_t)blockIdx.x * 256 + t] = a + b;
}

int main(int argc, char** argv) {
  const int blocks_d = 1024, rows = argc > 1 ? std::atoi(argv[1]) : 4096;
  const int passes = argc > 4 ? std::atoi(argv[4]) : 20;
  const int blocks_v = argc > 2 ? std::atoi(argv[2]) : 4096, iters = argc > 3 ? std::atoi(argv[3]) : 200;
  const size_t nl = (size_t)blocks_d * 256;
  double *in, *out, *ov;
  CK(hipMalloc(&in, (size_t)rows * nl * 8));
  CK(hipMalloc(&out, (size_t)(rows / 8 + 1) * nl * 8));
  CK(hipMalloc(&ov, (size_t)blocks_v * 256 * 8));
  CK(hipMemset(in, 0, (size_t)rows * nl * 8));
  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](int which) {
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, sa));
    CK(hipStreamWaitEvent(sb, e0, 0));
    if (which & 1) k_stream<<<blocks_d, 256, 0, sa>>>(in, out, rows, passes);
    if (which & 2) k_valu<<<blocks_v, 256, 0, sb>>>(ov, iters);
    hipEvent_t eb;
    CK(hipEventCreate(&eb));
    CK(hipEventRecord(eb, sb));
    CK(hipStreamWaitEvent(sa, eb, 0));
    CK(hipEventRecord(e1, sa));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(eb));
    return ms;
  };
  run(3);
  const char* nm[4] = {"", "stream (D)", "valu (V)", "D || V"};
  for (int rep = 0; rep < 2; ++rep)
    for (int w = 1; w <= 3; ++w) std::printf("%s: %.2f ms\n", nm[w], run(w));
  std::printf("D bytes %.2f GB\n", (double)passes * rows * nl * 8 / 1e9);
  return 0;
}
