// Microbenchmark: HBM write bandwidth of a pure store stream on MI355X --
// 16-B stores per lane (1 KB per wave instruction), plain against nontemporal
// (__builtin_nontemporal_store), and a read + write copy for reference.
//   hipcc -O3 --offload-arch=gfx950 wbw_bench.hip -o wbw_bench && ./wbw_bench [MiB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef double dv2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s\n", hipGetErrorString(e_)); exit(1); } } while (0)

template <bool NT>
__global__ __launch_bounds__(256) void k_write(double2* __restrict__ y, size_t n, int per) {
  const size_t base = ((size_t)blockIdx.x * per) * 256 + threadIdx.x;
  const double2 v = make_double2((double)threadIdx.x, 1.0);
  for (int i = 0; i < per; ++i) {
    const size_t k = base + (size_t)i * 256;
    if (k < n) {
      if constexpr (NT) __builtin_nontemporal_store(dv2{v.x, v.y}, reinterpret_cast<dv2*>(y + k));
      else y[k] = v;
    }
  }
}
template <bool NT>
__global__ __launch_bounds__(256) void k_copy(const double2* __restrict__ x, double2* __restrict__ y, size_t n, int per) {
  const size_t base = ((size_t)blockIdx.x * per) * 256 + threadIdx.x;
  for (int i = 0; i < per; ++i) {
    const size_t k = base + (size_t)i * 256;
    if (k < n) {
      const double2 v = x[k];
      if constexpr (NT) __builtin_nontemporal_store(dv2{v.x, v.y}, reinterpret_cast<dv2*>(y + k));
      else y[k] = v;
    }
  }
}

int main(int argc, char** argv) {
  const size_t mib = argc > 1 ? atol(argv[1]) : 4096;
  const size_t n = mib * 1024 * 1024 / 16;
  double2 *x, *y;
  CK(hipMalloc(&x, n * 16));
  CK(hipMalloc(&y, n * 16));
  CK(hipMemset(x, 0, n * 16));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int per : {1, 4, 16}) {
    const unsigned blocks = (unsigned)((n + 256 * per - 1) / (256 * per));
    auto run = [&](const char* name, auto f, double bytes) {
      f();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a));
      for (int r = 0; r < 5; ++r) f();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      ms /= 5;
      printf("{\"kernel\": \"%s\", \"per_thread\": %d, \"MiB\": %zu, \"ms\": %.3f, \"GBps\": %.1f}\n", name, per, mib, ms,
             bytes / ms / 1e6);
    };
    run("write", [&] { hipLaunchKernelGGL(k_write<false>, dim3(blocks), dim3(256), 0, 0, y, n, per); }, n * 16.0);
    run("write_nt", [&] { hipLaunchKernelGGL(k_write<true>, dim3(blocks), dim3(256), 0, 0, y, n, per); }, n * 16.0);
    run("copy", [&] { hipLaunchKernelGGL(k_copy<false>, dim3(blocks), dim3(256), 0, 0, x, y, n, per); }, n * 32.0);
    run("copy_nt", [&] { hipLaunchKernelGGL(k_copy<true>, dim3(blocks), dim3(256), 0, 0, x, y, n, per); }, n * 32.0);
  }
  return 0;
}
