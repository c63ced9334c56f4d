// Microbenchmark for the turbo decoder's HBM access shape: every wave streams
// its own regions (as a decoder wave streams its 64 code blocks' rows), three
// at once (the LS / LP / LE rows of a sweep), with 4, 8 or 16 B per lane per
// load instruction (256-B, 512-B or 1-KB wave requests).  Occupancy pinned to 3
// waves per SIMD (the decoder's, 133 VGPRs) with dynamic LDS, and unpinned.
// Prints GB/s per shape.
// Build: hipcc -O3 --offload-arch=gfx950 -o scripts/row_width_bench scripts/row_width_bench.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

template <int W>   // dwords per lane per load
__global__ __launch_bounds__(256) void k_stream3(const uint32_t* __restrict__ x, int64_t region_dw, int rows,
                                                 uint32_t* out) {
  extern __shared__ uint32_t pad[];
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t* r0 = x + (size_t)(3 * w + 0) * region_dw + lane * W;
  const uint32_t* r1 = x + (size_t)(3 * w + 1) * region_dw + lane * W;
  const uint32_t* r2 = x + (size_t)(3 * w + 2) * region_dw + lane * W;
  uint32_t acc = 0;
#pragma unroll 4
  for (int i = 0; i < rows; ++i) {
    const size_t o = (size_t)i * 64 * W;
    if constexpr (W == 1) {
      acc ^= r0[o] ^ r1[o] ^ r2[o];
    } else if constexpr (W == 2) {
      const uint2 a = *reinterpret_cast<const uint2*>(r0 + o), b = *reinterpret_cast<const uint2*>(r1 + o),
                  c = *reinterpret_cast<const uint2*>(r2 + o);
      acc ^= a.x ^ a.y ^ b.x ^ b.y ^ c.x ^ c.y;
    } else {
      const uint4 a = *reinterpret_cast<const uint4*>(r0 + o), b = *reinterpret_cast<const uint4*>(r1 + o),
                  c = *reinterpret_cast<const uint4*>(r2 + o);
      acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w;
    }
  }
  if (acc == 0x12345678u) out[w * 64 + lane] = acc + pad[0];
}

template <int W>
static double run(const uint32_t* x, int64_t region_dw, int waves, uint32_t* out, size_t lds) {
  const int rows = (int)(region_dw / (64 * W));
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(k_stream3<W>, dim3(waves / 4), dim3(256), lds, 0, x, region_dw, rows, out);   // warm
  (void)hipEventRecord(a, 0);
  for (int rep = 0; rep < 3; ++rep)
    hipLaunchKernelGGL(k_stream3<W>, dim3(waves / 4), dim3(256), lds, 0, x, region_dw, rows, out);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  return 3.0 * 3.0 * (double)waves * region_dw * 4 / (ms * 1e-3) / 1e9;
}

int main() {
  const int waves = 3072;                     // one generation at 3 waves / SIMD
  const int64_t region_dw = 64 * 4 * 1024;    // 1 MiB per region, 3 regions per wave: 9 GiB
  const size_t bytes = (size_t)3 * waves * region_dw * 4;
  uint32_t *x, *out;
  if (hipMalloc(&x, bytes) || hipMalloc(&out, (size_t)waves * 64 * 4)) {
    printf("alloc failed\n");
    return 1;
  }
  (void)hipMemset(x, 0, bytes);
  (void)hipDeviceSynchronize();
  const size_t lds = 52 * 1024;               // 3 blocks (= 3 waves per SIMD) per CU
  const double g1 = run<1>(x, region_dw, waves, out, lds);
  const double g2 = run<2>(x, region_dw, waves, out, lds);
  const double g4 = run<4>(x, region_dw, waves, out, lds);
  const double h1 = run<1>(x, region_dw, waves, out, 0);
  const double h4 = run<4>(x, region_dw, waves, out, 0);
  if (hipDeviceSynchronize() != hipSuccess) {
    printf("kernel failed\n");
    return 1;
  }
  printf("{\"GBs_256B_3wps\": %.1f, \"GBs_512B_3wps\": %.1f, \"GBs_1KB_3wps\": %.1f, \"GBs_256B_free\": %.1f, "
         "\"GBs_1KB_free\": %.1f}\n",
         g1, g2, g4, h1, h4);
  (void)hipFree(x);
  (void)hipFree(out);
  return 0;
}
