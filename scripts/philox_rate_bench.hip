// Chip-wide Philox4x32-10 throughput on MI355X in two instruction forms of
// the round's 32x32 products: (a) separate low / high halves (v_mul_lo_u32 +
// v_mul_hi_u32), (b) one 64-bit product (v_mad_u64_u32), plus the single
// instruction rates of each, for the channel kernels' noise cost.
// build: hipcc -O3 --offload-arch=gfx950 -o scripts/philox_rate_bench scripts/philox_rate_bench.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int CH = 4, ITERS = 256;
struct q4 { uint32_t x, y, z, w; };

template <bool WIDE>
__device__ __forceinline__ q4 philox(q4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t lo0, hi0, lo1, hi1;
    if (WIDE) {
      const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
      lo0 = (uint32_t)p0; hi0 = (uint32_t)(p0 >> 32);
      lo1 = (uint32_t)p1; hi1 = (uint32_t)(p1 >> 32);
    } else {
      lo0 = 0xD2511F53u * c.x; hi0 = __umulhi(0xD2511F53u, c.x);
      lo1 = 0xCD9E8D57u * c.z; hi1 = __umulhi(0xCD9E8D57u, c.z);
    }
    c = {hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

template <bool WIDE>
__global__ __launch_bounds__(256) void k_philox(uint32_t* out, uint32_t seed) {
  uint32_t acc = 0;
  const uint32_t id = blockIdx.x * 256 + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const q4 r = philox<WIDE>({id, (uint32_t)(i * CH + c), 7u, 0u}, seed, ~seed);
      acc ^= r.x ^ r.y ^ r.z ^ r.w;
    }
  }
  out[id] = acc;
}

// single-instruction chains: 0 mul_lo, 1 mul_hi, 2 64-bit product, 3 f64 fma
template <int OP>
__global__ __launch_bounds__(256) void k_op(uint64_t* out, uint32_t s) {
  constexpr int NC = 8;
  uint64_t a[NC];
  double f[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) { a[c] = threadIdx.x + c; f[c] = (double)(threadIdx.x + c); }
  for (int i = 0; i < ITERS * 16; ++i) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (OP == 0) a[c] = (uint32_t)a[c] * s;
      if (OP == 1) a[c] = __umulhi((uint32_t)a[c], s);
      if (OP == 2) a[c] = (uint64_t)(uint32_t)a[c] * s + (a[c] >> 32);
      if (OP == 3) f[c] = fma(f[c], 1.0000001, 0.5);
    }
  }
  uint64_t t = 0;
#pragma unroll
  for (int c = 0; c < NC; ++c) t += a[c] + (uint64_t)f[c];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

template <class K>
static float time_it(K launch) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  launch();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) launch();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  const int blocks = 256 * 4 * 8 / 4;   // 8 waves per SIMD over 256 CUs
  uint64_t* d;
  (void)hipMalloc(&d, (size_t)blocks * 256 * sizeof(uint64_t));
  const double lanes = blocks * 256.0;
  float ms = time_it([&] { hipLaunchKernelGGL(k_philox<false>, dim3(blocks), dim3(256), 0, 0, (uint32_t*)d, 5u); });
  printf("{\"form\": \"philox mul_lo+mul_hi\", \"draws_per_s\": %.4e, \"ms\": %.3f}\n", lanes * ITERS * CH / (ms * 1e-3), ms);
  ms = time_it([&] { hipLaunchKernelGGL(k_philox<true>, dim3(blocks), dim3(256), 0, 0, (uint32_t*)d, 5u); });
  printf("{\"form\": \"philox 64-bit product\", \"draws_per_s\": %.4e, \"ms\": %.3f}\n", lanes * ITERS * CH / (ms * 1e-3), ms);
  const char* names[4] = {"v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32 (+add)", "v_fma_f64"};
  for (int op = 0; op < 4; ++op) {
    auto L = [&] {
      if (op == 0) hipLaunchKernelGGL(k_op<0>, dim3(blocks), dim3(256), 0, 0, d, 3u);
      if (op == 1) hipLaunchKernelGGL(k_op<1>, dim3(blocks), dim3(256), 0, 0, d, 3u);
      if (op == 2) hipLaunchKernelGGL(k_op<2>, dim3(blocks), dim3(256), 0, 0, d, 3u);
      if (op == 3) hipLaunchKernelGGL(k_op<3>, dim3(blocks), dim3(256), 0, 0, d, 3u);
    };
    ms = time_it(L);
    printf("{\"op\": \"%s\", \"lane_ops_per_s\": %.4e, \"ms\": %.3f}\n", names[op], lanes * ITERS * 16 * 8 / (ms * 1e-3), ms);
  }
  (void)hipFree(d);
  return 0;
}
