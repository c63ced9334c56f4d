// Chip-wide non-packed VALU throughput of the turbo decoder's instruction
// classes on MI355X: add / max in f32 and f64, many resident waves, 8
// independent dependency chains per lane.  Prints lane-ops/s per class; the
// bench.py roofline peaks (VALU_PEAK_OPS) are checked against these.
// build: hipcc -O3 --offload-arch=gfx950 -o scripts/valu_peak_bench scripts/valu_peak_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int CH = 8, ITERS = 4096;

template <class T, bool MAX>
__global__ __launch_bounds__(256) void k_valu(T* out, T s) {
  T a[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) a[c] = (T)(threadIdx.x + c);
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      if (MAX) a[c] = (a[c] > s ? a[c] : s) + (T)0;   // v_max + keep a dependency chain
      else a[c] = a[c] + s;
    }
    s = -s;
  }
  T t = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) t += a[c];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

template <class T, bool MAX>
static double run(const char* name, int blocks) {
  T* d;
  (void)hipMalloc(&d, (size_t)blocks * 256 * sizeof(T));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL((k_valu<T, MAX>), dim3(blocks), dim3(256), 0, 0, d, (T)1.0);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k_valu<T, MAX>), dim3(blocks), dim3(256), 0, 0, d, (T)1.0);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  // ops per lane per iteration: CH (add) or 2*CH (max + add)
  const double ops = 5.0 * blocks * 256.0 * ITERS * CH * (MAX ? 2 : 1);
  const double rate = ops / (ms * 1e-3);
  printf("{\"class\": \"%s\", \"lane_ops_per_s\": %.4e, \"ms\": %.3f}\n", name, rate, ms);
  (void)hipFree(d);
  return rate;
}

int main() {
  const int blocks = 256 * 4 * 8 / 4;   // 8 waves per SIMD over 256 CUs
  run<float, false>("v_add_f32", blocks);
  run<float, true>("v_max_f32+v_add_f32", blocks);
  run<double, false>("v_add_f64", blocks);
  run<double, true>("v_max_f64+v_add_f64", blocks);
  return 0;
}
