// PMC calibration for the turbo decoder's access pattern: every wave reads /
// writes 256-B rows (one dword per lane) through a buffer resource, strided
// over a buffer far larger than the 256 MiB Infinity Cache.  The known byte
// counts let FETCH_SIZE / WRITE_SIZE be converted to bytes for this width.
// Build: hipcc -O3 --offload-arch=gfx950 -o scripts/pmc_calib scripts/pmc_calib.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  void* pu = (void*)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32) |
                     __builtin_amdgcn_readfirstlane((uint32_t)a));
  return __builtin_amdgcn_make_buffer_rsrc(pu, (short)0, (int)bytes, 0x00020000);
}

// wave w owns rows [w*R, (w+1)*R) of 64 floats
__global__ __launch_bounds__(256) void k_read_rows(const float* x, int R, float* out) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t r = rsrc(x + (size_t)w * R * 64, (uint32_t)R * 256u);
  float acc = 0.0f;
#pragma unroll 4
  for (int i = 0; i < R; ++i) acc += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, lane * 4, i * 256, 0));
  if (acc == 1234.5f) out[w * 64 + lane] = acc;  // never true for the zero input: keeps the loads live
}

__global__ __launch_bounds__(256) void k_write_rows(float* x, int R) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t r = rsrc(x + (size_t)w * R * 64, (uint32_t)R * 256u);
  for (int i = 0; i < R; ++i) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)i), r, lane * 4, i * 256, 0);
}

int main() {
  const int waves = 8192, R = 1024;                 // 8192 * 1024 * 256 B = 2 GiB
  const size_t bytes = (size_t)waves * R * 256;
  float *x, *out;
  if (hipMalloc(&x, bytes) || hipMalloc(&out, (size_t)waves * 64 * 4)) { printf("alloc failed\n"); return 1; }
  (void)hipMemset(x, 0, bytes);
  (void)hipDeviceSynchronize();
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_read_rows, dim3(waves / 4), dim3(256), 0, 0, x, R, out);
    hipLaunchKernelGGL(k_write_rows, dim3(waves / 4), dim3(256), 0, 0, x, R);
  }
  if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
  printf("{\"calib_bytes_per_launch\": %zu}\n", bytes);
  (void)hipFree(x); (void)hipFree(out);
  return 0;
}
