// Shared device helpers for the gfx950 LTE PHY kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LTE_NEG_BIG (-1.0e30f)

// ---------------------------------------------------------------- RNG
// Philox4x32-10 (counter-based, stateless): every random number is a pure
// function of (seed, frame id, stream, index), so results do not depend on
// how frames are sharded over workgroups or GPUs.
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox4x32(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = {hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

enum : uint32_t {
  RNG_STREAM_BITS = 1u,
  RNG_STREAM_FADE = 0x100u,   // + rx*64 + tx
  RNG_STREAM_NOISE = 0x10000u, // + rx
  RNG_STREAM_MIMO_FADE = 0x20000u,  // + (rx*16 + tx)*16 + path
  RNG_STREAM_MIMO_LINK = 0x30000u,  // + rx*16 + tx : link noise (transmit_mimo) / flat link gain (spatial)
  RNG_STREAM_BF = 0x40000u,         // + rx*num_tx + tx : beamforming flat channel H
};

__device__ __forceinline__ u32x4 rng4(uint64_t seed, uint64_t frame, uint32_t stream, uint32_t idx) {
  return philox4x32({idx, stream, (uint32_t)frame, (uint32_t)(frame >> 32)},
                    (uint32_t)seed, (uint32_t)(seed >> 32));
}

// uniform in (0, 1]
__device__ __forceinline__ float u01(uint32_t v) { return ((v >> 8) + 1u) * (1.0f / 16777216.0f); }

// two standard normals from two uniforms (Box-Muller)
__device__ __forceinline__ float2 box_muller(uint32_t a, uint32_t b) {
  const float r = sqrtf(-2.0f * __logf(u01(a)));
  float s, c;
  __sincosf(6.2831853071795864f * u01(b), &s, &c);
  return make_float2(r * c, r * s);
}

// ---------------------------------------------------------------- complex
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cmulc(float2 a, float2 b) {  // a * conj(b)
  return make_float2(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y);
}
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
// Complex division with Smith's scaling (the algorithm NumPy's complex divide uses).
__device__ __forceinline__ float2 cdiv(float2 a, float2 b) {
  if (fabsf(b.x) >= fabsf(b.y)) {
    if (b.x == 0.0f && b.y == 0.0f) return make_float2(a.x / b.x, a.y / b.x);
    const float rat = b.y / b.x, scl = 1.0f / (b.x + b.y * rat);
    return make_float2((a.x + a.y * rat) * scl, (a.y - a.x * rat) * scl);
  }
  const float rat = b.x / b.y, scl = 1.0f / (b.y + b.x * rat);
  return make_float2((a.x * rat + a.y) * scl, (a.y * rat - a.x) * scl);
}

// ---------------------------------------------------------------- FFT
// Stockham radix-4 (+ one radix-2 stage when log2 N is odd) complex FFT held
// in LDS.  One transform of N points is done by T = N/8 threads (tid in
// [0,T)); every stage is register-staged (read -> barrier -> write ->
// barrier), so several transforms of the same N can share a workgroup.
// tw[e] = exp(-2*pi*i*e/N), e in [0, N).  Unscaled.  All threads of the
// workgroup must call it (it contains __syncthreads).
template <bool INV>
__device__ __forceinline__ float2 twid(const float2* __restrict__ tw, int e) {
  const float2 w = tw[e];
  return INV ? make_float2(w.x, -w.y) : w;
}

template <bool INV>
__device__ __forceinline__ void fft_lds(float2* buf, int N, int log2N, const float2* __restrict__ tw,
                                        int tid, bool active) {
  const int T = N >> 3;
  const int q4 = N >> 2;
  int Ns = 1, lNs = 0;   // Ns = 4^s; all index arithmetic is shifts (N, Ns powers of 2)
  const int n4 = log2N >> 1;
  for (int s = 0; s < n4; ++s) {
    float2 v[2][4];
    int jj[2];
    if (active) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int j = tid + q * T;
        jj[q] = j;
        const int k = j & (Ns - 1);
        const int step = 1 << (log2N - lNs - 2);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[q][r] = buf[j + r * q4];
#pragma unroll
        for (int r = 1; r < 4; ++r) v[q][r] = cmul(v[q][r], twid<INV>(tw, k * r * step));
        // radix-4 butterfly
        const float2 a0 = cadd(v[q][0], v[q][2]), a1 = csub(v[q][0], v[q][2]);
        const float2 a2 = cadd(v[q][1], v[q][3]), d = csub(v[q][1], v[q][3]);
        const float2 a3 = INV ? make_float2(-d.y, d.x) : make_float2(d.y, -d.x);
        v[q][0] = cadd(a0, a2);
        v[q][2] = csub(a0, a2);
        v[q][1] = cadd(a1, a3);
        v[q][3] = csub(a1, a3);
      }
    }
    __syncthreads();
    if (active) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int j = jj[q];
        const int idx = ((j >> lNs) << (lNs + 2)) + (j & (Ns - 1));
#pragma unroll
        for (int r = 0; r < 4; ++r) buf[idx + r * Ns] = v[q][r];
      }
    }
    __syncthreads();
    Ns <<= 2;
    lNs += 2;
  }
  if (log2N & 1) {  // final radix-2 stage (Ns == N/2)
    const int h = N >> 1;
    float2 v[4][2];
    int jj[4];
    if (active) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = tid + q * T;
        jj[q] = j;
        const int k = j & (Ns - 1);
        const int step = 1 << (log2N - lNs - 1);
        v[q][0] = buf[j];
        v[q][1] = cmul(buf[j + h], twid<INV>(tw, k * step));
        const float2 t0 = cadd(v[q][0], v[q][1]), t1 = csub(v[q][0], v[q][1]);
        v[q][0] = t0;
        v[q][1] = t1;
      }
    }
    __syncthreads();
    if (active) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = jj[q];
        const int idx = ((j >> lNs) << (lNs + 1)) + (j & (Ns - 1));
        buf[idx] = v[q][0];
        buf[idx + Ns] = v[q][1];
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- bits
// Packed bit streams are MSB-first: bit i of a stream lives in word i>>5 at
// bit position 31-(i&31).
__device__ __forceinline__ uint32_t getbit(const uint32_t* __restrict__ w, int64_t i) {
  return (w[i >> 5] >> (31 - (i & 31))) & 1u;
}
