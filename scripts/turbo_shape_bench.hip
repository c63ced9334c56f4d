// Microbenchmark: the f64 turbo decoder's HBM access shape with the
// arithmetic removed -- the measured ceiling of k_turbo64's row stream.
//
// Same geometry as k_turbo64 (lte_decoder.hip, LTE_TURBO_ILV = 1): one wave
// per SIMD (a 256-thread block holds 96 KB of LDS, so one block = 4 waves per
// CU), a wave = 64 code blocks of one K, 512-B rows [row][64 lanes] f64, LS /
// LE interleaved ([2k] LS, [2k+1] LE), LP1 / LP2 after them; per half
// iteration a forward sweep of 8-step windows (3 rows per step: LS, LP, LE;
// decoder 2 at the QPP address pi(k), wave-uniform), an alpha checkpoint of 8
// rows stored every 24 steps, then a backward sweep of 24-step super-windows
// (8 checkpoint rows + 3 x 24 input rows loaded, 24 extrinsic rows stored);
// 8 iterations + the final pass; the first pass skips the LE loads.  Config 2
// at 65 536 frames: 5 jobs (K = 5568 x 4, 5632), 1 024 waves each.
//
// The loaded values are folded with XOR into what is stored, so no load can be
// dropped.  Prints bytes moved per launch and GB/s, for the decoder's shape
// with and without the checkpoint rows, and with two waves per SIMD; _seq:
// decoder 2 addressed in natural order (what a QPP-free layout would reach).
// Build: hipcc -O3 --offload-arch=gfx950 -o scripts/turbo_shape_bench scripts/turbo_shape_bench.hip
// Usage: turbo_shape_bench [frames] [decoder]   (decoder: the decoder's layout only, one JSON line)
// (-DLTE_SHAPE_AUX=3: the decoder's sc0|nt policy, LTE_TURBO_CPOL).  The
// CH lines place the rows of CH consecutive waves side by side, as the decoder
// does since round 3 (TURBO_CH = 32, lte_internal.h); "decoder_layout" is that
// shape at one / two / three waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
// row stride in bytes: 512 (a wave's rows contiguous) or CH x 512 (rows of CH
// consecutive waves side by side: [chunk][row][wave in chunk][lane])
// cache-policy bits of the row loads / stores (LTE_SHAPE_AUX: 0 default, 1 glc,
// 2 slc, 3 glc|slc); LTE_SHAPE_NOST: the extrinsic and checkpoint stores
// dropped (reads only; the "decoder" mode also runs that variant at run time)
#ifndef LTE_SHAPE_AUX
#define LTE_SHAPE_AUX 0
#endif
#ifndef LTE_SHAPE_AUXL
#define LTE_SHAPE_AUXL LTE_SHAPE_AUX
#endif
#ifndef LTE_SHAPE_AUXS
#define LTE_SHAPE_AUXS LTE_SHAPE_AUX
#endif
#ifndef LTE_SHAPE_NOST
#define LTE_SHAPE_NOST 0
#endif
// LTE_SHAPE_SEPLE: LS rows [0, K), LE rows [K, 2K) (not interleaved);
// LTE_SHAPE_XCD: a chunk's groups taken from blocks on one XCD (blocks are
// dispatched round-robin over the 8 XCDs), within windows of 64 blocks
#ifndef LTE_SHAPE_SEPLE
#define LTE_SHAPE_SEPLE 0
#endif
#ifndef LTE_SHAPE_XCD
#define LTE_SHAPE_XCD 0
#endif
// LTE_SHAPE_CKCH1: checkpoint rows of each group contiguous (not chunked);
// LTE_SHAPE_SYNC: the block's 4 waves meet at a barrier every 24 steps
#ifndef LTE_SHAPE_CKCH1
#define LTE_SHAPE_CKCH1 0
#endif
#ifndef LTE_SHAPE_SYNC
#define LTE_SHAPE_SYNC 0
#endif
#define RSC(rs) (LTE_SHAPE_CKCH1 ? 512 : (rs))
#define ROW_LS(p) (LTE_SHAPE_SEPLE ? (p) : 2 * (p))
#define ROW_LE(p) (LTE_SHAPE_SEPLE ? K + (p) : 2 * (p) + 1)
__device__ __forceinline__ uint64_t ld(__amdgpu_buffer_rsrc_t r, int vo, int row, int rs) {
  return __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(r, vo, row * rs, LTE_SHAPE_AUXL));
}
template <bool NOST = false>
__device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t r, int vo, int row, uint64_t v, int rs) {
  if ((NOST || LTE_SHAPE_NOST) && v != 0x0123456789abcdefull) return;
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), r, vo, row * rs, LTE_SHAPE_AUXS);
}

struct Job {
  uint64_t* blk;
  uint64_t* ck;
  int K, f1, f2, G;
};
struct Jobs {
  Job j[5];
  int prefix[6];
  int n;
};

__device__ __forceinline__ int modadd(int a, int b, int K) { a += b; return a >= K ? a - K : a; }
__device__ __forceinline__ int modsub(int a, int b, int K) { a -= b; return a < 0 ? a + K : a; }

template <bool CKPT, bool dec2, bool first, bool SEQ = false, bool NOST = false>
__device__ void pass(__amdgpu_buffer_rsrc_t rb, __amdgpu_buffer_rsrc_t rc, int vo, int K, int f1, int f2,
                     uint64_t& acc, int rs) {
  const int nsub = K / 8, tf2 = (2 * f2) % K;
  const int lp0 = dec2 ? 3 * K + 6 : 2 * K + 3;
  int pi = 0, d = (f1 + f2) % K;
#pragma unroll 1
  for (int w = 0; w < nsub; ++w) {
    if (LTE_SHAPE_SYNC && w % 3 == 0) __syncthreads();
    if (CKPT && w % 3 == 0) {
#pragma unroll
      for (int s = 0; s < 8; ++s) st<NOST>(rc, vo, (w / 3) * 8 + s, acc + s, RSC(rs));
    }
    uint64_t xs[8], xp[8], xe[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {   // the window's loads first (as the decoder's ldwin), then the fold
      const int k = w * 8 + j, p = (dec2 && !SEQ) ? pi : k;
      xs[j] = ld(rb, vo, ROW_LS(p), rs);
      xp[j] = ld(rb, vo, lp0 + k, rs);
      xe[j] = first ? 0 : ld(rb, vo, ROW_LE(p), rs);
      if (dec2) { pi = modadd(pi, d, K); d = modadd(d, tf2, K); }
    }
    uint64_t x = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) x ^= xs[j] ^ xp[j] ^ xe[j];
    acc = acc * 3 + x;
  }
  // tails: 3 termination steps (2 rows each)
#pragma unroll
  for (int j = 0; j < 3; ++j) acc ^= ld(rb, vo, 2 * K + j, rs) ^ ld(rb, vo, lp0 + K + j, rs);
  const int nsw = (nsub + 2) / 3;
#pragma unroll 1
  for (int q = nsw - 1; q >= 0; --q) {
    if (LTE_SHAPE_SYNC) __syncthreads();
    const int ns = min(3, nsub - q * 3), n = ns * 8, k0 = q * 24;
    if (dec2) {
#pragma unroll 1
      for (int j = 0; j < n; ++j) { d = modsub(d, tf2, K); pi = modsub(pi, d, K); }
    }
    uint64_t v[24], vp[24], ve[24];
    int pp = pi, dd = d;
#pragma unroll
    for (int i = 0; i < 24; ++i) {
      if (i < n) {
        const int k = k0 + i, p = (dec2 && !SEQ) ? pp : k;
        v[i] = ld(rb, vo, ROW_LS(p), rs);
        vp[i] = ld(rb, vo, lp0 + k, rs);
        ve[i] = first ? 0 : ld(rb, vo, ROW_LE(p), rs);
        if (dec2) { pp = modadd(pp, dd, K); dd = modadd(dd, tf2, K); }
      }
    }
#pragma unroll
    for (int i = 0; i < 24; ++i) v[i] ^= vp[i] ^ ve[i];
    if (CKPT) {
#pragma unroll
      for (int s = 0; s < 8; ++s) acc ^= ld(rc, vo, q * 8 + s, RSC(rs));
    }
#pragma unroll
    for (int i = 23; i >= 0; --i) {
      if (i < n) {
        const int k = k0 + i;
        int p = k;
        if (dec2) { dd = modsub(dd, tf2, K); pp = modsub(pp, dd, K); p = SEQ ? k : pp; }
        st<NOST>(rb, vo, ROW_LE(p), v[i] + acc, rs);
      }
    }
    if (dec2) { pi = pp; d = dd; }
  }
}

template <bool CKPT, bool SEQ = false, bool NOST = false>
__global__ __launch_bounds__(256) void k_shape(Jobs J, int iters, int CH) {
  extern __shared__ uint64_t lds_pad[];
  const int wg = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wg >= J.prefix[J.n]) return;
  int r = 0;
  while (wg >= J.prefix[r + 1]) ++r;
  const Job jb = J.j[r];
  const int g = wg - J.prefix[r], K = jb.K, lane = threadIdx.x & 63, vo = lane * 8;
  const size_t rows = 4 * (size_t)K + 12, ckrows = (size_t)(K / 8 + 1) * 8;
  size_t gg = g;
  if (LTE_SHAPE_XCD && CH == 32 && (J.prefix[r] % 256) == 0) {   // g = 4 (8 q + x) + w -> chunk (q / 8) * 8 + x
    const int b = g >> 2, w = g & 3, x = b & 7, q = b >> 3;
    if ((b | 63) < J.prefix[r + 1] / 4 - J.prefix[r] / 4) gg = (size_t)((q >> 3) * 8 + x) * 32 + (q & 7) * 4 + w;
  }
  const size_t ch = gg / CH, gi = gg % CH;   // CH = 1: each group's block contiguous
  const __amdgpu_buffer_rsrc_t rb = rsrc(jb.blk + (ch * rows * CH + gi) * 64, (uint32_t)(rows * 512 * CH));
  const __amdgpu_buffer_rsrc_t rc = LTE_SHAPE_CKCH1 ? rsrc(jb.ck + gg * ckrows * 64, (uint32_t)(ckrows * 512))
                                                    : rsrc(jb.ck + (ch * ckrows * CH + gi) * 64, (uint32_t)(ckrows * 512 * CH));
  uint64_t acc = lane;
  const int rs = 512 * CH;
  for (int it = 0; it < iters; ++it) {
    if (it == 0) pass<CKPT, false, true, SEQ, NOST>(rb, rc, vo, K, jb.f1, jb.f2, acc, rs);
    else pass<CKPT, false, false, SEQ, NOST>(rb, rc, vo, K, jb.f1, jb.f2, acc, rs);
    pass<CKPT, true, false, SEQ, NOST>(rb, rc, vo, K, jb.f1, jb.f2, acc, rs);
  }
  pass<CKPT, false, false, false, NOST>(rb, rc, vo, K, jb.f1, jb.f2, acc, rs);
  if (acc == 0x123456789abcdefull) lds_pad[0] = acc;   // never true; keeps the LDS request
}

// bytes one wave moves (the loop structure above, counted on the host);
// stores_only: just the extrinsic and checkpoint rows it writes
// (bench.py shape_bytes mirrors this count)
static double wave_bytes(int K, int iters, bool ckpt, bool stores_only = false) {
  const int nsub = K / 8, nsw = (nsub + 2) / 3;
  double rows = 0;
  for (int p = 0; p < 2 * iters + 1; ++p) {
    const bool first = p == 0;
    const double per = first ? 2 : 3;
    if (!stores_only) rows += per * K * 2 + 6;   // fwd + bwd loads, tails
    rows += K;                                   // extrinsic stores
    if (ckpt) rows += (double)((nsub + 2) / 3) * 8 + (stores_only ? 0 : nsw * 8);   // checkpoint stores + loads
  }
  return rows * 512;
}

int main(int argc, char** argv) {
  const int F = argc > 1 ? atoi(argv[1]) : 65536, iters = 8, G = F / 64;
  const int Ks[5] = {5568, 5568, 5568, 5568, 5632}, f1s[5] = {43, 43, 43, 43, 45}, f2s[5] = {174, 174, 174, 174, 176};
  Jobs J{};
  J.n = 5;
  std::vector<void*> bufs;
  double bytes_ck = 0, bytes_nock = 0, bytes_st = 0;
  for (int r = 0; r < 5; ++r) {
    const size_t rows = 4 * (size_t)Ks[r] + 12, ckrows = (size_t)(Ks[r] / 8 + 1) * 8;
    void *b, *c;
    if (hipMalloc(&b, rows * 512 * G) || hipMalloc(&c, ckrows * 512 * G)) {
      printf("alloc failed\n");
      return 1;
    }
    (void)hipMemset(b, 0, rows * 512 * G);
    (void)hipMemset(c, 0, ckrows * 512 * G);
    bufs.push_back(b);
    bufs.push_back(c);
    J.j[r] = Job{(uint64_t*)b, (uint64_t*)c, Ks[r], f1s[r], f2s[r], G};
    J.prefix[r + 1] = J.prefix[r] + G;
    bytes_ck += wave_bytes(Ks[r], iters, true) * G;
    bytes_nock += wave_bytes(Ks[r], iters, false) * G;
    bytes_st += wave_bytes(Ks[r], iters, true, true) * G;
  }
  const int waves = J.prefix[5];
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto run = [&](bool ck, size_t lds, bool seq = false, int CH = 1, bool nost = false) {
    auto k = nost ? k_shape<true, false, true> : seq ? k_shape<true, true> : ck ? k_shape<true> : k_shape<false>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k, dim3((waves + 3) / 4), dim3(256), lds, 0, J, iters, CH);   // warm
    (void)hipEventRecord(a, 0);
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k, dim3((waves + 3) / 4), dim3(256), lds, 0, J, iters, CH);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / 3.0;
  };
  if (argc > 2 && std::string(argv[2]) == "decoder") {   // the decoder's layout only (bench.py --shape-ceiling)
    const double a1 = run(true, 96 * 1024, false, 32), a2 = run(true, 64 * 1024, false, 32), a3 = run(true, 0, false, 32);
    const double best = a1 < a2 ? (a1 < a3 ? a1 : a3) : (a2 < a3 ? a2 : a3);
    // the same shape with its stores dropped (extrinsic + checkpoint rows):
    // what the 17 % of bytes that are stores cost in time, on this box
    const double an = run(true, 96 * 1024, false, 32, true);
    if (hipDeviceSynchronize() != hipSuccess) {
      printf("kernel failed\n");
      return 1;
    }
    printf("{\"frames\": %d, \"waves\": %d, \"bytes_per_launch_ckpt\": %.0f, \"bytes_per_launch_stores\": %.0f, "
           "\"decoder_layout\": {\"CH\": 32, "
           "\"aux\": %d, \"ms_1wps\": %.3f, \"ms_2wps\": %.3f, \"ms_free\": %.3f, \"GBs_best\": %.1f, "
           "\"ms_1wps_reads_only\": %.3f}}\n",
           F, waves, bytes_ck, bytes_st, LTE_SHAPE_AUXL, a1, a2, a3, bytes_ck / (best * 1e-3) / 1e9, an);
    for (void* p : bufs) (void)hipFree(p);
    return 0;
  }
  const double m1 = run(true, 96 * 1024), m0 = run(false, 96 * 1024), m2 = run(true, 64 * 1024),
               m3 = run(true, 0), m4 = run(true, 96 * 1024, true), m5 = run(true, 0, true);
  if (hipDeviceSynchronize() != hipSuccess) {
    printf("kernel failed\n");
    return 1;
  }
  printf("{\"frames\": %d, \"waves\": %d, \"bytes_per_launch_ckpt\": %.0f, \"bytes_per_launch_nockpt\": %.0f, "
         "\"ms_1wps_ckpt\": %.3f, \"GBs_1wps_ckpt\": %.1f, \"ms_1wps_nockpt\": %.3f, \"GBs_1wps_nockpt\": %.1f, "
         "\"ms_2wps_ckpt\": %.3f, \"GBs_2wps_ckpt\": %.1f, \"ms_free_ckpt\": %.3f, \"GBs_free_ckpt\": %.1f}\n",
         F, waves, bytes_ck, bytes_nock, m1, bytes_ck / (m1 * 1e-3) / 1e9, m0, bytes_nock / (m0 * 1e-3) / 1e9, m2,
         bytes_ck / (m2 * 1e-3) / 1e9, m3, bytes_ck / (m3 * 1e-3) / 1e9);
  printf("{\"ms_1wps_ckpt_seq\": %.3f, \"GBs_1wps_ckpt_seq\": %.1f, \"ms_free_ckpt_seq\": %.3f, \"GBs_free_ckpt_seq\": %.1f}\n",
         m4, bytes_ck / (m4 * 1e-3) / 1e9, m5, bytes_ck / (m5 * 1e-3) / 1e9);
  // chunked layouts: rows of CH consecutive waves side by side (G = 1024 is a multiple of every CH)
  const int chs[6] = {2, 4, 8, 16, 32, 64};
  for (int c = 0; c < 6; ++c) {
    const double m = run(true, 96 * 1024, false, chs[c]);
    printf("{\"CH\": %d, \"ms_1wps_ckpt\": %.3f, \"GBs_1wps_ckpt\": %.1f}\n", chs[c], m, bytes_ck / (m * 1e-3) / 1e9);
  }
  {   // the decoder's layout (TURBO_CH = 32 groups per chunk; build with -DLTE_SHAPE_AUX=3 for its policy)
    const double a1 = run(true, 96 * 1024, false, 32), a2 = run(true, 64 * 1024, false, 32), a3 = run(true, 0, false, 32);
    const double best = a1 < a2 ? (a1 < a3 ? a1 : a3) : (a2 < a3 ? a2 : a3);
    printf("{\"decoder_layout\": {\"CH\": 32, \"aux\": %d, \"ms_1wps\": %.3f, \"ms_2wps\": %.3f, \"ms_free\": %.3f, "
           "\"GBs_1wps\": %.1f, \"GBs_best\": %.1f}}\n", LTE_SHAPE_AUXL, a1, a2, a3, bytes_ck / (a1 * 1e-3) / 1e9,
           bytes_ck / (best * 1e-3) / 1e9);
  }
  {
    const double m = run(true, 96 * 1024, false, 1);
    printf("{\"CH\": 1, \"ms_1wps_ckpt\": %.3f, \"GBs_1wps_ckpt\": %.1f, \"repeat\": true}\n", m, bytes_ck / (m * 1e-3) / 1e9);
  }
  if (hipDeviceSynchronize() != hipSuccess) {
    printf("kernel failed\n");
    return 1;
  }
  for (void* p : bufs) (void)hipFree(p);
  return 0;
}
