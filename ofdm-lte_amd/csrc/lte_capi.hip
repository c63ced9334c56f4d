// C ABI of liblte_hip.so (include/lte_phy.h): plan construction (all index /
// permutation tables are built here, natively, once per configuration),
// device workspace ownership, and orchestration of the kernel chain on the
// plan's HIP stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <complex>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "lte_common.h"
#include "lte_internal.h"

using namespace lte;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                         \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess) return fail(LTE_EHIP, std::string(#expr ": ") + hipGetErrorString(_e)); \
  } while (0)
#define LCHK(expr)                                                                           \
  do {                                                                                       \
    int _e = (expr);                                                                         \
    if (_e != 0) return fail(LTE_EHIP, std::string(#expr ": ") + hipGetErrorString((hipError_t)_e)); \
  } while (0)

// ------------------------------------------------------------------ MT19937
// NumPy legacy RandomState: seed(s) = init_genrand(s); choice([1,-1], n) =
// randint(0, 2, n) = (next_uint32 & 1) per draw (masked bounded ints).
struct MT19937 {
  uint32_t mt[624];
  int idx;
  explicit MT19937(uint32_t s) {
    mt[0] = s;
    for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    idx = 624;
  }
  uint32_t next() {
    if (idx >= 624) {
      for (int i = 0; i < 624; ++i) {
        const uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7fffffffu);
        mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      }
      idx = 0;
    }
    uint32_t y = mt[idx++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
};

// QPP table (3GPP TS 36.212 Table 5.1.3-3; turbo_encoder.py:34-73)
const int QPP_TAB[][3] = {
    {40, 3, 10}, {48, 7, 12}, {56, 19, 42}, {64, 7, 16}, {72, 7, 18}, {80, 11, 20}, {88, 5, 22}, {96, 11, 24},
    {104, 7, 26}, {112, 41, 84}, {120, 103, 90}, {128, 15, 32}, {136, 9, 34}, {144, 17, 108}, {152, 9, 38},
    {160, 21, 120}, {168, 101, 84}, {176, 21, 44}, {184, 57, 46}, {192, 23, 48}, {200, 13, 50}, {208, 27, 52},
    {216, 11, 36}, {224, 27, 56}, {232, 85, 58}, {240, 29, 60}, {248, 33, 62}, {256, 15, 32}, {264, 17, 198},
    {272, 33, 68}, {280, 103, 210}, {288, 19, 36}, {296, 19, 74}, {304, 37, 76}, {312, 19, 78}, {320, 21, 120},
    {328, 21, 82}, {336, 115, 84}, {344, 193, 86}, {352, 21, 44}, {360, 133, 90}, {368, 81, 46}, {376, 45, 94},
    {384, 23, 48}, {392, 243, 98}, {400, 151, 40}, {408, 155, 102}, {416, 25, 52}, {424, 51, 106}, {432, 47, 72},
    {440, 91, 110}, {448, 29, 168}, {456, 29, 114}, {464, 247, 58}, {472, 29, 118}, {480, 89, 180},
    {488, 91, 122}, {496, 157, 62}, {504, 55, 84}, {512, 31, 64}, {528, 17, 66}, {544, 35, 68}, {560, 227, 420},
    {576, 65, 96}, {592, 19, 74}, {608, 37, 76}, {624, 41, 234}, {640, 39, 80}, {656, 185, 82}, {672, 43, 252},
    {688, 21, 86}, {704, 155, 44}, {720, 79, 120}, {736, 139, 92}, {752, 23, 94}, {768, 217, 48}, {784, 25, 98},
    {800, 17, 80}, {816, 127, 102}, {832, 25, 52}, {848, 239, 106}, {864, 17, 48}, {880, 137, 110},
    {896, 215, 112}, {912, 29, 114}, {928, 15, 58}, {944, 147, 118}, {960, 29, 60}, {976, 59, 122},
    {992, 65, 124}, {1008, 55, 84}, {1024, 31, 64}, {1056, 17, 66}, {1088, 171, 204}, {1120, 67, 140},
    {1152, 35, 72}, {1184, 19, 74}, {1216, 39, 76}, {1248, 19, 78}, {1280, 199, 240}, {1312, 21, 82},
    {1344, 211, 252}, {1376, 21, 86}, {1408, 43, 88}, {1440, 149, 60}, {1472, 45, 92}, {1504, 49, 846},
    {1536, 71, 48}, {1568, 13, 28}, {1600, 17, 80}, {1632, 25, 102}, {1664, 183, 104}, {1696, 55, 954},
    {1728, 127, 96}, {1760, 27, 110}, {1792, 29, 112}, {1824, 29, 114}, {1856, 57, 116}, {1888, 45, 354},
    {1920, 31, 120}, {1952, 59, 610}, {1984, 185, 124}, {2016, 113, 420}, {2048, 31, 64}, {2112, 17, 66},
    {2176, 171, 136}, {2240, 209, 420}, {2304, 253, 216}, {2368, 367, 444}, {2432, 265, 456}, {2496, 181, 468},
    {2560, 39, 80}, {2624, 27, 164}, {2688, 127, 504}, {2752, 143, 172}, {2816, 43, 88}, {2880, 29, 300},
    {2944, 45, 92}, {3008, 157, 188}, {3072, 47, 96}, {3136, 13, 28}, {3200, 111, 240}, {3264, 443, 204},
    {3328, 51, 104}, {3392, 51, 212}, {3456, 451, 192}, {3520, 257, 220}, {3584, 57, 336}, {3648, 313, 228},
    {3712, 271, 232}, {3776, 179, 236}, {3840, 331, 120}, {3904, 363, 244}, {3968, 375, 248}, {4032, 127, 168},
    {4096, 31, 64}, {4160, 33, 130}, {4224, 43, 264}, {4288, 33, 134}, {4352, 477, 408}, {4416, 35, 138},
    {4480, 233, 280}, {4544, 357, 142}, {4608, 337, 480}, {4672, 37, 146}, {4736, 71, 444}, {4800, 71, 120},
    {4864, 37, 152}, {4928, 39, 462}, {4992, 127, 234}, {5056, 39, 158}, {5120, 39, 80}, {5184, 31, 96},
    {5248, 113, 902}, {5312, 41, 166}, {5376, 251, 336}, {5440, 43, 170}, {5504, 21, 86}, {5568, 43, 174},
    {5632, 45, 176}, {5696, 45, 178}, {5760, 161, 120}, {5824, 89, 182}, {5888, 323, 184}, {5952, 47, 186},
    {6016, 23, 94}, {6080, 47, 190}, {6144, 263, 480}};
const int N_QPP = sizeof(QPP_TAB) / sizeof(QPP_TAB[0]);

bool qpp_lookup(int K, int* f1, int* f2) {
  for (int i = 0; i < N_QPP; ++i)
    if (QPP_TAB[i][0] == K) { *f1 = QPP_TAB[i][1]; *f2 = QPP_TAB[i][2]; return true; }
  return false;
}

int find_interleaver_size(int n) {  // segmentation.py:53-71
  for (int i = 0; i < N_QPP; ++i)
    if (QPP_TAB[i][0] >= n) return QPP_TAB[i][0];
  return -1;
}

// segment_code_blocks (segmentation.py:74-263) as a table of CB slots.
bool segmentation_plan(int B, std::vector<CbInfo>& out) {
  const int Z = 6144;
  out.clear();
  if (B <= Z) {
    const int K = find_interleaver_size(B);
    if (K < 0) return false;
    CbInfo c{K, K - B, B, 0, 0, 0, 0, 3 * K + 12};
    qpp_lookup(K, &c.f1, &c.f2);
    out.push_back(c);
    return true;
  }
  const int L = 24;
  const int C = (B + (Z - L) - 1) / (Z - L);
  const int Bp = B + C * L;
  const int Kp = find_interleaver_size((Bp + C - 1) / C);
  if (Kp < 0) return false;
  int ki = 0;
  while (QPP_TAB[ki][0] != Kp) ++ki;
  const int Km = ki > 0 ? QPP_TAB[ki - 1][0] : Kp;
  const int dK = Kp - Km;
  const int Cm = dK > 0 ? (C * Kp - Bp) / dK : 0;
  int rem = B, off = 0;
  for (int r = 0; r < C; ++r) {
    const int K = r < Cm ? Km : Kp;
    const int avail = K - L;
    const int info = (r == C - 1) ? rem : std::min(avail, rem / (C - r));
    rem -= info;
    CbInfo c{K, (K - L) - info, info, off, 1, 0, 0, 3 * K + 12};
    qpp_lookup(K, &c.f1, &c.f2);
    out.push_back(c);
    off += info;
  }
  return true;
}

const int SBI_P[32] = {0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30,
                       1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31};

// sub_block_interleaver index map (rate_matching.py:25-94): v[i] = d[perm[i]]
std::vector<int> subblock_perm(int n) {
  const int R = (n + 31) / 32;
  std::vector<int> p;
  p.reserve(n);
  for (int row = 0; row < R; ++row)
    for (int j = 0; j < 32; ++j) {
      const int idx = SBI_P[j] * R + row;
      if (idx < n) p.push_back(idx);
    }
  return p;
}

// Where coded bit i of CB (K, rv) comes from: stream (0/1/2) and index in that
// stream, or stream -1 (padding of v1/v2).  rate_matching.py:249-297.
struct RmSrc { int stream, idx; };
void rm_source(int K, int rv, int E, std::vector<RmSrc>& out) {
  const int ml = K + 6, Ncb = 3 * ml;
  const int starts[4] = {0, Ncb / 4, Ncb / 2, 3 * Ncb / 4};
  const int st = starts[rv & 3];
  const std::vector<int> p0 = subblock_perm(K + 6), p1 = subblock_perm(K + 3);
  out.resize(E);
  for (int i = 0; i < E; ++i) {
    const int c = (st + i) % Ncb;
    const int s = c % 3, v = c / 3;
    if (s == 0) out[i] = {0, p0[v]};
    else if (v < K + 3) out[i] = {s, p1[v]};
    else out[i] = {-1, 0};
  }
}

// ------------------------------------------------------------------ buffers
template <class T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  int alloc(size_t count) {
    if (count <= n && p) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    if (count == 0) return 0;
    if (hipMalloc(&p, count * sizeof(T)) != hipSuccess) return -1;
    n = count;
    return 0;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

int ilog2(int n) {
  int l = 0;
  while ((1 << l) < n) ++l;
  return l;
}

struct GridHost {
  int N, Nc, cp, Nd, Np;
  std::vector<int32_t> data, pilot, seg;
  std::vector<float> inv_gap;
};

// LTEResourceGrid._init_subcarrier_types (resource_mapper.py:57-93)
GridHost make_grid(int N, int Nc, int cp) {
  GridHost g;
  g.N = N; g.Nc = Nc; g.cp = cp;
  const int gl = (N - Nc) / 2, gr = N - Nc - gl, dc = N / 2;
  for (int k = 0; k < N; ++k) {
    if (k < gl || k >= N - gr) continue;
    if (k == dc) continue;
    if (((k - gl) % 6) == 3) g.pilot.push_back(k);
    else g.data.push_back(k);
  }
  g.Nd = (int)g.data.size();
  g.Np = (int)g.pilot.size();
  g.seg.assign(N, -1);
  int s = -1;
  for (int k = 0; k < N; ++k) {
    while (s + 1 < g.Np && g.pilot[s + 1] <= k) ++s;
    g.seg[k] = s;
  }
  g.inv_gap.assign(std::max(g.Np, 1), 0.f);
  for (int i = 0; i + 1 < g.Np; ++i) g.inv_gap[i] = (float)(1.0 * (1.0 / (g.pilot[i + 1] - g.pilot[i])));
  return g;
}

// Grid::kinfo: data ordinal, -(pilot ordinal + 2) or -1 per subcarrier
std::vector<int32_t> make_kinfo(const GridHost& g) {
  std::vector<int32_t> k(g.N, -1);
  for (int j = 0; j < g.Nd; ++j) k[g.data[j]] = j;
  for (int i = 0; i < g.Np; ++i) k[g.pilot[i]] = -(i + 2);
  return k;
}

std::vector<float2> make_constellation(int bps) {  // modulator.py:28-59
  std::vector<float2> c;
  if (bps == 2) {
    const double s = 1.0 / std::sqrt(2.0);
    c = {make_float2(s, s), make_float2(s, -s), make_float2(-s, s), make_float2(-s, -s)};
    return c;
  }
  const int nl = 1 << (bps / 2);
  const double sc = bps == 4 ? std::sqrt(10.0) : std::sqrt(42.0);
  for (int i = 0; i < nl; ++i)
    for (int q = 0; q < nl; ++q)
      c.push_back(make_float2((float)((2 * i - (nl - 1)) / sc), (float)((2 * q - (nl - 1)) / sc)));
  return c;
}

std::vector<double2> make_twiddles64(int N) {
  std::vector<double2> t(N);
  for (int k = 0; k < N; ++k) {
    const double a = -2.0 * M_PI * (double)k / (double)N;
    t[k] = make_double2(std::cos(a), std::sin(a));
  }
  return t;
}

std::vector<float2> make_twiddles(int N) {
  const std::vector<double2> w = make_twiddles64(N);
  std::vector<float2> t(N);
  for (int k = 0; k < N; ++k) t[k] = make_float2((float)w[k].x, (float)w[k].y);
  return t;
}

// SC-FDM tables for the M-point DFT by Bluestein on N-point FFTs (N >= 2M - 1):
// chirp[n] = exp(-i pi n^2 / M); bhat = FFT_N(b) / (N sqrt(M)) with the circular
// b[m] = b[N - m] = exp(+i pi m^2 / M), |m| < M.  Angles reduced with exact
// integer n^2 mod 2M; the FFT of b is a float64 radix-2 on the host.
void make_bluestein64(int N, int M, std::vector<double2>& chirp, std::vector<double2>& bhat) {
  auto w = [M](int64_t m) {
    const int64_t r = (m * m) % (2LL * M);
    const double a = M_PI * (double)r / (double)M;
    return std::complex<double>(std::cos(a), std::sin(a));
  };
  chirp.resize(M);
  for (int n = 0; n < M; ++n) {
    const std::complex<double> c = std::conj(w(n));
    chirp[n] = make_double2(c.real(), c.imag());
  }
  std::vector<std::complex<double>> b(N, 0.0);
  for (int m = 0; m < M; ++m) {
    b[m] = w(m);
    if (m) b[N - m] = w(m);
  }
  // iterative radix-2 forward FFT, exp(-2 pi i k n / N)
  for (int i = 1, j = 0; i < N; ++i) {
    int bit = N >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) std::swap(b[i], b[j]);
  }
  for (int len = 2; len <= N; len <<= 1) {
    const double a = -2.0 * M_PI / len;
    for (int i = 0; i < N; i += len)
      for (int k = 0; k < len / 2; ++k) {
        const std::complex<double> tw(std::cos(a * k), std::sin(a * k));
        const std::complex<double> u = b[i + k], v = b[i + k + len / 2] * tw;
        b[i + k] = u + v;
        b[i + k + len / 2] = u - v;
      }
  }
  const double sc = 1.0 / ((double)N * std::sqrt((double)M));
  bhat.resize(N);
  for (int k = 0; k < N; ++k) bhat[k] = make_double2(b[k].real() * sc, b[k].imag() * sc);
}

void make_bluestein(int N, int M, std::vector<float2>& chirp, std::vector<float2>& bhat) {
  std::vector<double2> c, b;
  make_bluestein64(N, M, c, b);
  chirp.resize(c.size());
  bhat.resize(b.size());
  for (size_t i = 0; i < c.size(); ++i) chirp[i] = make_float2((float)c[i].x, (float)c[i].y);
  for (size_t i = 0; i < b.size(); ++i) bhat[i] = make_float2((float)b[i].x, (float)b[i].y);
}

void make_pilots(int cell, int n, std::vector<double>& re_im) {
  MT19937 mt((uint32_t)cell);
  re_im.resize(2 * (size_t)n);
  const double v = 1.0 / std::sqrt(2.0);
  for (int i = 0; i < n; ++i) {
    const double s = (mt.next() & 1u) ? -1.0 : 1.0;
    re_im[2 * i] = v * s;
    re_im[2 * i + 1] = v * s;
  }
}

struct TableSet {  // device copies of the static grid tables for one N (f64 copies in f64 plans)
  DBuf<int32_t> data, pilot, seg, kinfo;
  DBuf<float> inv_gap;
  DBuf<float2> pilots, tw, constel, chirp, bhat;
  DBuf<double> inv_gap64;
  DBuf<double2> pilots64, tw64, chirp64, bhat64;
  void release() {
    data.release(); pilot.release(); seg.release(); kinfo.release(); inv_gap.release(); pilots.release();
    tw.release(); constel.release(); chirp.release(); bhat.release();
    inv_gap64.release(); pilots64.release(); tw64.release(); chirp64.release(); bhat64.release();
  }
};

// per-precision device buffers of the signal chains (R = float / double)
template <class R>
struct ChainBufs {
  DBuf<cx<R>> x, y, coef, H, capbuf, captx, xh, tcoef;
  DBuf<R> gains, phases, pow_part, pstats, npow, llr, snr_lin, inj_ph, inj_z;
  // multi-antenna chains: received data SCs [B][n_sym][num_rx][n_dsc] (H holds
  // the estimates [B][num_rx][n_est][num_tx][n_dsc]), transmit_mimo's link
  // power partials / noise sigmas, link injections
  DBuf<cx<R>> Ym;
  DBuf<R> link_part, link_sigma, inj_lz, inj_lh;
  std::vector<DBuf<R>> blk, ckpt;
  DBuf<R*> blk_ptrs;
  void release() {
    x.release(); y.release(); coef.release(); H.release(); capbuf.release(); captx.release(); xh.release();
    tcoef.release();
    gains.release(); phases.release(); pow_part.release(); pstats.release(); npow.release(); llr.release();
    snr_lin.release(); inj_ph.release(); inj_z.release();
    Ym.release(); link_part.release(); link_sigma.release(); inj_lz.release(); inj_lh.release();
    for (auto& b : blk) b.release();
    for (auto& b : ckpt) b.release();
    blk_ptrs.release();
  }
};

template <class T>
int upload(DBuf<T>& d, const std::vector<T>& h) {
  if (d.alloc(std::max<size_t>(h.size(), 1))) return -1;
  if (!h.empty() && hipMemcpy(d.p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess) return -1;
  return 0;
}

const char* KNAMES[] = {"payload", "encode", "ofdm_tx", "fading", "channel", "rx_chest", "rx_data",
                        "dematch", "turbo",   "crc_count", "accumulate", "capture"};
enum { KN_PAYLOAD, KN_ENCODE, KN_OFDM_TX, KN_FADING, KN_CHANNEL, KN_RX_CHEST, KN_RX_DATA, KN_DEMATCH, KN_TURBO,
       KN_CRC, KN_ACC, KN_CAP, KN_COUNT };

}  // namespace

// ------------------------------------------------------------------ capture kernel
namespace lte {
// received stream with its noise, as the reference returns it (signal + noise)
template <class R>
__global__ void k_cap_rx(int L, int num_rx, int B, const cx<R>* __restrict__ y, int64_t y_rx_stride,
                         int64_t y_frame_stride, const R* __restrict__ npow, const uint64_t* __restrict__ fid,
                         uint64_t seed, const R* __restrict__ inj_z, int64_t inj_stride, cx<R>* __restrict__ out) {
  const int nb = (L + 255) / 256;
  const int n = (blockIdx.x % nb) * blockDim.x + threadIdx.x;
  const int rx = blockIdx.y, b = blockIdx.x / nb;
  if (n >= L) return;
  const R sigma = sqrt(npow[(size_t)b * num_rx + rx] / (R)2);
  cx<R> z;
  if (inj_z) {
    const R* zf = inj_z + (size_t)b * inj_stride + (size_t)rx * 2 * L;
    z = mkc(zf[n], zf[L + n]);
  } else {
    const u32x4 r = rng4(seed, fid[b], RNG_STREAM_NOISE + (uint32_t)rx, (uint32_t)(n >> 1));
    z = (n & 1) ? gauss2<R>(r.z, r.w) : gauss2<R>(r.x, r.y);
  }
  const cx<R> v = y[b * y_frame_stride + rx * y_rx_stride + n];
  out[((size_t)b * num_rx + rx) * L + n] = mkc(v.x + sigma * z.x, v.y + sigma * z.y);
}
}  // namespace lte

struct lte_plan {
  lte_plan_desc d;
  int L, n_sym, Nd, Np, n_grp, nblk, PW, C = 0, KWmax = 0, EW = 0, enc_words = 0;
  int coded_len = 0, n_re_bits = 0;
  int log2N;
  GridHost gh;
  TableSet tabs;
  Grid grid;
  hipStream_t stream = nullptr;
  int f64 = 0;                       // signal chain + decoder in float64 (every chain but beamforming)
  int n_layers = 1;                  // rx_map layers (> 1: rate-matching repetition, E > N_cb)
  std::vector<CbInfo> cbs;
  // device
  DBuf<CbInfo> cbi;
  DBuf<int32_t> tx_map, rx_map, delays;
  DBuf<int32_t> txf_map, txf_re;   // k_ofdm_txf's bank-aware lane order (empty: RE order)
  double txf_model[2] = {0, 0};     // modelled extra LDS cycles per 32-lane gather: RE order, lane order
  DBuf<uint32_t> pw, enc, inj_bits;
  DBuf<uint8_t> inj_bytes;   // the caller's payload bits as given (packed on the device)
  DBuf<uint16_t> enc_qmask;   // encoder 2's per-bit segment-state contributions (encode_qmask)
  int qstride = 0;
  ChainBufs<float> c32;              // f32 plans (and the beamforming chain)
  ChainBufs<double> c64;             // f64 plans
  DBuf<uint32_t> frame_err, frame_crc;
  DBuf<int32_t> snr_idx;
  DBuf<double> nvar;                 // spatial detectors' noise variance 10 ** (-snr_db / 10), float64
  DBuf<uint64_t> fid;
  DBuf<unsigned long long> counts;
  DBuf<uint8_t> cap_bits;
  std::vector<DBuf<uint32_t>> decb;
  DBuf<int64_t> rows_dev;
  DBuf<uint32_t*> dec_ptrs;
  DBuf<int> kw_dev;
  // multi-antenna chains (lte_mimo.hip)
  bool mimo = false;
  // beamforming chain (lte_bf.hip)
  bool bf = false;
  int bf_ncb = 0;
  DBuf<double> bf_cb;
  DBuf<BfFrameT<float>> bf_fr;
  DBuf<BfFrameT<double>> bf_fr64;
  int res = 0;                       // QAM symbols per OFDM symbol (= Nd for SISO / SIMO)
  MimoGrid mg{};
  DBuf<int32_t> m_np, m_ppos, m_pseg;
  DBuf<float2> m_pval;
  DBuf<double2> m_pval64;
  DBuf<float> m_pig;
  DBuf<double> m_pig64, m_W;
  // timing
  bool timing = false;
  double kms[KN_COUNT] = {0};
  int64_t klaunch[KN_COUNT] = {0};
  std::vector<hipEvent_t> evpool;
  std::vector<std::pair<int, int>> evuse;  // (kernel id, first event index)
};

namespace {

struct Timer {  // brackets one launch with events when timing is on
  lte_plan* p;
  int id, e0;
  hipStream_t st;
  Timer(lte_plan* pl, int kid, hipStream_t s_ = nullptr) : p(pl), id(kid), e0(-1), st(s_ ? s_ : pl->stream) {
    if (!p->timing) return;
    e0 = (int)p->evuse.size() * 2;
    if ((int)p->evpool.size() < e0 + 2) {
      hipEvent_t a, b;
      (void)hipEventCreate(&a);
      (void)hipEventCreate(&b);
      p->evpool.push_back(a);
      p->evpool.push_back(b);
    }
    (void)hipEventRecord(p->evpool[e0], st);
  }
  ~Timer() {
    if (e0 < 0) return;
    (void)hipEventRecord(p->evpool[e0 + 1], st);
    p->evuse.push_back({id, e0});
  }
};

template <class R> ChainBufs<R>& cbuf(lte_plan* p);
template <class R> BfFrameT<R>* bf_frames(lte_plan* p);
template <> BfFrameT<float>* bf_frames<float>(lte_plan* p) { return p->bf_fr.p; }
template <> BfFrameT<double>* bf_frames<double>(lte_plan* p) { return p->bf_fr64.p; }
template <> ChainBufs<float>& cbuf<float>(lte_plan* p) { return p->c32; }
template <> ChainBufs<double>& cbuf<double>(lte_plan* p) { return p->c64; }

// an on/off switch from the environment (A/B knobs): unset -> def
bool env_on(const char* name, bool def) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) != 0 : def;
}

// chunk width of the plan's decoder rows (allocated for ceil(max_frames / 64) groups)
int turbo_plan_ch(const lte_plan* p) { return turbo_chunk((p->d.max_frames + 63) / 64); }

void collect_timing(lte_plan* p) {
  for (auto& u : p->evuse) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, p->evpool[u.second], p->evpool[u.second + 1]) == hipSuccess) {
      p->kms[u.first] += ms;
      p->klaunch[u.first] += 1;
    }
  }
  p->evuse.clear();
}

}  // namespace

extern "C" {

int lte_version(void) { return LTE_ABI_VERSION; }   // 3: snr_db is double (include/lte_phy.h history)

int lte_abi_check(int abi_version) {
  if (abi_version == LTE_ABI_VERSION) return LTE_OK;
  return fail(LTE_EUNSUP, "ABI mismatch: caller built against version " + std::to_string(abi_version) +
                              ", library implements " + std::to_string(LTE_ABI_VERSION));
}

const char* lte_last_error(void) { return g_err.c_str(); }

const char* lte_strerror(int code) {
  switch (code) {
    case LTE_OK: return "ok";
    case LTE_EINVAL: return "invalid argument";
    case LTE_EHIP: return "HIP runtime error";
    case LTE_ENOMEM: return "device out of memory";
    case LTE_ENODEV: return "no gfx950 device";
    case LTE_EUNSUP: return "unsupported configuration";
    default: return "unknown error";
  }
}

int lte_device_init(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(LTE_ENODEV, "no HIP device visible");
  if (device < 0 || device >= n) return fail(LTE_EINVAL, "device index out of range");
  HIPCHK(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(LTE_ENODEV, std::string("device is ") + prop.gcnArchName + ", kernels are built for gfx950");
  return LTE_OK;
}

int lte_pilots(int cell_id, int n, double* out) {
  if (n < 0 || !out) return fail(LTE_EINVAL, "bad pilot request");
  std::vector<double> v;
  make_pilots(cell_id, n, v);
  std::memcpy(out, v.data(), v.size() * sizeof(double));
  return LTE_OK;
}

int lte_philox_host(uint64_t seed, int n_frames, const uint64_t* frame_ids, uint32_t stream, int64_t n_ctr,
                    uint32_t* out_u32, double* out_gauss64, float* out_gauss32) {
  if (n_frames < 0 || n_ctr < 0 || n_ctr > 0xFFFFFFFFll || (n_frames && !frame_ids))
    return fail(LTE_EINVAL, "bad philox arguments");
  const int64_t n = (int64_t)n_frames * n_ctr;
  if (n == 0) return LTE_OK;
  DBuf<uint64_t> dfid;
  DBuf<uint32_t> du;
  DBuf<double> d64;
  DBuf<float> d32;
  auto rel = [&] { dfid.release(); du.release(); d64.release(); d32.release(); };
  if (dfid.alloc(n_frames) || (out_u32 && du.alloc(4 * n)) || (out_gauss64 && d64.alloc(4 * n)) ||
      (out_gauss32 && d32.alloc(4 * n))) {
    rel();
    return fail(LTE_ENOMEM, "philox buffers");
  }
  int rc = LTE_OK;
  if (hipMemcpy(dfid.p, frame_ids, n_frames * 8, hipMemcpyHostToDevice) != hipSuccess ||
      launch_philox_draws(nullptr, seed, dfid.p, n_frames, stream, n_ctr, du.p, d64.p, d32.p) ||
      hipDeviceSynchronize() != hipSuccess ||
      (out_u32 && hipMemcpy(out_u32, du.p, 16 * n, hipMemcpyDeviceToHost) != hipSuccess) ||
      (out_gauss64 && hipMemcpy(out_gauss64, d64.p, 32 * n, hipMemcpyDeviceToHost) != hipSuccess) ||
      (out_gauss32 && hipMemcpy(out_gauss32, d32.p, 16 * n, hipMemcpyDeviceToHost) != hipSuccess))
    rc = fail(LTE_EHIP, "philox failed");
  rel();
  return rc;
}

}  // extern "C"

// OFDMChannel.transmit on an arbitrary stream in precision R (lte_channel_host / _host64).
template <class R>
static int channel_host(int64_t L, int num_rx, int channel, int n_paths, const int32_t* delays, const double* gains,
                        double fD, double fs, double snr_db, uint64_t seed, const R* x, const double* phases,
                        const double* noise, R* y, R* noise_power) {
  using V = cx<R>;
  if (L < 1 || L > (1LL << 30) || num_rx < 1 || !x || !y) return fail(LTE_EINVAL, "bad channel arguments");
  const bool ray = channel == LTE_CH_RAYLEIGH;
  if (!ray && channel != LTE_CH_AWGN) return fail(LTE_EINVAL, "Tipo de canal desconocido");
  if (ray && (n_paths < 1 || n_paths > LTE_MAX_PATHS || !delays || !gains)) return fail(LTE_EINVAL, "bad paths");
  Grid g{};
  g.L = (int)L;
  const int nblk = channel_nblk((int)L);
  DBuf<V> dx, dy, dcoef, dout;
  DBuf<R> dph, dpp, dsl, dnp, dz, dgain, dinj;
  DBuf<int32_t> ddel;
  DBuf<uint64_t> dfid;
  int rc = LTE_OK;
  auto cleanup = [&]() {
    dx.release(); dy.release(); dcoef.release(); dout.release(); dph.release(); dpp.release(); dsl.release();
    dnp.release(); dz.release(); dgain.release(); dinj.release(); ddel.release(); dfid.release();
  };
  if (dx.alloc(L) || dout.alloc((size_t)num_rx * L) || dpp.alloc((size_t)num_rx * nblk) || dsl.alloc(1) ||
      dnp.alloc(num_rx) || dfid.alloc(1) || (ray && (dy.alloc((size_t)num_rx * L) ||
      dcoef.alloc((size_t)num_rx * n_paths) || dph.alloc((size_t)num_rx * n_paths * 16)))) {
    cleanup();
    return fail(LTE_ENOMEM, "channel buffers");
  }
  const R sl = (R)std::pow(10.0, snr_db / 10.0);
  const uint64_t fid0 = 0;
  bool ok = hipMemcpy(dx.p, x, L * sizeof(V), hipMemcpyHostToDevice) == hipSuccess &&
            hipMemcpy(dsl.p, &sl, sizeof(R), hipMemcpyHostToDevice) == hipSuccess &&
            hipMemcpy(dfid.p, &fid0, 8, hipMemcpyHostToDevice) == hipSuccess;
  if (ok && ray) {
    std::vector<int32_t> dl(delays, delays + n_paths);
    std::vector<R> hg(gains, gains + n_paths);
    ok = upload(ddel, dl) == 0 && upload(dgain, hg) == 0;
    if (ok && phases) {
      std::vector<R> hp(phases, phases + (size_t)num_rx * n_paths * 16);
      ok = upload(dinj, hp) == 0;
    }
    ok = ok && launch_fading<R>(nullptr, 1, num_rx, n_paths, dgain.p, dfid.p, seed, phases ? dinj.p : nullptr, 0,
                                dph.p, dcoef.p) == 0;
  }
  if (ok && noise) {
    std::vector<R> hz(noise, noise + (size_t)num_rx * 2 * L);
    ok = upload(dz, hz) == 0;
  }
  ok = ok && launch_channel<R>(nullptr, g, 1, num_rx, ray ? 1 : 0, n_paths, ddel.p, dgain.p, (R)fD, (R)fs, dph.p,
                               dcoef.p, dx.p, dy.p, dpp.p, nblk, ray ? *std::max_element(delays, delays + n_paths) : 0) == 0;
  ok = ok && launch_npow<R>(nullptr, 1, num_rx, dpp.p, nblk, (int)L, dsl.p, dnp.p) == 0;
  if (ok) {
    const V* ys = ray ? dy.p : dx.p;
    hipLaunchKernelGGL(k_cap_rx<R>, dim3((unsigned)((L + 255) / 256), num_rx), dim3(256), 0, nullptr, (int)L, num_rx,
                       1, ys, ray ? L : 0, ray ? (int64_t)num_rx * L : L, dnp.p, dfid.p, seed,
                       noise ? dz.p : nullptr, 0, dout.p);
    ok = hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
         hipMemcpy(y, dout.p, (size_t)num_rx * L * sizeof(V), hipMemcpyDeviceToHost) == hipSuccess &&
         (!noise_power || hipMemcpy(noise_power, dnp.p, num_rx * sizeof(R), hipMemcpyDeviceToHost) == hipSuccess);
  }
  if (!ok) rc = fail(LTE_EHIP, std::string("channel failed: ") + hipGetErrorString(hipGetLastError()));
  cleanup();
  return rc;
}

extern "C" {

int lte_channel_host(int64_t L, int num_rx, int channel, int n_paths, const int32_t* delays, const double* gains,
                     double fD, double fs, double snr_db, uint64_t seed, const float* x, const double* phases,
                     const double* noise, float* y, float* noise_power) {
  return channel_host<float>(L, num_rx, channel, n_paths, delays, gains, fD, fs, snr_db, seed, x, phases, noise, y,
                             noise_power);
}

int lte_channel_host64(int64_t L, int num_rx, int channel, int n_paths, const int32_t* delays, const double* gains,
                       double fD, double fs, double snr_db, uint64_t seed, const double* x, const double* phases,
                       const double* noise, double* y, double* noise_power) {
  return channel_host<double>(L, num_rx, channel, n_paths, delays, gains, fD, fs, snr_db, seed, x, phases, noise, y,
                              noise_power);
}

}  // extern "C"

// Multi-antenna channel on arbitrary streams in precision R (lte_channel_mimo_host / _host64).
template <class R>
static int channel_mimo_host(int64_t L, int num_tx, int num_rx, int mode, int channel, int n_paths,
                             const int32_t* delays, const double* gains, double fD, double fs, double snr_db,
                             uint64_t seed, const R* x, const double* phases, const double* link_noise,
                             const double* link_h, const double* noise, R* y, R* link_stats, R* noise_power) {
  using V = cx<R>;
  if (L < 1 || L > (1LL << 28) || num_tx < 1 || num_tx > 8 || num_rx < 1 || num_rx > 16 || !x || !y)
    return fail(LTE_EINVAL, "bad channel arguments");
  if (mode != 0 && mode != 1) return fail(LTE_EINVAL, "mode must be 0 (transmit_mimo) or 1 (spatial)");
  const bool ray = channel == LTE_CH_RAYLEIGH;
  if (!ray && channel != LTE_CH_AWGN) return fail(LTE_EINVAL, "Tipo de canal desconocido");
  if (ray && (n_paths < 1 || n_paths > LTE_MAX_PATHS || !delays || !gains)) return fail(LTE_EINVAL, "bad paths");
  // an arbitrary stream is cut into 1024-sample chunks for the fD != 0
  // expansion (f32: second order; f64: degree 5, or the per-sample sum past
  // mimo_taylor_ok)
  const int chunk = 1024;
  Grid g{};
  g.N = chunk;
  g.cp = 0;
  g.L = (int)L;
  MimoGrid m{};
  m.mode = mode == 0 ? MIMO_SFBC : MIMO_SPATIAL;
  m.num_tx = num_tx;
  m.num_rx = num_rx;
  m.exact_jakes = ray && fD != 0.0 && !mimo_taylor_ok_prec(sizeof(R) == 8, fD, fs, chunk);
  for (int k = 0; k < 16; ++k) m.jw[k] = 6.283185307179586 * fD * std::cos(6.283185307179586 * (k + 1) / 16.0);
  m.n_cs = (ray && fD != 0.0 && !m.exact_jakes) ? (int)((L + chunk - 1) / chunk) : 1;
  const int np = ray ? n_paths : 1;
  // partial-sum slots: 256-sample blocks (link stats) or OFDM-symbol blocks (channel), whichever is more
  const int nblk = std::max((int)((L + 255) / 256), mimo_channel_nblk(g.L, g.N + g.cp));
  const size_t links = (size_t)num_rx * num_tx;
  const bool link_noise_on = mode == 0 && ray;
  DBuf<V> dx, dy, dcoef, dout;
  DBuf<R> dgain, dph, dlz, dlh, dz, dpp, dlp, dls, dsl, dnp, dstp, dst, dphs;
  DBuf<int32_t> ddel;
  DBuf<uint64_t> dfid;
  auto cleanup = [&]() {
    dx.release(); dy.release(); dcoef.release(); dout.release(); dgain.release(); dph.release(); dlz.release();
    dlh.release(); dz.release(); dpp.release(); dlp.release(); dls.release(); dsl.release(); dnp.release();
    dstp.release(); dst.release(); dphs.release(); ddel.release(); dfid.release();
  };
  if (dx.alloc((size_t)num_tx * L) || dy.alloc((size_t)num_rx * L) || dout.alloc((size_t)num_rx * L) ||
      dcoef.alloc(links * np * m.n_cs * mimo_ncf<R>()) || dpp.alloc((size_t)num_rx * nblk) || dsl.alloc(1) ||
      dnp.alloc(num_rx) || dfid.alloc(1) || (m.exact_jakes && dphs.alloc(links * np * 16)) ||
      (link_noise_on && (dlp.alloc(links * nblk) || dls.alloc(links)))) {
    cleanup();
    return fail(LTE_ENOMEM, "channel buffers");
  }
  auto up = [&](DBuf<R>& d, const double* src, size_t n) {
    std::vector<R> h(src, src + n);
    return upload(d, h) == 0;
  };
  const R sl = (R)std::pow(10.0, snr_db / 10.0);
  const uint64_t fid0 = 0;
  bool ok = hipMemcpy(dx.p, x, (size_t)num_tx * L * sizeof(V), hipMemcpyHostToDevice) == hipSuccess &&
            hipMemcpy(dsl.p, &sl, sizeof(R), hipMemcpyHostToDevice) == hipSuccess &&
            hipMemcpy(dfid.p, &fid0, 8, hipMemcpyHostToDevice) == hipSuccess;
  if (ok && ray) {
    std::vector<int32_t> dl(delays, delays + n_paths);
    ok = upload(ddel, dl) == 0 && up(dgain, gains, n_paths);
  }
  if (ok && ray && phases) ok = up(dph, phases, links * n_paths * 16);
  if (ok && link_noise_on && link_noise) ok = up(dlz, link_noise, links * 2 * L);
  if (ok && !ray && mode == 1 && link_h) ok = up(dlh, link_h, links * 2);
  if (ok && noise) ok = up(dz, noise, (size_t)num_rx * 2 * L);
  ok = ok && launch_fading_mimo<R>(nullptr, g, m, 1, ray ? 1 : 0, n_paths, dgain.p, fD, fs, dfid.p, seed,
                                   (ray && phases) ? dph.p : nullptr, 0,
                                   (!ray && mode == 1 && link_h) ? dlh.p : nullptr, 0, dcoef.p, dphs.p) == 0;
  const R* lz = (link_noise_on && link_noise) ? dlz.p : nullptr;
  ok = ok && launch_channel_mimo<R>(nullptr, g, m, 1, np, ray ? ddel.p : nullptr, dcoef.p, dphs.p, dgain.p, fs, dx.p,
                                    dy.p, link_noise_on ? 1 : 0, dfid.p, seed, lz, 0, dlp.p, dls.p, dpp.p, nblk, 0) == 0;
  ok = ok && launch_npow_mimo<R>(nullptr, 1, num_rx, dpp.p, mimo_channel_nblk(g.L, g.N + g.cp), (int)L, dsl.p,
                                 mode == 0 ? (double)num_tx : 1.0, dnp.p) == 0;
  if (ok) {
    hipLaunchKernelGGL(k_cap_rx<R>, dim3((unsigned)((L + 255) / 256), num_rx), dim3(256), 0, nullptr, (int)L, num_rx, 1,
                       dy.p, (int64_t)L, (int64_t)num_rx * L, dnp.p, dfid.p, seed, noise ? dz.p : nullptr, 0,
                       dout.p);
    ok = hipGetLastError() == hipSuccess;
  }
  if (ok && link_stats) {
    ok = dstp.alloc(links * 4 * nblk) == 0 && dst.alloc(links * 4) == 0 &&
         launch_link_stats<R>(nullptr, g, m, 1, np, ray ? ddel.p : nullptr, dcoef.p, dphs.p, dgain.p, fs, dx.p,
                              link_noise_on ? dls.p : nullptr, dfid.p, seed, lz, 0, dstp.p, nblk, dst.p) == 0;
  }
  ok = ok && hipDeviceSynchronize() == hipSuccess &&
       hipMemcpy(y, dout.p, (size_t)num_rx * L * sizeof(V), hipMemcpyDeviceToHost) == hipSuccess &&
       (!noise_power || hipMemcpy(noise_power, dnp.p, num_rx * sizeof(R), hipMemcpyDeviceToHost) == hipSuccess) &&
       (!link_stats || hipMemcpy(link_stats, dst.p, links * 4 * sizeof(R), hipMemcpyDeviceToHost) == hipSuccess);
  int rc = LTE_OK;
  if (!ok) rc = fail(LTE_EHIP, std::string("mimo channel failed: ") + hipGetErrorString(hipGetLastError()));
  cleanup();
  return rc;
}

extern "C" {

int lte_channel_mimo_host(int64_t L, int num_tx, int num_rx, int mode, int channel, int n_paths,
                          const int32_t* delays, const double* gains, double fD, double fs, double snr_db,
                          uint64_t seed, const float* x, const double* phases, const double* link_noise,
                          const double* link_h, const double* noise, float* y, float* link_stats,
                          float* noise_power) {
  return channel_mimo_host<float>(L, num_tx, num_rx, mode, channel, n_paths, delays, gains, fD, fs, snr_db, seed, x,
                                  phases, link_noise, link_h, noise, y, link_stats, noise_power);
}

int lte_channel_mimo_host64(int64_t L, int num_tx, int num_rx, int mode, int channel, int n_paths,
                            const int32_t* delays, const double* gains, double fD, double fs, double snr_db,
                            uint64_t seed, const double* x, const double* phases, const double* link_noise,
                            const double* link_h, const double* noise, double* y, double* link_stats,
                            double* noise_power) {
  return channel_mimo_host<double>(L, num_tx, num_rx, mode, channel, n_paths, delays, gains, fD, fs, snr_db, seed, x,
                                   phases, link_noise, link_h, noise, y, link_stats, noise_power);
}

int lte_mimo_detect_host(int detector, int num_rx, int num_tx, int rank, int bps, int64_t n_sc, const double* y,
                         const double* H, const double* W, double sigma2, double* out) {
  if (num_rx < rank) return fail(LTE_EINVAL, "num_rx (" + std::to_string(num_rx) + ") debe ser >= num_layers (" +
                                                 std::to_string(rank) + ")");
  if (detector < LTE_DET_MMSE || detector > LTE_DET_MRC) return fail(LTE_EINVAL, "Detector no soportado");
  if (detector == LTE_DET_MRC && rank != 1) return fail(LTE_EINVAL, "MRC solo soporta num_layers=1 (rank-1)");
  if (num_rx < 1 || num_rx > 4 || num_tx < 1 || num_tx > 4 || rank < 1 || rank > num_tx)
    return fail(LTE_EUNSUP, "GPU detector: num_rx, num_tx <= 4, 1 <= rank <= num_tx");
  if (bps != 0 && bps != 2 && bps != 4 && bps != 6) return fail(LTE_EINVAL, "Unsupported modulation");
  if (n_sc < 1 || n_sc > (1LL << 26) || !y || !H || !W || !out) return fail(LTE_EINVAL, "bad detector arguments");
  std::vector<double> w4(32, 0.0);
  for (int t = 0; t < num_tx; ++t)
    for (int c = 0; c < rank; ++c) {
      w4[(t * 4 + c) * 2] = W[(t * rank + c) * 2];
      w4[(t * 4 + c) * 2 + 1] = W[(t * rank + c) * 2 + 1];
    }
  DBuf<double> dy, dH, dW, dout;
  const size_t ny = (size_t)num_rx * n_sc * 2, nh = (size_t)num_rx * num_tx * n_sc * 2, no = (size_t)rank * n_sc * 2;
  bool ok = dy.alloc(ny) == 0 && dH.alloc(nh) == 0 && dout.alloc(no) == 0 && upload(dW, w4) == 0 &&
            hipMemcpy(dy.p, y, ny * 8, hipMemcpyHostToDevice) == hipSuccess &&
            hipMemcpy(dH.p, H, nh * 8, hipMemcpyHostToDevice) == hipSuccess;
  ok = ok && launch_det_stage(nullptr, detector, num_rx, num_tx, rank, bps, n_sc, dy.p, dH.p, dW.p, sigma2, dout.p) == 0;
  ok = ok && hipDeviceSynchronize() == hipSuccess && hipMemcpy(out, dout.p, no * 8, hipMemcpyDeviceToHost) == hipSuccess;
  int rc = LTE_OK;
  if (!ok) rc = fail(LTE_EHIP, std::string("mimo detect failed: ") + hipGetErrorString(hipGetLastError()));
  dy.release(); dH.release(); dW.release(); dout.release();
  return rc;
}

// SFBCAlamouti.encode / .decode on host arrays (core/sfbc_alamouti.py:45-163).
static int sfbc_stage(int decode, int64_t n, const double* a, const double* h0, const double* h1, double reg,
                      double* o0, double* o1) {
  if (n % 2 != 0)
    return fail(LTE_EINVAL, decode ? "Number of RX symbols must be even, got " + std::to_string(n)
                                   : "Number of symbols must be even for Alamouti coding, got " + std::to_string(n));
  if (n < 0 || n > (1LL << 28) || !a || !o0 || (decode ? (!h0 || !h1) : !o1))
    return fail(LTE_EINVAL, "bad SFBC arguments");
  if (n == 0) return LTE_OK;
  const size_t nr = (size_t)n * 2;
  DBuf<double> da, dh0, dh1, d0, d1;
  bool ok = da.alloc(nr) == 0 && d0.alloc(nr) == 0 && (decode ? dh0.alloc(nr) == 0 && dh1.alloc(nr) == 0
                                                                : d1.alloc(nr) == 0) &&
            hipMemcpy(da.p, a, nr * 8, hipMemcpyHostToDevice) == hipSuccess;
  if (ok && decode)
    ok = hipMemcpy(dh0.p, h0, nr * 8, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(dh1.p, h1, nr * 8, hipMemcpyHostToDevice) == hipSuccess;
  ok = ok && launch_sfbc_stage(nullptr, decode, n, da.p, dh0.p, dh1.p, reg, d0.p, d1.p) == 0;
  ok = ok && hipDeviceSynchronize() == hipSuccess && hipMemcpy(o0, d0.p, nr * 8, hipMemcpyDeviceToHost) == hipSuccess;
  if (ok && !decode) ok = hipMemcpy(o1, d1.p, nr * 8, hipMemcpyDeviceToHost) == hipSuccess;
  int rc = LTE_OK;
  if (!ok) rc = fail(LTE_EHIP, std::string("SFBC stage failed: ") + hipGetErrorString(hipGetLastError()));
  da.release(); dh0.release(); dh1.release(); d0.release(); d1.release();
  return rc;
}

int lte_sfbc_encode_host64(int64_t n, const double* syms, double* tx0, double* tx1) {
  return sfbc_stage(0, n, syms, nullptr, nullptr, 0.0, tx0, tx1);
}

int lte_sfbc_decode_host64(int64_t n, const double* rx, const double* H0, const double* H1, double regularization,
                           double* out) {
  return sfbc_stage(1, n, rx, H0, H1, regularization, out, nullptr);
}

// Output position j of [3K+12] (turbo_encode order) fed by rate-matched index
// i (E <= N_cb) -- rate_dematching_turbo's de-collection + sub-block
// de-interleave + re-interleave (rate_matching.py:428-489) as one map.
static int dematch_first_map(int K, int E, int rv_idx, int32_t* src, bool* repeats) {
  int f1, f2;
  if (!qpp_lookup(K, &f1, &f2)) return fail(LTE_EINVAL, "Invalid interleaver size K=" + std::to_string(K));
  if (E <= 0 || !src) return fail(LTE_EINVAL, "bad E");
  const int Ncb = 3 * (K + 6);
  std::vector<RmSrc> rs;
  rm_source(K, rv_idx, std::min(E, Ncb), rs);
  const int n = 3 * K + 12;
  for (int j = 0; j < n; ++j) src[j] = -1;
  for (int i = 0; i < (int)rs.size(); ++i) {
    const RmSrc s = rs[i];
    if (s.stream < 0) continue;
    int j;
    if (s.stream == 0) {
      if (s.idx < K) j = 3 * s.idx;
      else if (s.idx < K + 3) j = 3 * K + (s.idx - K);
      else j = 3 * K + 6 + (s.idx - K - 3);
    } else if (s.stream == 1) {
      j = s.idx < K ? 3 * s.idx + 1 : 3 * K + 3 + (s.idx - K);
    } else {
      j = s.idx < K ? 3 * s.idx + 2 : 3 * K + 9 + (s.idx - K);
    }
    src[j] = i;
  }
  if (repeats) *repeats = E > Ncb;
  return LTE_OK;
}

int lte_rate_dematch_map(int K, int E, int rv_idx, int32_t* src) {
  bool rep = false;
  const int rc = dematch_first_map(K, E, rv_idx, src, &rep);
  if (rc != LTE_OK) return rc;
  if (rep) return fail(LTE_EUNSUP, "E > N_cb repeats LLRs: use lte_rate_dematch_host64 (sums the repeats)");
  return LTE_OK;
}

int lte_rate_dematch_host64(int K, int E, int rv_idx, int64_t ncb, const double* llr, double* out) {
  if (E == 0) {   // nothing received: every position punctured, zeros(3K + 12) like the reference
    if (K < 0 || ncb < 0 || (ncb > 0 && !out)) return fail(LTE_EINVAL, "bad arguments");
    std::fill(out, out + (size_t)ncb * (3 * (size_t)K + 12), 0.0);
    return LTE_OK;
  }
  if (ncb < 0 || (ncb > 0 && (!llr || !out))) return fail(LTE_EINVAL, "bad arguments");
  std::vector<int32_t> src(3 * (size_t)K + 12);
  const int rc = dematch_first_map(K, E, rv_idx, src.data(), nullptr);
  if (rc != LTE_OK || ncb == 0) return rc;
  const int n = 3 * K + 12;
  DBuf<double> dl, dout;
  DBuf<int32_t> dsrc;
  if (dl.alloc((size_t)ncb * E) || dout.alloc((size_t)ncb * n) || upload(dsrc, src))
    return fail(LTE_ENOMEM, "dematch buffers");
  int r = LTE_OK;
  if (hipMemcpy(dl.p, llr, (size_t)ncb * E * 8, hipMemcpyHostToDevice) != hipSuccess ||
      launch_rate_dematch(nullptr, dl.p, E, 3 * (K + 6), n, dsrc.p, ncb, dout.p) ||
      hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(out, dout.p, (size_t)ncb * n * 8, hipMemcpyDeviceToHost) != hipSuccess)
    r = fail(LTE_EHIP, std::string("rate dematch failed: ") + hipGetErrorString(hipGetLastError()));
  dl.release(); dout.release(); dsrc.release();
  return r;
}

int lte_qpp_perm(int K, int32_t* perm) {
  int f1, f2;
  if (!qpp_lookup(K, &f1, &f2)) return fail(LTE_EINVAL, "Invalid interleaver size K=" + std::to_string(K));
  if (!perm) return fail(LTE_EINVAL, "null perm");
  for (int64_t i = 0; i < K; ++i) perm[i] = (int32_t)((f1 * i + f2 * i * i) % K);   // turbo_encoder.py:76-103
  return LTE_OK;
}

int lte_subblock_perm(int n, int32_t* perm) {
  if (n < 0 || (n > 0 && !perm)) return fail(LTE_EINVAL, "bad arguments");
  const std::vector<int> p = subblock_perm(n);   // rate_matching.py:25-94, <NULL>s removed
  std::copy(p.begin(), p.end(), perm);
  return LTE_OK;
}

int lte_set_decoder_mode(int use_max_log_map) {
  set_logmap(use_max_log_map ? 0 : 1);
  return LTE_OK;
}

static int plan_tables(lte_plan* p) {
  const lte_plan_desc& d = p->d;
  p->gh = make_grid(d.N, d.Nc, d.cp_len);
  p->Nd = p->gh.Nd;
  p->Np = p->gh.Np;
  p->log2N = ilog2(d.N);
  std::vector<double> pr;
  make_pilots(d.cell_id, p->Np, pr);
  std::vector<float2> pil(p->Np);
  for (int i = 0; i < p->Np; ++i) pil[i] = make_float2((float)pr[2 * i], (float)pr[2 * i + 1]);
  if (upload(p->tabs.data, p->gh.data) || upload(p->tabs.pilot, p->gh.pilot) || upload(p->tabs.seg, p->gh.seg) ||
      upload(p->tabs.inv_gap, p->gh.inv_gap) || upload(p->tabs.pilots, pil) || upload(p->tabs.kinfo, make_kinfo(p->gh)) ||
      upload(p->tabs.tw, make_twiddles(d.N)) || upload(p->tabs.constel, make_constellation(d.bps)))
    return fail(LTE_ENOMEM, "table upload failed");
  if (d.sc_fdm) {   // SC-FDM DFT of size M = Nd (DFTPrecodifier, core/dft_precoding.py:20-118)
    std::vector<float2> ch, bh;
    make_bluestein(d.N, p->Nd, ch, bh);
    if (upload(p->tabs.chirp, ch) || upload(p->tabs.bhat, bh)) return fail(LTE_ENOMEM, "table upload failed");
  }
  if (p->f64) {   // float64 copies for the f64 chain
    std::vector<double2> pil64(p->Np);
    for (int i = 0; i < p->Np; ++i) pil64[i] = make_double2(pr[2 * i], pr[2 * i + 1]);
    std::vector<double> ig64(std::max(p->Np, 1), 0.0);
    for (int i = 0; i + 1 < p->Np; ++i) ig64[i] = 1.0 / (double)(p->gh.pilot[i + 1] - p->gh.pilot[i]);
    if (upload(p->tabs.pilots64, pil64) || upload(p->tabs.inv_gap64, ig64) ||
        upload(p->tabs.tw64, make_twiddles64(d.N)))
      return fail(LTE_ENOMEM, "table upload failed");
    if (d.sc_fdm) {
      std::vector<double2> ch, bh;
      make_bluestein64(d.N, p->Nd, ch, bh);
      if (upload(p->tabs.chirp64, ch) || upload(p->tabs.bhat64, bh)) return fail(LTE_ENOMEM, "table upload failed");
    }
  }
  return LTE_OK;
}

}  // extern "C"

void lte::plan_txf_lane_order(const std::vector<int32_t>& tx_map, const std::vector<int32_t>& data_idx, int n_sym,
                         int Nd, int bps, int slots, std::vector<int32_t>& txf_map, std::vector<int32_t>& txf_re,
                         double model[2]) {
  constexpr int GL = 32;   // ds_read_b32 lane group; banks = word mod 32
  txf_map.assign((size_t)n_sym * slots * bps, -1);
  txf_re.assign((size_t)n_sym * slots, -1);
  auto word = [&](int l, int j, int m) {
    const int32_t v = tx_map[((size_t)l * Nd + j) * bps + m];
    return v >= 0 ? (int)(v >> 5) : -1;
  };
  // Per (gather m, bank), the distinct words a lane group touches: fixed-size
  // sets (a group has at most GL lanes, so at most GL words per bank) -- no heap
  // allocation inside the search (the round-4 version built 32 std::vectors per
  // gather of every group).
  struct BankSets {
    int n[8][GL];
    int w[8][GL][GL];
    void clear(int bps_) { for (int m = 0; m < bps_; ++m) for (int b = 0; b < GL; ++b) n[m][b] = 0; }
    bool has(int m, int x) const {
      const int b = x % GL;
      for (int i = 0; i < n[m][b]; ++i) if (w[m][b][i] == x) return true;
      return false;
    }
    void add(int m, int x) { if (!has(m, x)) { const int b = x % GL; w[m][b][n[m][b]++] = x; } }
    int size(int m, int x) const { return n[m][x % GL]; }
  };
  BankSets bs;
  // extra cycles of the bps gathers of one lane group: per gather, the most
  // distinct words on one bank, minus one
  auto group_extra = [&](int l, const int* re, int n) {
    bs.clear(bps);
    int ex = 0;
    for (int m = 0; m < bps; ++m) {
      int mx = 1;
      for (int k = 0; k < n; ++k) {
        const int x = word(l, re[k], m);
        if (x < 0) continue;
        bs.add(m, x);
        mx = std::max(mx, bs.size(m, x));
      }
      ex += mx - 1;
    }
    return ex;
  };
  double ex0 = 0, ex1 = 0, ng = 0;
  std::vector<char> used(Nd);
  std::vector<int> grp(GL), ident(GL);
  BankSets wb;
  for (int l = 0; l < n_sym; ++l) {
    std::fill(used.begin(), used.end(), 0);
    for (int g = 0; g * GL < Nd; ++g) {
      const int n = std::min(GL, Nd - g * GL);
      for (int k = 0; k < n; ++k) ident[k] = g * GL + k;
      ex0 += group_extra(l, ident.data(), n);
      wb.clear(bps);   // bps <= 8: per gather and bank, the group's words
      int cnt8[GL / 8][8] = {};
      for (int k = 0; k < n; ++k) {
        int best = -1, bc = 1 << 30;
        for (int j = 0; j < Nd; ++j) {
          if (used[j]) continue;
          int c = cnt8[k / 8][data_idx[j] & 7];
          for (int m = 0; m < bps && c < bc; ++m) {
            const int x = word(l, j, m);
            if (x < 0) continue;
            const int sz = wb.size(m, x);
            if (sz && !wb.has(m, x)) c += sz;
          }
          if (c < bc) { bc = c; best = j; if (c == 0) break; }
        }
        used[best] = 1;
        grp[k] = best;
        ++cnt8[k / 8][data_idx[best] & 7];
        for (int m = 0; m < bps; ++m) {
          const int x = word(l, best, m);
          if (x >= 0) wb.add(m, x);
        }
        const size_t sl = (size_t)l * slots + g * GL + k;
        txf_re[sl] = best;
        for (int m = 0; m < bps; ++m) txf_map[sl * bps + m] = tx_map[((size_t)l * Nd + best) * bps + m];
      }
      ex1 += group_extra(l, grp.data(), n);
      ng += bps;
    }
  }
  model[0] = ng ? ex0 / ng : 0;
  model[1] = ng ? ex1 / ng : 0;
}

extern "C" {

static int plan_coded_maps(lte_plan* p) {
  const lte_plan_desc& d = p->d;
  if (!segmentation_plan(d.n_bits + 24, p->cbs)) return fail(LTE_EINVAL, "No valid interleaver size");
  p->C = (int)p->cbs.size();
  int Kmax = 0;
  std::vector<int> Eoff(p->C + 1, 0);
  for (int r = 0; r < p->C; ++r) {
    Kmax = std::max(Kmax, p->cbs[r].K);
    Eoff[r + 1] = Eoff[r] + p->cbs[r].E;
  }
  p->coded_len = Eoff[p->C];
  p->KWmax = (Kmax + 31) / 32 + 1;
  p->EW = (Kmax + 6 + 31) / 32;
  p->enc_words = p->C * 3 * p->EW;
  const int bps = d.bps, Nd = p->res;   // REs per OFDM symbol (SFBC: Nd & ~1)
  const int ncs_tx = (p->coded_len + bps - 1) / bps;  // bits_to_symbols pads (modulator.py:74-75)
  const int rows = (ncs_tx + Nd - 1) / Nd;
  p->n_sym = rows;
  const int ncs_rx = p->coded_len / bps;               // ofdm_core.py:1140
  const int rows_rx = (ncs_rx + Nd - 1) / Nd;
  const int n_re = p->n_sym * Nd;
  p->n_re_bits = n_re * bps;
  std::vector<std::vector<RmSrc>> rs(p->C);
  for (int r = 0; r < p->C; ++r) rm_source(p->cbs[r].K, 0, p->cbs[r].E, rs[r]);
  auto locate = [&](int e, int& r, int& i) {
    r = 0;
    while (e >= Eoff[r + 1]) ++r;
    i = e - Eoff[r];
  };
  // rx_map layers: LLR i of CB r goes to layer i / N_cb (E > N_cb repeats the
  // circular buffer; rate_dematching_turbo sums the repeats in order of i)
  int layers = 1;
  for (int r = 0; r < p->C; ++r) {
    const int ncb = 3 * (p->cbs[r].K + 6);
    layers = std::max(layers, (p->cbs[r].E + ncb - 1) / ncb);
  }
  p->n_layers = layers;
  std::vector<int32_t> txm(p->n_re_bits), rxm((size_t)layers * p->n_re_bits, -1);
  for (int re = 0; re < n_re; ++re) {
    // TX: interleaved position re <- padded coded symbol q (ofdm_core.py:1046-1060)
    const int c = re / rows, rr = re % rows;
    const int q = rr * Nd + c;
    for (int m = 0; m < bps; ++m) {
      int32_t v;
      if (q >= ncs_tx) v = -2;
      else {
        const int e = q * bps + m;
        if (e >= p->coded_len) v = -1;
        else {
          int r, i;
          locate(e, r, i);
          const RmSrc s = rs[r][i];
          v = s.stream < 0 ? -1 : ((r * 3 + s.stream) * p->EW) * 32 + s.idx;
        }
      }
      txm[(size_t)re * bps + m] = v;
    }
    // RX: de-interleave (ofdm_core.py:1176-1197) then rate dematch rows
    int qr = -1;
    if (re < rows_rx * Nd) {
      const int c2 = re / rows_rx, r2 = re % rows_rx;
      qr = r2 * Nd + c2;
      if (qr >= ncs_rx) qr = -1;
    }
    for (int m = 0; m < bps; ++m) {
      if (qr < 0) continue;
      const int e = qr * bps + m;
      if (e >= p->coded_len) continue;
      int r, i;
      locate(e, r, i);
      const int K = p->cbs[r].K;
      const RmSrc s = rs[r][i];
      int row = -1;
      if (s.stream == 0) row = (int)(s.idx < K + 3 ? trow_ls(K, s.idx) : trow_ls2t(K, s.idx - K - 3));
      else if (s.stream == 1) row = (int)trow_lp(K, 1, s.idx);
      else if (s.stream == 2) row = (int)trow_lp(K, 2, s.idx);
      if (row >= 0) rxm[(size_t)(i / (3 * (K + 6))) * p->n_re_bits + (size_t)re * bps + m] = (r << 24) | row;
    }
  }
  p->qstride = Kmax + 32;
  std::vector<uint16_t> qm((size_t)p->C * p->qstride, 0);
  encode_qmask(p->cbs.data(), p->C, p->qstride, qm.data());
  if (upload(p->tx_map, txm) || upload(p->rx_map, rxm) || upload(p->cbi, p->cbs) || upload(p->enc_qmask, qm))
    return fail(LTE_ENOMEM, "map upload failed");
  // k_ofdm_txf's bank-aware lane order (SISO grids with whole 32-lane groups per
  // transform): off by default since round 5 -- it cut the modelled gather
  // conflicts 2.07 -> 0.19 cycles and the measured ones 0.91 -> 0.18 per LDS
  // instruction but not the kernel time (15.34 ms with it, 15.17 without,
  // DESIGN.md §5 round 4), and its greedy search costs plan-create time on every
  // plan-cache miss.  LTE_TXF_LANE_ORDER=1 turns it on.
  if (p->res == p->Nd && d.N >= 512 && p->Nd <= d.N / 2 && env_on("LTE_TXF_LANE_ORDER", false)) {
    std::vector<int32_t> tfm, tfr;
    plan_txf_lane_order(txm, p->gh.data, p->n_sym, Nd, bps, d.N / 2, tfm, tfr, p->txf_model);
    if (env_on("LTE_TXF_LANE_ORDER_REPORT", false))
      std::fprintf(stderr, "txf lane order: modelled extra LDS cycles per 32-lane gather %.3f (RE order) -> %.3f\n",
                   p->txf_model[0], p->txf_model[1]);
    if (upload(p->txf_map, tfm) || upload(p->txf_re, tfr)) return fail(LTE_ENOMEM, "map upload failed");
  }
  return LTE_OK;
}

// Per-TX CRS subsets (MIMOChannelEstimatorPeriodic.get_orthogonal_pilot_indices,
// core/mimo_channel_estimator_periodic.py:75-107: pilots[t::step], step =
// min(num_tx, 4); SFBCResourceMapper uses the same even/odd split for 2 TX)
// with PilotPattern(t % 4) symbols, gaps and, for every data SC that carries
// data, its left pilot within the subset.
static int plan_mimo_tables(lte_plan* p) {
  const lte_plan_desc& d = p->d;
  const int nt = d.num_tx, step = nt <= 4 ? nt : 4;
  std::vector<std::vector<int>> sub(nt);
  for (int t = 0; t < nt; ++t)
    for (int i = t % step; i < p->Np; i += step) sub[t].push_back(p->gh.pilot[i]);
  int maxP = 1;
  for (auto& v : sub) maxP = std::max<int>(maxP, (int)v.size());
  const int nd = p->mg.n_dsc;
  std::vector<int32_t> np(nt), ppos((size_t)nt * maxP, 0), pseg((size_t)nt * nd, -1);
  std::vector<float2> pval((size_t)nt * maxP, make_float2(0.f, 0.f));
  std::vector<float> pig((size_t)nt * maxP, 0.f);
  std::vector<double2> pval64((size_t)nt * maxP, make_double2(0.0, 0.0));
  std::vector<double> pig64((size_t)nt * maxP, 0.0);
  for (int t = 0; t < nt; ++t) {
    const int n = (int)sub[t].size();
    if (n < 1) return fail(LTE_EUNSUP, "no pilots for a TX antenna");
    np[t] = n;
    std::vector<double> pr;
    make_pilots(t % 4, n, pr);
    for (int i = 0; i < n; ++i) {
      ppos[(size_t)t * maxP + i] = sub[t][i];
      pval[(size_t)t * maxP + i] = make_float2((float)pr[2 * i], (float)pr[2 * i + 1]);
      pval64[(size_t)t * maxP + i] = make_double2(pr[2 * i], pr[2 * i + 1]);
      // np.linspace's step: delta * (1 / gap) (complex / int divides by Smith's rule)
      if (i + 1 < n) {
        pig64[(size_t)t * maxP + i] = 1.0 / (double)(sub[t][i + 1] - sub[t][i]);
        pig[(size_t)t * maxP + i] = (float)pig64[(size_t)t * maxP + i];
      }
    }
    int sidx = -1;
    for (int j = 0; j < nd; ++j) {
      const int k = p->gh.data[j];
      while (sidx + 1 < n && sub[t][sidx + 1] <= k) ++sidx;
      pseg[(size_t)t * nd + j] = sidx;
    }
  }
  if (upload(p->m_np, np) || upload(p->m_ppos, ppos) || upload(p->m_pseg, pseg) || upload(p->m_pval, pval) ||
      upload(p->m_pig, pig) || upload(p->m_pval64, pval64) || upload(p->m_pig64, pig64))
    return fail(LTE_ENOMEM, "mimo table upload failed");
  p->mg.maxP = maxP;
  p->mg.np_tx = p->m_np.p;
  p->mg.ppos = p->m_ppos.p;
  p->mg.pval = p->m_pval.p;
  p->mg.pig = p->m_pig.p;
  p->mg.pval64 = p->m_pval64.p;
  p->mg.pig64 = p->m_pig64.p;
  p->mg.pseg = p->m_pseg.p;
  return LTE_OK;
}

}  // extern "C"

// Device workspace of the SISO / SIMO chains in precision R.  The TX signal x
// is allocated on first use (the fused TX + channel path never writes it).
template <class R>
static bool alloc_siso(lte_plan* p, bool coded) {
  const lte_plan_desc& d = p->d;
  ChainBufs<R>& c = cbuf<R>(p);
  const size_t B = (size_t)d.max_frames;
  const int G = (int)((B + 63) / 64);
  const int rx = d.num_rx;
  const bool ray = d.channel == LTE_CH_RAYLEIGH;
  bool bad = false;
  if (ray) {
    bad |= c.y.alloc(B * rx * p->L) != 0;
    bad |= c.phases.alloc(std::max<size_t>(B * rx * d.n_paths * 16, 1)) != 0;
    bad |= c.coef.alloc(std::max<size_t>(B * rx * d.n_paths, 1)) != 0;
    std::vector<R> gh(d.gains, d.gains + d.n_paths);
    bad |= upload(c.gains, gh) != 0;
  }
  bad |= c.pow_part.alloc(B * rx * p->nblk) != 0;
  bad |= c.H.alloc(B * rx * p->n_grp * d.N) != 0;
  bad |= c.pstats.alloc(B * rx * p->n_grp * 2) != 0;
  bad |= c.npow.alloc(B * rx) != 0;
  bad |= c.snr_lin.alloc(B) != 0;
  if (coded) {
    // the fused demap path keeps (z, nv) = 3 R per RE here; the LLR path
    // (captures, QPSK) grows it to bps R per RE on first use
    const size_t n_re = p->n_re_bits / d.bps;
    bad |= c.llr.alloc(B * (d.bps >= 4 ? 3 * n_re : (size_t)p->n_re_bits)) != 0;
    c.blk.resize(p->C);
    c.ckpt.resize(p->C);
    std::vector<R*> bp(p->C);
    for (int r = 0; r < p->C; ++r) {
      const int K = p->cbs[r].K;
      bad |= c.blk[r].alloc((size_t)turbo_galloc(G) * turbo_rows(K) * 64) != 0;
      bad |= c.ckpt[r].alloc((size_t)turbo_galloc(G) * turbo_nwin(K) * turbo_ck_rows(sizeof(R) == 8) * 64) != 0;
      if (!bad && hipMemset(c.blk[r].p, 0, c.blk[r].n * sizeof(R)) != hipSuccess) bad = true;
      bp[r] = c.blk[r].p;
    }
    if (!bad) bad |= upload(c.blk_ptrs, bp) != 0;
  }
  return !bad;
}

// Device workspace of the multi-antenna chains in precision R.
template <class R>
static bool alloc_mimo(lte_plan* p, bool coded) {
  const lte_plan_desc& d = p->d;
  ChainBufs<R>& c = cbuf<R>(p);
  const size_t B = (size_t)d.max_frames;
  const int G = (int)((B + 63) / 64);
  const bool ray = d.channel == LTE_CH_RAYLEIGH;
  const MimoGrid& m = p->mg;
  const size_t links = (size_t)m.num_rx * m.num_tx;
  bool bad = false;
  // c.x (the TX streams) is allocated by run_mimo when a path writes it (the
  // fused flat-link TX never does)
  bad |= c.y.alloc(B * m.num_rx * p->L) != 0;
  bad |= c.coef.alloc(B * links * (ray ? d.n_paths : 1) * m.n_cs * (p->f64 ? mimo_ncf<double>() : mimo_ncf<float>())) != 0;
  if (ray && m.exact_jakes) bad |= c.phases.alloc(B * links * d.n_paths * 16) != 0;
  if (ray && d.chain != LTE_CHAIN_SPATIAL) {
    bad |= c.link_part.alloc(B * links * p->nblk) != 0;
    bad |= c.link_sigma.alloc(B * links) != 0;
  }
  // received grids and estimates: SFBC allocates them on the first run that
  // takes the separate receiver + detector (k_rx_sfbc never uses them);
  // spatial holds the pilot estimates (maxP per TX) until a run captures H
  if (m.mode != MIMO_SFBC) {
    bad |= c.Ym.alloc(B * p->n_sym * m.num_rx * m.n_dsc) != 0;
    bad |= c.H.alloc(B * m.num_rx * m.n_est * m.num_tx * std::min(m.maxP, m.n_dsc)) != 0;
  }
  if (ray) {
    std::vector<R> gh(d.gains, d.gains + d.n_paths);
    bad |= upload(c.gains, gh) != 0;
  }
  bad |= c.pow_part.alloc(B * m.num_rx * p->nblk) != 0;
  bad |= c.npow.alloc(B * m.num_rx) != 0;
  bad |= c.snr_lin.alloc(B) != 0;
  if (coded) {
    bad |= c.llr.alloc(B * p->n_re_bits) != 0;
    c.blk.resize(p->C);
    c.ckpt.resize(p->C);
    std::vector<R*> bp(p->C);
    for (int r = 0; r < p->C; ++r) {
      const int K = p->cbs[r].K;
      bad |= c.blk[r].alloc((size_t)turbo_galloc(G) * turbo_rows(K) * 64) != 0;
      bad |= c.ckpt[r].alloc((size_t)turbo_galloc(G) * turbo_nwin(K) * turbo_ck_rows(sizeof(R) == 8) * 64) != 0;
      if (!bad && hipMemset(c.blk[r].p, 0, c.blk[r].n * sizeof(R)) != hipSuccess) bad = true;
      bp[r] = c.blk[r].p;
    }
    if (!bad) bad |= upload(c.blk_ptrs, bp) != 0;
  }
  return !bad;
}

extern "C" {

static int plan_alloc(lte_plan* p) {
  const lte_plan_desc& d = p->d;
  const size_t B = (size_t)d.max_frames;
  const int G = (int)((B + 63) / 64);
  const bool coded = d.chain == LTE_CHAIN_CODED || d.chain == LTE_CHAIN_SFBC_CODED;
  bool bad = false;
  bad |= p->pw.alloc(B * p->PW) != 0;
  if (p->mimo) {
    bad |= !(p->f64 ? alloc_mimo<double>(p, coded) : alloc_mimo<float>(p, coded));
  } else if (p->bf) {   // per frame: the BfFrameT state and the noise scale (in snr_lin)
    if (p->f64) {
      bad |= p->bf_fr64.alloc(B) != 0;
      bad |= p->c64.snr_lin.alloc(B) != 0;
    } else {
      bad |= p->bf_fr.alloc(B) != 0;
      bad |= p->c32.snr_lin.alloc(B) != 0;
    }
  } else {
    bad |= !(p->f64 ? alloc_siso<double>(p, coded) : alloc_siso<float>(p, coded));
  }
  bad |= p->snr_idx.alloc(B) != 0;
  if (p->mimo) bad |= p->nvar.alloc(B) != 0;
  bad |= p->fid.alloc(B) != 0;
  bad |= p->frame_err.alloc(B) != 0;
  bad |= p->frame_crc.alloc(B) != 0;
  if (coded) {
    bad |= p->enc.alloc(B * p->enc_words) != 0;
    p->decb.resize(p->C);
    std::vector<int64_t> rows(p->C);
    std::vector<uint32_t*> dp(p->C);
    std::vector<int> kw(p->C);
    for (int r = 0; r < p->C; ++r) {
      const int K = p->cbs[r].K;
      rows[r] = turbo_rows(K);
      kw[r] = turbo_kw(K);
      bad |= p->decb[r].alloc((size_t)G * kw[r] * 64) != 0;
      dp[r] = p->decb[r].p;
    }
    if (!bad) bad |= upload(p->rows_dev, rows) || upload(p->dec_ptrs, dp) || upload(p->kw_dev, kw);
  }
  if (bad) return fail(LTE_ENOMEM, "device workspace allocation failed (max_frames too large?)");
  return LTE_OK;
}

int lte_plan_create(const lte_plan_desc* desc, lte_plan** out) {
  if (!desc || !out) return fail(LTE_EINVAL, "null argument");
  const lte_plan_desc& d = *desc;
  if (d.N < 128 || d.N > 2048 || (d.N & (d.N - 1))) return fail(LTE_EUNSUP, "N must be a power of two in [128, 2048]");
  if (d.Nc <= 0 || d.Nc >= d.N || d.cp_len < 0 || d.cp_len > d.N) return fail(LTE_EINVAL, "bad Nc / cp_len");
  if (d.bps != 2 && d.bps != 4 && d.bps != 6) return fail(LTE_EINVAL, "Unsupported modulation");
  if (d.chain < 0 || d.chain > LTE_CHAIN_BEAMFORMING) return fail(LTE_EINVAL, "bad chain");
  if (d.channel != LTE_CH_AWGN && d.channel != LTE_CH_RAYLEIGH) return fail(LTE_EINVAL, "Tipo de canal desconocido");
  if (d.num_rx < 1 || d.num_rx > 16) return fail(LTE_EINVAL, "num_rx must be >= 1");
  const bool bf = d.chain == LTE_CHAIN_BEAMFORMING;
  const bool mimo = d.chain >= LTE_CHAIN_SFBC && !bf;
  const int num_tx = d.num_tx > 0 ? d.num_tx : 1;
  if (!mimo && !bf && num_tx != 1) return fail(LTE_EINVAL, "num_tx > 1 needs a multi-antenna chain");
  if (!mimo && !bf && d.chain != LTE_CHAIN_SIMO && d.num_rx != 1)
    return fail(LTE_EINVAL, "SISO chains need num_rx == 1");
  if (bf && num_tx != 2 && num_tx != 4 && num_tx != 8)
    return fail(LTE_EINVAL, "num_tx=" + std::to_string(num_tx) + " no soportado en TM6");
  if (bf && d.num_rx > LTE_BF_MAX_RX) return fail(LTE_EUNSUP, "beamforming: at most 8 RX antennas");
  if ((d.chain == LTE_CHAIN_SFBC || d.chain == LTE_CHAIN_SFBC_CODED) && num_tx != 2)
    return fail(LTE_EINVAL, "Alamouti SFBC requires exactly 2 TX antennas");
  if ((d.chain == LTE_CHAIN_SFBC || d.chain == LTE_CHAIN_SFBC_CODED) && d.num_rx > 8)
    return fail(LTE_EUNSUP, "SFBC: at most 8 RX antennas");
  const int rank = d.chain == LTE_CHAIN_SPATIAL ? (d.rank > 0 ? d.rank : num_tx) : 0;
  if (d.chain == LTE_CHAIN_SPATIAL) {
    if (d.num_rx < rank)
      return fail(LTE_EINVAL, "num_rx (" + std::to_string(d.num_rx) + ") debe ser >= num_layers (" +
                                  std::to_string(rank) + ")");
    if (d.detector < LTE_DET_MMSE || d.detector > LTE_DET_MRC) return fail(LTE_EINVAL, "Detector no soportado");
    if (d.detector == LTE_DET_MRC && rank != 1) return fail(LTE_EINVAL, "MRC solo soporta num_layers=1 (rank-1)");
    if ((num_tx != 2 && num_tx != 4) || d.num_rx > 4 || rank < 1 || rank > num_tx)
      return fail(LTE_EUNSUP, "spatial multiplexing on the GPU path: 2 or 4 TX, 1-4 RX, rank <= num_tx");
  }
  if (d.channel == LTE_CH_RAYLEIGH && (d.n_paths < 1 || d.n_paths > LTE_MAX_PATHS))
    return fail(LTE_EINVAL, "bad n_paths");
  if (d.max_frames < 1) return fail(LTE_EINVAL, "max_frames must be >= 1");
  if (d.n_bits < 1) return fail(LTE_EINVAL, "Bits array cannot be empty");
  if (d.precision != LTE_PREC_DEFAULT && d.precision != LTE_PREC_F32 && d.precision != LTE_PREC_F64)
    return fail(LTE_EINVAL, "precision must be LTE_PREC_DEFAULT, LTE_PREC_F32 or LTE_PREC_F64");
  // float64 (the reference's arithmetic) is the default of every chain
  lte_plan* p = new lte_plan();
  p->d = d;
  p->d.num_tx = num_tx;
  p->mimo = mimo;
  p->f64 = d.precision != LTE_PREC_F32;
  const bool coded = d.chain == LTE_CHAIN_CODED || d.chain == LTE_CHAIN_SFBC_CODED;
  if (coded && d.turbo_iters < 0) { delete p; return fail(LTE_EINVAL, "bad turbo_iters"); }
  int rc = plan_tables(p);
  if (rc) { delete p; return rc; }
  // Nd < N/2 is assumed by k_rx_data (4 data REs per thread)
  if (p->Nd * 2 >= d.N) { delete p; return fail(LTE_EUNSUP, "Nd >= N/2 not supported"); }
  const bool sfbc = d.chain == LTE_CHAIN_SFBC || d.chain == LTE_CHAIN_SFBC_CODED;
  // REs per OFDM symbol: SFBC drops an odd last data SC (core/sfbc_alamouti.py:196-200, Q18)
  p->res = sfbc ? (p->Nd & ~1) : p->Nd;
  if (coded) {
    rc = plan_coded_maps(p);
    if (rc) { p->tabs.release(); delete p; return rc; }
    p->PW = (d.n_bits + 24 + 31) / 32 + 1;
  } else {
    if (d.n_sym < 1) { delete p; return fail(LTE_EINVAL, "n_sym must be >= 1"); }
    p->n_sym = d.n_sym;
    if ((int64_t)d.n_bits > (int64_t)p->n_sym * p->res * d.bps) { delete p; return fail(LTE_EINVAL, "n_bits exceeds frame capacity"); }
    p->PW = (p->n_sym * p->res * d.bps + 31) / 32 + 1;
  }
  p->L = bf ? p->n_sym * p->Nd : p->n_sym * (d.N + d.cp_len);   // beamforming: REs per antenna
  p->n_grp = (p->n_sym + 13) / 14;
  p->nblk = bf ? (p->L + 255) / 256 : std::max((p->L + 255) / 256, mimo_channel_nblk(p->L, d.N + d.cp_len));
  p->bf = bf;
  if (bf) {   // rank-1 codebook (TM6 == TM4 rank 1), core/codebook_lte.py:58-96
    std::vector<double> cb;
    const double r2 = 1.0 / std::sqrt(2.0);
    if (num_tx == 2) {
      const double v[4][2] = {{1, 0}, {-1, 0}, {0, 1}, {0, -1}};
      for (int i = 0; i < 4; ++i) {
        cb.push_back(r2); cb.push_back(0.0);
        cb.push_back(v[i][0] * r2); cb.push_back(v[i][1] * r2);
      }
    } else {
      const double sc = num_tx == 4 ? 0.5 : 1.0 / std::sqrt(8.0);
      for (int i = 0; i < 16; ++i)
        for (int a = 0; a < num_tx; ++a) {
          const double ph = 2.0 * M_PI * i * a / 16.0;
          cb.push_back(std::cos(ph) * sc);
          cb.push_back(std::sin(ph) * sc);
        }
    }
    p->bf_ncb = (int)(cb.size() / (2 * num_tx));
    if (upload(p->bf_cb, cb)) { p->tabs.release(); delete p; return fail(LTE_ENOMEM, "codebook upload"); }
  }
  if (mimo) {
    MimoGrid& m = p->mg;
    m.mode = sfbc ? MIMO_SFBC : MIMO_SPATIAL;
    m.num_tx = num_tx;
    m.num_rx = d.num_rx;
    m.res = p->res;
    m.rank = rank;
    m.det = d.detector;
    m.n_dsc = sfbc ? p->res : (p->Nd + rank - 1) / rank;   // layers fill the first ceil(Nd/rank) data SCs (Q20)
    m.n_est = sfbc ? p->n_grp : p->n_sym;
    // fD != 0: the Jakes sum expanded per OFDM symbol (f32 second order, f64
    // degree 5); past mimo_taylor_ok f64 evaluates it per sample (jw[m] = (2 pi
    // fD) cos(alpha_m), rayleighchannel.py:28-38)
    m.exact_jakes = d.channel == LTE_CH_RAYLEIGH && d.fD != 0.0 &&
                    !mimo_taylor_ok_prec(p->f64, d.fD, d.fs, d.N + d.cp_len);
    for (int k = 0; k < 16; ++k) m.jw[k] = 6.283185307179586 * d.fD * std::cos(6.283185307179586 * (k + 1) / 16.0);
    m.n_cs = (d.channel == LTE_CH_RAYLEIGH && d.fD != 0.0 && !m.exact_jakes) ? p->n_sym : 1;
    rc = plan_mimo_tables(p);
    if (rc) { p->tabs.release(); delete p; return rc; }
    if (!sfbc) {   // precoder W [num_tx][rank] in a [4][4] table; rank 0 in the descriptor -> identity
      std::vector<double> w4(32, 0.0);
      for (int t = 0; t < num_tx; ++t)
        for (int c = 0; c < rank; ++c) {
          if (d.rank > 0) {
            w4[(t * 4 + c) * 2] = d.precoder[(t * 4 + c) * 2];
            w4[(t * 4 + c) * 2 + 1] = d.precoder[(t * 4 + c) * 2 + 1];
          } else {
            w4[(t * 4 + c) * 2] = t == c ? 1.0 : 0.0;
          }
        }
      if (upload(p->m_W, w4)) { p->tabs.release(); delete p; return fail(LTE_ENOMEM, "precoder upload"); }
      m.W = p->m_W.p;
    }
  }
  p->grid = Grid{d.N, p->log2N, d.Nc, d.cp_len, p->Nd, p->Np, d.bps, p->n_sym, p->L, p->n_grp,
                 p->tabs.data.p, p->tabs.pilot.p, p->tabs.pilots.p, p->tabs.seg.p, p->tabs.inv_gap.p,
                 p->tabs.tw.p, p->tabs.constel.p,
                 (float)(d.bps == 2 ? std::sqrt(2.0) : d.bps == 4 ? std::sqrt(10.0) : std::sqrt(42.0)),
                 p->tabs.chirp.p, p->tabs.bhat.p, d.no_equalization && d.chain == LTE_CHAIN_UNCODED ? 1 : 0,
                 p->tabs.pilots64.p, p->tabs.inv_gap64.p, p->tabs.tw64.p, p->tabs.chirp64.p, p->tabs.bhat64.p,
                 p->tabs.kinfo.p};
  if (d.channel == LTE_CH_RAYLEIGH) {
    std::vector<int32_t> dl(d.delays, d.delays + d.n_paths);
    for (int i = 0; i < d.n_paths; ++i)
      if (dl[i] < 0) { p->tabs.release(); delete p; return fail(LTE_EINVAL, "negative delay"); }
    if (upload(p->delays, dl)) { p->tabs.release(); delete p; return fail(LTE_ENOMEM, "upload"); }
  }
  if (hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess) {
    delete p;
    return fail(LTE_EHIP, "stream creation failed");
  }
  rc = plan_alloc(p);
  if (rc) { lte_plan_destroy(p); return rc; }
  if (p->counts.alloc(4 * 64)) { lte_plan_destroy(p); return fail(LTE_ENOMEM, "counts"); }
  *out = p;
  return LTE_OK;
}

int lte_plan_destroy(lte_plan* p) {
  if (!p) return LTE_OK;
  if (p->stream) (void)hipStreamSynchronize(p->stream);
  p->tabs.release();
  p->cbi.release(); p->tx_map.release(); p->rx_map.release(); p->delays.release();
  p->txf_map.release(); p->txf_re.release();
  p->pw.release(); p->enc.release(); p->inj_bits.release(); p->inj_bytes.release(); p->enc_qmask.release();
  p->c32.release(); p->c64.release();
  p->frame_err.release(); p->frame_crc.release(); p->snr_idx.release(); p->nvar.release(); p->fid.release(); p->counts.release();
  p->cap_bits.release();
  for (auto& b : p->decb) b.release();
  p->rows_dev.release(); p->dec_ptrs.release(); p->kw_dev.release();
  p->m_np.release(); p->m_ppos.release(); p->m_pseg.release(); p->m_pval.release(); p->m_pval64.release();
  p->m_pig.release(); p->m_pig64.release(); p->m_W.release(); p->bf_cb.release();
  p->bf_fr.release();
  p->bf_fr64.release();
  for (auto e : p->evpool) (void)hipEventDestroy(e);
  if (p->stream) (void)hipStreamDestroy(p->stream);
  delete p;
  return LTE_OK;
}

int lte_plan_info(const lte_plan* p, int64_t* info) {
  if (!p || !info) return fail(LTE_EINVAL, "null argument");
  info[0] = p->L; info[1] = p->n_sym; info[2] = p->Nd; info[3] = p->Np;
  info[4] = p->n_grp; info[5] = p->C; info[6] = p->coded_len; info[7] = p->n_re_bits;
  return LTE_OK;
}

int lte_plan_precision(const lte_plan* p) {
  if (!p) return fail(LTE_EINVAL, "null plan");
  return p->f64 ? LTE_PREC_F64 : LTE_PREC_F32;
}

int lte_timing_enable(lte_plan* p, int on) {
  if (!p) return fail(LTE_EINVAL, "null plan");
  p->timing = on != 0;
  return LTE_OK;
}

int lte_timing_reset(lte_plan* p) {
  if (!p) return fail(LTE_EINVAL, "null plan");
  for (int i = 0; i < KN_COUNT; ++i) { p->kms[i] = 0; p->klaunch[i] = 0; }
  return LTE_OK;
}

int lte_timing_read(lte_plan* p, char* names, int names_len, double* ms, int64_t* launches, int n_max) {
  if (!p) return fail(LTE_EINVAL, "null plan");
  std::string s;
  for (int i = 0; i < KN_COUNT; ++i) {
    if (i) s += ",";
    s += KNAMES[i];
    if (i < n_max) {
      if (ms) ms[i] = p->kms[i];
      if (launches) launches[i] = p->klaunch[i];
    }
  }
  if (names && names_len > 0) {
    std::strncpy(names, s.c_str(), names_len - 1);
    names[names_len - 1] = 0;
  }
  return KN_COUNT;
}

static void pack_bits(const uint8_t* bits, int n, uint32_t* w, int nw) {
  std::memset(w, 0, sizeof(uint32_t) * nw);
  for (int i = 0; i < n; ++i)
    if (bits[i] & 1) w[i >> 5] |= 1u << (31 - (i & 31));
}

}  // extern "C"

// Host injection (float64 from the caller) -> device buffer of R, frames
// [0, nf) of `per` values each; synchronous (the host copy is a temporary).
template <class R>
static int upload_inj(DBuf<R>& dst, const double* src, int64_t stride, int B, size_t per, hipStream_t s,
                      const R** out, int64_t* out_stride) {
  const int nf = stride ? B : 1;
  if (dst.alloc((size_t)nf * per)) return fail(LTE_ENOMEM, "injection buffer");
  if (sizeof(R) == 8 && (!stride || (size_t)stride == per)) {   // float64, dense: straight from the caller
    HIPCHK(hipMemcpyAsync(dst.p, src, (size_t)nf * per * sizeof(R), hipMemcpyHostToDevice, s));
  } else {
    std::vector<R> h((size_t)nf * per);
    for (int f = 0; f < nf; ++f)
      for (size_t i = 0; i < per; ++i) h[f * per + i] = (R)src[(size_t)f * stride + i];
    HIPCHK(hipMemcpyAsync(dst.p, h.data(), h.size() * sizeof(R), hipMemcpyHostToDevice, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  *out = dst.p;
  *out_stride = stride ? (int64_t)per : 0;
  return LTE_OK;
}

// (z, nv) of the fused demap path in the LLR buffer: [max_frames][n_re] z,
// then the noise variances (see demap_in_dematch; k_det_sfbc's per RE pair)
template <class R>
static cx<R>* zn_z(lte_plan* p) { return reinterpret_cast<cx<R>*>(cbuf<R>(p).llr.p); }
template <class R>
static R* zn_nv(lte_plan* p) {
  return cbuf<R>(p).llr.p + 2 * (size_t)p->d.max_frames * (p->n_re_bits / p->d.bps);
}

// Multi-antenna chains (SFBC 2xN, uncoded / coded; TM4 spatial multiplexing)
// in precision R.
template <class R>
static int run_mimo(lte_plan* p, const lte_run_args* a, int B, int n_snr, const std::vector<double>& snr_lin,
                    const uint32_t* inj_bits, int64_t inj_bits_stride) {
  using V = cx<R>;
  const lte_plan_desc& d = p->d;
  const Grid& g = p->grid;
  const MimoGrid& m = p->mg;
  ChainBufs<R>& c = cbuf<R>(p);
  hipStream_t s = p->stream;
  const bool coded = d.chain == LTE_CHAIN_SFBC_CODED;
  const bool ray = d.channel == LTE_CH_RAYLEIGH;
  const bool sfbc = m.mode == MIMO_SFBC;
  const bool link_noise = sfbc && ray;  // transmit_mimo's per-link 100 dB ChannelSimulator (core/ofdm_core.py:490-503)
  const size_t links = (size_t)m.num_rx * m.num_tx;
  std::vector<R> sl(B);
  for (int b = 0; b < B; ++b) sl[b] = (R)snr_lin[b];
  HIPCHK(hipMemcpyAsync(c.snr_lin.p, sl.data(), B * sizeof(R), hipMemcpyHostToDevice, s));
  std::vector<double> nv;
  if (!sfbc) {   // MIMODetector's noise_variance = 10 ** (-snr_db / 10) (core/ofdm_core.py:2737), float64
    nv.resize(B);
    for (int b = 0; b < B; ++b) nv[b] = std::pow(10.0, -a->snr_db[b] / 10.0);
    HIPCHK(hipMemcpyAsync(p->nvar.p, nv.data(), B * sizeof(double), hipMemcpyHostToDevice, s));
  }
  // injections (the reference's own draws, ref-compat mode)
  const R *inj_ph = nullptr, *inj_z = nullptr, *inj_lz = nullptr, *inj_lh = nullptr;
  int64_t inj_ph_stride = 0, inj_z_stride = 0, inj_lz_stride = 0, inj_lh_stride = 0;
  if (a->phases && ray) {
    const int e = upload_inj<R>(c.inj_ph, a->phases, a->phases_stride, B, links * d.n_paths * 16, s, &inj_ph,
                                &inj_ph_stride);
    if (e != LTE_OK) return e;
  }
  if (a->noise) {
    const int e = upload_inj<R>(c.inj_z, a->noise, a->noise_stride, B, (size_t)m.num_rx * 2 * p->L, s, &inj_z,
                                &inj_z_stride);
    if (e != LTE_OK) return e;
  }
  if (a->link_noise && link_noise) {
    const int e = upload_inj<R>(c.inj_lz, a->link_noise, a->link_noise_stride, B, links * 2 * p->L, s, &inj_lz,
                                &inj_lz_stride);
    if (e != LTE_OK) return e;
  }
  if (a->link_h && !ray && !sfbc) {
    const int e = upload_inj<R>(c.inj_lh, a->link_h, a->link_h_stride, B, links * 2, s, &inj_lh, &inj_lh_stride);
    if (e != LTE_OK) return e;
  }
  {
    Timer t(p, KN_PAYLOAD);
    LCHK(launch_payload(s, p->pw.p, p->PW, d.n_bits, coded ? CRC24A_POLY : 0, p->fid.p, a->seed, B, inj_bits, inj_bits_stride));
  }
  if (coded) {
    Timer t(p, KN_ENCODE);
    LCHK(launch_encode(s, p->pw.p, p->PW, p->KWmax, p->enc.p, p->EW, p->cbi.p, p->C, B, p->enc_qmask.p, p->qstride));
  }
  const int np = ray ? d.n_paths : 1;
  R* phases = (ray && m.exact_jakes) ? c.phases.p : nullptr;
  {
    Timer t(p, KN_FADING);
    LCHK(launch_fading_mimo<R>(s, g, m, B, ray ? 1 : 0, d.n_paths, c.gains.p, d.fD, d.fs, p->fid.p, a->seed, inj_ph,
                               inj_ph_stride, inj_lh, inj_lh_stride, c.coef.p, phases));
  }
  // transmit_mimo's link power on the TX symbols in LDS (static taps, N >= 512,
  // delays within the CP): the channel pass then reads x once
  TxLinkPower<R> lp{};
  const int maxd = ray ? *std::max_element(d.delays, d.delays + d.n_paths) : 0;
  const bool lp_fuse = link_noise && m.n_cs == 1 && !m.exact_jakes && (g.N >> 3) >= 64 && maxd <= g.cp &&
                       d.n_paths <= TXCH_MAXP &&
                       env_on("LTE_MIMO_LP_FUSE", true);
  // (partials [link][symbol]: the layout k_link_power writes, nch = n_sym blocks per link)
  if (lp_fuse) lp = TxLinkPower<R>{p->delays.p, c.coef.p, c.link_part.p, d.n_paths, maxd,
                                   mimo_channel_nblk(p->L, g.N + g.cp)};
  // flat links (AWGN: spatial CN(0,1), SFBC exp(j t pi/2)): TX and channel in
  // one pass per (frame, symbol, RX) -- y_r = IFFT(sum_t h_rt G_t) -- when no
  // TX-stream capture needs x
  const int nch = mimo_channel_nblk(p->L, g.N + g.cp);
  const bool flat_fuse = !ray && !a->cap_signal_tx && !a->cap_link_stats && (g.N >> 3) >= 64 && m.num_tx <= 4 &&
                         env_on("LTE_MIMO_FLAT_FUSE", true);
  // config 4 (SFBC, static-tap Rayleigh links with the 100 dB link noise, Philox
  // draws): TX and the links' fading in one pass per frame writing the faded RX
  // signals (k_ofdm_txch_sfbc), then the link noise + RX power (k_link_noise_pairs)
  // -- x never goes through HBM.  Captures of x / the link statistics and the
  // reference's own (injected) link noise keep the separate kernels.
  int npow_nblk = nch;   // RX power partials per (frame, RX) that k_npow_mimo sums
  const bool sfbc_fuse = link_noise && !inj_lz && !inj_z && !a->cap_signal_tx && !a->cap_link_stats &&
                         sfbc_txch_supported<R>(g, m, d.n_paths, maxd) && env_on("LTE_SFBC_TXCH_FUSE", true);
  // the merged link noise (launch_npow_sfbc_merged): the fused TX, then one
  // noise draw per RX sample in the fused receiver -- only when nothing
  // observes the received streams or noise powers in between
  const bool zn0_ = coded && (d.bps == 4 || d.bps == 6) && !a->cap_llr && (m.res & 1) == 0 && m.n_dsc <= m.res &&
                    env_on("LTE_DEMAP_IN_DEMATCH", true);
  const bool sfbc_merge = sfbc_fuse && !a->cap_signal_rx && !a->cap_noise_power && !a->cap_H && !a->cap_data_syms &&
                          !(a->cap_bits_rx && !coded) && (zn0_ || !coded) && rx_sfbc_supported<R>(g, m) &&
                          env_on("LTE_SFBC_RX_FUSE", true) && env_on("LTE_SFBC_LINK_MERGE", true);
  if (sfbc_fuse) {
    TxLinkPower<R> lf{p->delays.p, c.coef.p, c.link_part.p, d.n_paths, maxd, 1};
    lf.merged = sfbc_merge ? 1 : 0;
    {
      Timer t(p, KN_OFDM_TX);
      LCHK(launch_ofdm_txch_sfbc<R>(s, g, m, coded ? 1 : 0, p->pw.p, p->PW, p->enc.p, p->enc_words, p->tx_map.p, lf,
                                    c.y.p, B));
    }
    // (chunks of frames with each chunk's noise pass on a second stream beside
    // the next chunk's TX measured no overlap: TX + noise 67.3-68.0 ms per
    // 65 536 frames with 1, 2, 4 or 8 chunks)
    Timer t(p, KN_CHANNEL);
    if (sfbc_merge)
      LCHK(launch_npow_sfbc_merged<R>(s, B, m.num_rx, m.num_tx, c.link_part.p, p->L, c.snr_lin.p, c.npow.p));
    else
      LCHK(launch_link_noise_add<R>(s, g, m, B, c.link_part.p, c.link_sigma.p, c.y.p, p->fid.p, a->seed,
                                    c.pow_part.p, &npow_nblk));
  } else if (flat_fuse) {
    Timer t(p, KN_OFDM_TX);
    LCHK(launch_ofdm_txch_flat<R>(s, g, m, coded ? 1 : 0, p->pw.p, p->PW, p->enc.p, p->enc_words, p->tx_map.p,
                                  c.coef.p, c.y.p, c.pow_part.p, nch, B));
  } else {
    if (c.x.alloc((size_t)d.max_frames * m.num_tx * p->L)) return fail(LTE_ENOMEM, "TX signal buffer");
    {
      Timer t(p, KN_OFDM_TX);
      LCHK(launch_ofdm_tx_mimo<R>(s, g, m, coded ? 1 : 0, p->pw.p, p->PW, p->enc.p, p->enc_words, p->tx_map.p, c.x.p,
                                  B, lp));
    }
    Timer t(p, KN_CHANNEL);
    LCHK(launch_channel_mimo<R>(s, g, m, B, np, ray ? p->delays.p : nullptr, c.coef.p, phases, c.gains.p, d.fs, c.x.p,
                                c.y.p, link_noise ? 1 : 0, p->fid.p, a->seed, inj_lz, inj_lz_stride, c.link_part.p,
                                c.link_sigma.p, c.pow_part.p, p->nblk, lp_fuse ? 1 : 0));
  }
  if (!sfbc_merge) {
    Timer t(p, KN_CHANNEL);
    // noise per RX: SFBC (P / num_tx) / SNR (core/ofdm_core.py:524-534); spatial P / SNR (channel.py:457-467)
    LCHK(launch_npow_mimo<R>(s, B, m.num_rx, c.pow_part.p, npow_nblk, p->L, c.snr_lin.p, sfbc ? (double)m.num_tx : 1.0,
                             c.npow.p));
  }
  // config 4 (SFBC on Philox draws, zn handoff or uncoded, no capture of the
  // received grids / estimates / symbols): receiver + detector in one pass
  const bool zn0 = coded && sfbc && (d.bps == 4 || d.bps == 6) && !a->cap_llr && (m.res & 1) == 0 &&
                   m.n_dsc <= m.res && env_on("LTE_DEMAP_IN_DEMATCH", true);
  // (a capture of the received bits needs the detector's decisions only
  // uncoded: coded, they come from k_crc_count)
  const bool rx_fuse = sfbc && !inj_z && !a->cap_H && !a->cap_data_syms && !(a->cap_bits_rx && !coded) &&
                       (zn0 || !coded) &&
                       rx_sfbc_supported<R>(g, m) && env_on("LTE_SFBC_RX_FUSE", true);
  if (sfbc_merge && !rx_fuse) return fail(LTE_EINVAL, "merged link noise without the fused SFBC receiver");
  // spatial multiplexing without a capture of H: the receiver hands over each
  // estimation symbol's LS pilot estimates and the detector interpolates them
  // per RE (the same mimo_interp), instead of a round trip of the interpolated
  // H (num_tx x n_dsc per RX and symbol) through HBM
  const bool h_pilots = !sfbc && !a->cap_H && env_on("LTE_SPATIAL_HP", true);
  if (rx_fuse) {
    Timer t(p, KN_RX_CHEST);
    LCHK(launch_rx_sfbc<R>(s, g, m, coded ? 1 : 0, B, c.y.p, c.npow.p, p->fid.p, a->seed, c.snr_lin.p, p->pw.p,
                           p->PW, d.n_bits, p->frame_err.p, coded ? zn_z<R>(p) : nullptr,
                           coded ? zn_nv<R>(p) : nullptr));
  } else {
    if (c.Ym.alloc((size_t)d.max_frames * p->n_sym * m.num_rx * m.n_dsc) ||
        c.H.alloc((size_t)d.max_frames * m.num_rx * m.n_est * m.num_tx * (h_pilots ? m.maxP : m.n_dsc)))
      return fail(LTE_ENOMEM, "received grids / estimates");
    Timer t(p, KN_RX_CHEST);
    LCHK(launch_rx_fft_mimo<R>(s, g, m, B, c.y.p, c.npow.p, p->fid.p, a->seed, inj_z, inj_z_stride, c.Ym.p, c.H.p,
                               h_pilots ? 1 : 0));
  }
  V* cap_syms_dev = nullptr;
  uint8_t* cap_bits_dev = nullptr;
  if (a->cap_data_syms) {
    if (c.capbuf.alloc((size_t)B * p->n_sym * m.res)) return fail(LTE_ENOMEM, "capture");
    cap_syms_dev = c.capbuf.p;
  }
  if (a->cap_bits_rx) {
    if (p->cap_bits.alloc((size_t)B * d.n_bits)) return fail(LTE_ENOMEM, "capture");
    cap_bits_dev = p->cap_bits.p;
  }
  // coded SFBC 16/64-QAM without an LLR capture: the detector hands over the
  // combined symbols and each RE pair's sigma^2_eff, k_dematch_zn demaps (as
  // the SISO chain does; LTE_DEMAP_IN_DEMATCH=0 keeps the LLR round trip)
  const bool zn = zn0;
  if (!rx_fuse) {
    Timer t(p, KN_RX_DATA);
    if (sfbc)
      LCHK(launch_det_sfbc<R>(s, g, m, coded ? 1 : 0, ray ? 1 : 0, B, c.Ym.p, c.H.p, c.snr_lin.p, p->pw.p, p->PW,
                              d.n_bits, p->frame_err.p, c.llr.p, cap_syms_dev, coded ? nullptr : cap_bits_dev,
                              zn ? zn_z<R>(p) : nullptr, zn ? zn_nv<R>(p) : nullptr));
    else
      LCHK(launch_det_spatial<R>(s, g, m, B, c.Ym.p, c.H.p, p->nvar.p, p->pw.p, p->PW, d.n_bits, p->frame_err.p,
                                 cap_syms_dev, cap_bits_dev, h_pilots ? 1 : 0));
  }
  if (coded) {
    {
      Timer t(p, KN_DEMATCH);
      if (zn)
        LCHK(launch_dematch_zn<R>(s, zn_z<R>(p), zn_nv<R>(p), p->n_re_bits / d.bps, m.res, d.bps, B, p->rx_map.p,
                                  p->n_layers, c.blk_ptrs.p, p->rows_dev.p, turbo_plan_ch(p), 0, 1));
      else
        LCHK(launch_dematch<R>(s, c.llr.p, p->n_re_bits, B, p->rx_map.p, p->n_layers, c.blk_ptrs.p, p->rows_dev.p,
                                 turbo_plan_ch(p)));
    }
    const int G = (B + 63) / 64;
    std::vector<TurboJob> jobs(p->C);
    for (int r = 0; r < p->C; ++r) {
      const CbInfo& cb = p->cbs[r];
      jobs[r] = TurboJob{c.blk[r].p, c.ckpt[r].p, p->decb[r].p, cb.K, cb.f1, cb.f2, G, turbo_plan_ch(p)};
    }
    {
      Timer t(p, KN_TURBO);
      LCHK(launch_turbo_jobs(s, jobs.data(), p->C, d.turbo_iters, TM_DEC1, sizeof(R) == 8 ? 1 : 0));
    }
    {
      Timer t(p, KN_CRC);
      LCHK(launch_crc_count(s, p->cbi.p, p->C, p->dec_ptrs.p, p->kw_dev.p, B, p->pw.p, p->PW, d.n_bits,
                            p->frame_err.p, p->frame_crc.p, cap_bits_dev, 0, inj_bits ? nullptr : p->fid.p,
                            a->seed));
    }
  }
  {
    Timer t(p, KN_ACC);
    LCHK(launch_accumulate(s, B, coded ? 1 : 0, d.n_bits, n_snr, p->snr_idx.p, p->frame_err.p, p->frame_crc.p, p->counts.p));
  }
  std::vector<unsigned long long> hc((size_t)4 * n_snr);
  HIPCHK(hipMemcpyAsync(hc.data(), p->counts.p, hc.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
  if (a->frame_errors)
    HIPCHK(hipMemcpyAsync(a->frame_errors, p->frame_err.p, B * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  std::vector<uint32_t> crc;
  if (a->frame_crc_ok && coded) {
    crc.resize(B);
    HIPCHK(hipMemcpyAsync(crc.data(), p->frame_crc.p, B * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  }
  if (a->cap_signal_tx)
    HIPCHK(hipMemcpyAsync(a->cap_signal_tx, c.x.p, (size_t)B * m.num_tx * p->L * sizeof(V), hipMemcpyDeviceToHost, s));
  if (a->cap_signal_rx) {
    DBuf<V> tmp;
    if (tmp.alloc((size_t)B * m.num_rx * p->L)) return fail(LTE_ENOMEM, "capture");
    {
      Timer t(p, KN_CAP);
      hipLaunchKernelGGL(k_cap_rx<R>, dim3(((p->L + 255) / 256) * B, m.num_rx), dim3(256), 0, s, p->L, m.num_rx, B,
                         c.y.p, (int64_t)p->L, (int64_t)m.num_rx * p->L, c.npow.p, p->fid.p, a->seed, inj_z,
                         inj_z_stride, tmp.p);
      LCHK((int)hipGetLastError());
    }
    HIPCHK(hipMemcpyAsync(a->cap_signal_rx, tmp.p, (size_t)B * m.num_rx * p->L * sizeof(V), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    tmp.release();
  }
  if (a->cap_data_syms)
    HIPCHK(hipMemcpyAsync(a->cap_data_syms, cap_syms_dev, (size_t)B * p->n_sym * m.res * sizeof(V),
                          hipMemcpyDeviceToHost, s));
  if (a->cap_H)   // multi-antenna layout [B][num_rx][n_est][num_tx][n_dsc]
    HIPCHK(hipMemcpyAsync(a->cap_H, c.H.p, (size_t)B * m.num_rx * m.n_est * m.num_tx * m.n_dsc * sizeof(V),
                          hipMemcpyDeviceToHost, s));
  if (a->cap_bits_rx)
    HIPCHK(hipMemcpyAsync(a->cap_bits_rx, cap_bits_dev, (size_t)B * d.n_bits, hipMemcpyDeviceToHost, s));
  if (a->cap_llr && coded)
    HIPCHK(hipMemcpyAsync(a->cap_llr, c.llr.p, (size_t)B * p->n_re_bits * sizeof(R), hipMemcpyDeviceToHost, s));
  if (a->cap_noise_power)
    HIPCHK(hipMemcpyAsync(a->cap_noise_power, c.npow.p, (size_t)B * m.num_rx * sizeof(R), hipMemcpyDeviceToHost, s));
  DBuf<R> lpart, lstats;
  if (a->cap_link_stats) {
    const int nb = (p->L + 255) / 256;
    if (lpart.alloc((size_t)B * links * 4 * nb) || lstats.alloc((size_t)B * links * 4))
      return fail(LTE_ENOMEM, "capture");
    {
      Timer t(p, KN_CAP);
      LCHK(launch_link_stats<R>(s, g, m, B, np, ray ? p->delays.p : nullptr, c.coef.p, phases, c.gains.p, d.fs, c.x.p,
                                link_noise ? c.link_sigma.p : nullptr, p->fid.p, a->seed, inj_lz, inj_lz_stride,
                                lpart.p, nb, lstats.p));
    }
    HIPCHK(hipMemcpyAsync(a->cap_link_stats, lstats.p, (size_t)B * links * 4 * sizeof(R), hipMemcpyDeviceToHost, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  if (p->timing) collect_timing(p);
  if (a->counts)
    for (size_t i = 0; i < hc.size(); ++i) a->counts[i] += hc[i];
  if (a->frame_crc_ok && coded)
    for (int b = 0; b < B; ++b) a->frame_crc_ok[b] = (uint8_t)crc[b];
  return LTE_OK;
}

extern "C" {

}  // extern "C"

// Beamforming chain (frequency domain, flat H per frame), R = double (the
// default) / float.  sig: the per-frame noise scale sqrt(10^(-SNR/10) / 2).
template <class R>
static int run_bf(lte_plan* p, const lte_run_args* a, int B, int n_snr, const std::vector<double>& sig,
                  const uint32_t* inj_bits, int64_t inj_bits_stride) {
  const lte_plan_desc& d = p->d;
  hipStream_t s = p->stream;
  ChainBufs<R>& c = cbuf<R>(p);
  BfFrameT<R>* frd = bf_frames<R>(p);
  const size_t links = (size_t)d.num_rx * d.num_tx;
  std::vector<R> sg(B);
  for (int b = 0; b < B; ++b) sg[b] = (R)sig[b];
  HIPCHK(hipMemcpyAsync(c.snr_lin.p, sg.data(), B * sizeof(R), hipMemcpyHostToDevice, s));
  const R *inj_h = nullptr, *inj_z = nullptr;
  int64_t inj_h_stride = 0, inj_z_stride = 0;
  if (a->link_h) {
    const int e = upload_inj<R>(c.inj_lh, a->link_h, a->link_h_stride, B, links * 2, s, &inj_h, &inj_h_stride);
    if (e != LTE_OK) return e;
  }
  if (a->noise) {
    const int e = upload_inj<R>(c.inj_z, a->noise, a->noise_stride, B, (size_t)d.num_rx * 2 * p->L, s, &inj_z,
                                &inj_z_stride);
    if (e != LTE_OK) return e;
  }
  {
    Timer t(p, KN_PAYLOAD);
    LCHK(launch_payload(s, p->pw.p, p->PW, d.n_bits, 0, p->fid.p, a->seed, B, inj_bits, inj_bits_stride));
  }
  cx<R>* cap_syms_dev = nullptr;
  uint8_t* cap_bits_dev = nullptr;
  if (a->cap_data_syms) {
    if (c.capbuf.alloc((size_t)B * p->L)) return fail(LTE_ENOMEM, "capture");
    cap_syms_dev = c.capbuf.p;
  }
  if (a->cap_bits_rx) {
    if (p->cap_bits.alloc((size_t)B * d.n_bits)) return fail(LTE_ENOMEM, "capture");
    cap_bits_dev = p->cap_bits.p;
  }
  {
    Timer t(p, KN_RX_DATA);
    LCHK(launch_bf<R>(s, B, p->n_sym, p->Nd, d.bps, d.num_tx, d.num_rx, d.bf_adaptive, p->bf_ncb, p->bf_cb.p,
                      p->fid.p, a->seed, inj_h, inj_h_stride, frd, c.snr_lin.p, p->pw.p, p->PW, d.n_bits, inj_z,
                      inj_z_stride, p->frame_err.p, cap_syms_dev, cap_bits_dev));
  }
  {
    Timer t(p, KN_ACC);
    LCHK(launch_accumulate(s, B, 0, d.n_bits, n_snr, p->snr_idx.p, p->frame_err.p, p->frame_crc.p, p->counts.p));
  }
  std::vector<unsigned long long> hc((size_t)4 * n_snr);
  HIPCHK(hipMemcpyAsync(hc.data(), p->counts.p, hc.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
  if (a->frame_errors)
    HIPCHK(hipMemcpyAsync(a->frame_errors, p->frame_err.p, B * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  if (a->cap_data_syms)
    HIPCHK(hipMemcpyAsync(a->cap_data_syms, cap_syms_dev, (size_t)B * p->L * sizeof(cx<R>), hipMemcpyDeviceToHost, s));
  if (a->cap_bits_rx)
    HIPCHK(hipMemcpyAsync(a->cap_bits_rx, cap_bits_dev, (size_t)B * d.n_bits, hipMemcpyDeviceToHost, s));
  std::vector<BfFrameT<R>> fr;
  if (a->cap_H || a->cap_pmi || a->cap_bf_gain) {
    fr.resize(B);
    HIPCHK(hipMemcpyAsync(fr.data(), frd, B * sizeof(BfFrameT<R>), hipMemcpyDeviceToHost, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  if (p->timing) collect_timing(p);
  for (int b = 0; b < (int)fr.size(); ++b) {
    if (a->cap_H)   // [n_frames][num_rx][num_tx] complex in the plan's type
      for (int r = 0; r < d.num_rx; ++r)
        for (int t = 0; t < d.num_tx; ++t) {
          R* o = static_cast<R*>(a->cap_H) + (((size_t)b * d.num_rx + r) * d.num_tx + t) * 2;
          o[0] = fr[b].H[r][t].x;
          o[1] = fr[b].H[r][t].y;
        }
    if (a->cap_pmi) a->cap_pmi[b] = fr[b].pmi;
    if (a->cap_bf_gain) a->cap_bf_gain[b] = fr[b].gain_db;
  }
  if (a->counts)
    for (size_t i = 0; i < hc.size(); ++i) a->counts[i] += hc[i];
  return LTE_OK;
}



// TX with the channel fused in (TxChannelT): SISO / SIMO Rayleigh (SC-FDM
// precoding included), delays within the CP, no TX / RX stream capture; static
// taps (fD = 0) or per-symbol Taylor sets while mimo_taylor_ok (3 km/h at
// 20 MHz: |w| S / 2 = 1.2e-3).
// LTE_TXCH_FUSE=0 selects the separate TX and channel kernels (A/B and
// parity tests).
static bool txch_fusable(const lte_plan* p, const lte_run_args* a, bool coded) {
  const lte_plan_desc& d = p->d;
  if (d.channel != LTE_CH_RAYLEIGH || d.num_rx < 1 || p->mimo || p->bf) return false;
  if (d.fD != 0.0 && !mimo_taylor_ok(d.fD, d.fs, d.N + d.cp_len)) return false;
  if (a->in_signal || a->cap_signal_tx || a->cap_signal_rx) return false;
  if (const char* e = std::getenv("LTE_TXCH_FUSE"))
    if (std::atoi(e) == 0) return false;
  return txch_supported(p->grid, d.n_paths, *std::max_element(d.delays, d.delays + d.n_paths));
}



// Coded TX + channel with one slot per frame (k_ofdm_txf) when its LDS fits
// (coded streams staged once per frame); LTE_TX_FRAME=0 keeps one slot per
// OFDM symbol (k_ofdm_tx<.., CH>, A/B and parity tests).
static bool tx_per_frame(const lte_plan* p) {
  if (const char* e = std::getenv("LTE_TX_FRAME"))
    if (std::atoi(e) == 0) return false;
  const int spw = 256 / (p->grid.N >> 3);
  const size_t el = p->f64 ? 16 : 8;
  return (size_t)spw * (p->grid.N * el + (size_t)p->enc_words * 4) <= 65536;
}

// Fading taps, fused TX + channel, first-samples power fix-up and noise power.
template <class R>
static int run_txch(lte_plan* p, hipStream_t s, const lte_run_args* a, int B, bool coded, const R* inj_ph,
                    int64_t inj_ph_stride, cx<R>* cap_tx_syms, cx<R>* x_out, TxChannelT<R>* ch_out) {
  const lte_plan_desc& d = p->d;
  ChainBufs<R>& c = cbuf<R>(p);
  const int maxd = *std::max_element(d.delays, d.delays + d.n_paths);
  if (c.xh.alloc((size_t)d.max_frames * p->n_sym * 2 * std::max(maxd, 1))) return fail(LTE_ENOMEM, "tx channel");
  const int rx = d.num_rx;
  const bool tv = d.fD != 0.0;   // time-varying taps: per-symbol Taylor sets
  if (tv && c.tcoef.alloc((size_t)d.max_frames * rx * d.n_paths * p->n_sym * mimo_ncf<R>()))
    return fail(LTE_ENOMEM, "tx channel");
  {
    Timer t(p, KN_FADING, s);
    LCHK(launch_fading<R>(s, B, rx, d.n_paths, c.gains.p, p->fid.p, a->seed, inj_ph, inj_ph_stride, c.phases.p,
                          c.coef.p));
    if (tv)   // one (frame, RX) at a time: phases / sets are [B][rx][path]
      LCHK(launch_jakes_sets<R>(s, B * rx, d.n_paths, p->n_sym, d.N + d.cp_len, c.phases.p, c.gains.p, d.fD, d.fs,
                                c.tcoef.p));
  }
  TxChannelT<R> ch{};
  ch.tcoef = tv ? c.tcoef.p : nullptr;
  ch.num_rx = rx;
  ch.n_paths = d.n_paths;
  ch.max_delay = maxd;
  for (int i = 0; i < d.n_paths; ++i) ch.delays[i] = d.delays[i];
  ch.coef = c.coef.p;
  ch.y = c.y.p;
  ch.xh = c.xh.p;
  ch.pow_part = c.pow_part.p;
  ch.x_out = x_out;
  if (ch_out) *ch_out = ch;
  {
    Timer t(p, KN_OFDM_TX, s);
    if (coded && tx_per_frame(p))
      LCHK(launch_ofdm_txf<R>(s, p->grid, p->enc.p, p->enc_words, p->tx_map.p, p->txf_map.p, p->txf_re.p, B,
                              cap_tx_syms, ch));
    else
      LCHK(launch_ofdm_tx_ch<R>(s, p->grid, coded ? 1 : 0, p->pw.p, p->PW, p->enc.p, p->enc_words, p->tx_map.p, B,
                                cap_tx_syms, ch, (d.sc_fdm && !coded) ? 1 : 0));
  }
  {
    Timer t(p, KN_CHANNEL, s);
    bool fix_fused = false;   // config 3's wave TX formed the head samples' power itself
    if constexpr (std::is_same_v<R, double>)
      fix_fused = !(coded && tx_per_frame(p)) && tx_simo_w_fuses_fix(p->grid, coded ? 1 : 0,
                                                                     (d.sc_fdm && !coded) ? 1 : 0, ch);
    if (!fix_fused) LCHK(launch_chan_fix<R>(s, p->grid, B, ch));
    LCHK(launch_npow<R>(s, B, rx, ch.pow_part, p->n_sym, p->L, c.snr_lin.p, c.npow.p));
  }
  return LTE_OK;
}

// Coded SISO 16/64-QAM without an LLR capture: k_rx_data hands over the
// equalised symbol and sigma^2_eff per RE and k_dematch_zn demaps while it
// builds the decoder rows, instead of a round trip of bps LLRs per RE.  The
// (z, nv) arrays live in the LLR buffer ([max_frames][n_re] z, then
// [max_frames][n_re] nv: 3 R per RE).  LTE_DEMAP_IN_DEMATCH=0 keeps the LLR path.
static bool demap_in_dematch(const lte_plan* p, const lte_run_args* a) {
  const lte_plan_desc& d = p->d;
  if (d.chain != LTE_CHAIN_CODED || p->mimo || p->bf || (d.bps != 4 && d.bps != 6) || a->cap_llr) return false;
  if (const char* e = std::getenv("LTE_DEMAP_IN_DEMATCH"))
    if (std::atoi(e) == 0) return false;
  return true;
}

// Fused SISO receiver (k_rx_frame): one RX, coded or uncoded, no SC-FDM.
// LTE_RX_FUSE=0 selects k_rx_chest + k_rx_data (A/B and parity tests).
static bool rx_fusable(const lte_plan* p, const lte_plan_desc& d) {
  if (const char* e = std::getenv("LTE_RX_FUSE"))
    if (std::atoi(e) == 0) return false;
  return rx_frame_supported(p->grid, d.chain, d.num_rx, (d.sc_fdm && d.chain == LTE_CHAIN_UNCODED) ? 1 : 0);
}
// Fused SIMO MRC receiver (k_rx_frame_simo), same switch.
static bool rx_simo_fusable(const lte_plan* p, const lte_plan_desc& d) {
  if (const char* e = std::getenv("LTE_RX_FUSE"))
    if (std::atoi(e) == 0) return false;
  return d.chain == LTE_CHAIN_SIMO && rx_frame_simo_supported(p->grid, d.num_rx);
}

// SISO / SIMO chains (uncoded, coded, MRC) in precision R.
template <class R>
static int run_siso(lte_plan* p, const lte_run_args* a, int B, int n_snr, const std::vector<double>& snr_lin,
                    const uint32_t* inj_bits, int64_t inj_bits_stride) {
  using V = cx<R>;
  const lte_plan_desc& d = p->d;
  ChainBufs<R>& c = cbuf<R>(p);
  const Grid& g = p->grid;
  const bool coded = d.chain == LTE_CHAIN_CODED, ray_cfg = d.channel == LTE_CH_RAYLEIGH;
  const int rx = d.num_rx;
  hipStream_t s = p->stream;
  const int stages = a->stages ? a->stages : LTE_STAGE_ALL;
  const bool do_tx = stages & LTE_STAGE_TX, do_ch = stages & LTE_STAGE_CHANNEL, do_rx = stages & LTE_STAGE_RX;
  // per-frame linear SNR (computed in float64 on the host, as 10 ** (snr_db / 10));
  // without the channel stage the input is the received signal: no noise
  std::vector<R> sl(B);
  for (int b = 0; b < B; ++b) sl[b] = do_ch ? (R)snr_lin[b] : (R)INFINITY;
  HIPCHK(hipMemcpyAsync(c.snr_lin.p, sl.data(), B * sizeof(R), hipMemcpyHostToDevice, s));
  const R* inj_ph = nullptr;
  int64_t inj_ph_stride = 0;
  if (a->phases && ray_cfg) {
    const int e = upload_inj<R>(c.inj_ph, a->phases, a->phases_stride, B, (size_t)rx * d.n_paths * 16, s, &inj_ph,
                                &inj_ph_stride);
    if (e != LTE_OK) return e;
  }
  const R* inj_z = nullptr;
  int64_t inj_z_stride = 0;
  if (a->noise) {
    const int e = upload_inj<R>(c.inj_z, a->noise, a->noise_stride, B, (size_t)rx * 2 * p->L, s, &inj_z,
                                &inj_z_stride);
    if (e != LTE_OK) return e;
  }
  // TX + static-tap channel in one kernel (the received stream is written once)
  const bool fuse = do_tx && do_ch && txch_fusable(p, a, coded);
  // SIMO into the paired receiver (config 3), opt-in (LTE_SIMO_XHAND=1): the
  // TX hands over its symbols and the receiver applies each RX's taps
  // (TxChannelT::x_out), one stream through HBM instead of num_rx.  Measured
  // slower (profiles/r6_simo_xhand_ab.md: TX 16.1 -> 12.9 ms, receiver 27.7 ->
  // 43.3 ms per 65 536 frames: the taps cost the VALU-bound receiver more than
  // the streams cost the HBM)
  const bool xhand = fuse && do_rx && d.fD == 0.0 && d.chain == LTE_CHAIN_SIMO &&
                     rx_simo_fusable(p, d) && rx_simo2_ok(g, rx, a->cap_H != nullptr, a->cap_pilot_stats != nullptr) &&
                     env_on("LTE_RXS_PAIRS", true) && env_on("LTE_SIMO_XHAND", false);
  TxChannelT<R> xch{};
  if (do_tx || a->bits) {
    Timer t(p, KN_PAYLOAD);
    LCHK(launch_payload(s, p->pw.p, p->PW, d.n_bits, coded ? CRC24A_POLY : 0, p->fid.p, a->seed, B, inj_bits, inj_bits_stride));
  }
  if ((!fuse || xhand) && c.x.alloc((size_t)d.max_frames * p->L)) return fail(LTE_ENOMEM, "TX signal buffer");
  if (do_tx) {
    if (coded) {
      Timer t(p, KN_ENCODE);
      LCHK(launch_encode(s, p->pw.p, p->PW, p->KWmax, p->enc.p, p->EW, p->cbi.p, p->C, B, p->enc_qmask.p, p->qstride));
    }
    V* cts = nullptr;
    if (a->cap_tx_syms) {
      if (c.captx.alloc((size_t)B * p->n_sym * p->Nd)) return fail(LTE_ENOMEM, "capture");
      cts = c.captx.p;
    }
    if (fuse) {
      const int e = run_txch<R>(p, s, a, B, coded, inj_ph, inj_ph_stride, cts, xhand ? c.x.p : nullptr, &xch);
      if (e != LTE_OK) return e;
    } else {
      Timer t(p, KN_OFDM_TX);
      // SC-FDM precodes the uncoded SISO / SIMO transmitters only: simulate_siso_coded
      // builds its own grids without the precoder (core/ofdm_core.py:1062-1099)
      LCHK(launch_ofdm_tx<R>(s, g, coded ? 1 : 0, p->pw.p, p->PW, p->enc.p, p->enc_words, p->tx_map.p, c.x.p, B, cts,
                             (d.sc_fdm && !coded) ? 1 : 0));
    }
  } else {
    const R* in = static_cast<const R*>(a->in_signal);
    std::vector<R> hx((size_t)B * p->L * 2);
    for (int b = 0; b < B; ++b)
      std::memcpy(&hx[(size_t)b * p->L * 2], in + (size_t)b * a->in_signal_stride, (size_t)p->L * 2 * sizeof(R));
    HIPCHK(hipMemcpyAsync(c.x.p, hx.data(), hx.size() * sizeof(R), hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
  }
  const bool ray = ray_cfg && do_ch;
  const V* ysrc = ray ? c.y.p : c.x.p;
  const int64_t yrs = ray ? p->L : 0, yfs = ray ? (int64_t)rx * p->L : p->L;
  if (ray && !fuse) {
    Timer t(p, KN_FADING);
    LCHK(launch_fading<R>(s, B, rx, d.n_paths, c.gains.p, p->fid.p, a->seed, inj_ph, inj_ph_stride, c.phases.p,
                          c.coef.p));
  }
  if (!fuse) {
    Timer t(p, KN_CHANNEL);
    LCHK(launch_channel<R>(s, g, B, rx, ray ? 1 : 0, d.n_paths, p->delays.p, c.gains.p, (R)d.fD, (R)d.fs,
                           c.phases.p, c.coef.p, c.x.p, c.y.p, c.pow_part.p, channel_nblk(p->L),
                           ray ? *std::max_element(d.delays, d.delays + d.n_paths) : 0));
    LCHK(launch_npow<R>(s, B, rx, c.pow_part.p, channel_nblk(p->L), p->L, c.snr_lin.p, c.npow.p));
  }
  // SISO receiver fused (estimation + data path per frame) unless LTE_RX_FUSE=0
  const bool rxf = do_rx && rx_fusable(p, d);
  const bool rxs = do_rx && !rxf && rx_simo_fusable(p, d);
  if (do_rx && !rxf && !rxs) {
    Timer t(p, KN_RX_CHEST);
    LCHK(launch_rx_chest<R>(s, g, B, rx, ysrc, yrs, yfs, c.npow.p, p->fid.p, a->seed, inj_z, inj_z_stride, c.H.p,
                            c.pstats.p));
  }
  V* cap_syms_dev = nullptr;
  uint8_t* cap_bits_dev = nullptr;
  if (a->cap_data_syms) {
    if (c.capbuf.alloc((size_t)B * p->n_sym * p->Nd)) return fail(LTE_ENOMEM, "capture");
    cap_syms_dev = c.capbuf.p;
  }
  if (a->cap_bits_rx) {
    if (p->cap_bits.alloc((size_t)B * d.n_bits)) return fail(LTE_ENOMEM, "capture");
    cap_bits_dev = p->cap_bits.p;
  }
  const bool zn = demap_in_dematch(p, a);
  if (coded && !zn && c.llr.alloc((size_t)d.max_frames * p->n_re_bits)) return fail(LTE_ENOMEM, "LLR buffer");
  if (rxf) {
    Timer t(p, KN_RX_DATA);
    LCHK(launch_rx_frame<R>(s, g, d.chain, ray ? 1 : 0, B, ysrc, yfs, c.npow.p, c.snr_lin.p, p->fid.p, a->seed, inj_z,
                            inj_z_stride, p->pw.p, p->PW, d.n_bits, p->frame_err.p,
                            zn ? reinterpret_cast<R*>(zn_z<R>(p)) : c.llr.p, cap_syms_dev,
                            coded ? nullptr : cap_bits_dev, zn ? zn_nv<R>(p) : nullptr,
                            a->cap_H ? c.H.p : nullptr, a->cap_pilot_stats ? c.pstats.p : nullptr));
  } else if (rxs) {
    Timer t(p, KN_RX_DATA);
    LCHK(launch_rx_frame_simo<R>(s, g, B, rx, ysrc, yrs, yfs, c.npow.p, p->fid.p, a->seed, inj_z, inj_z_stride,
                                 p->pw.p, p->PW, d.n_bits, p->frame_err.p, cap_syms_dev, cap_bits_dev,
                                 a->cap_H ? c.H.p : nullptr, a->cap_pilot_stats ? c.pstats.p : nullptr,
                                 xhand ? &xch : nullptr));
  } else if (do_rx) {
    Timer t(p, KN_RX_DATA);
    LCHK(launch_rx_data<R>(s, g, d.chain, ray ? 1 : 0, B, rx, ysrc, yrs, yfs, c.H.p, c.npow.p, c.snr_lin.p, p->fid.p,
                           a->seed, inj_z, inj_z_stride, p->pw.p, p->PW, d.n_bits, p->frame_err.p,
                           zn ? reinterpret_cast<R*>(zn_z<R>(p)) : c.llr.p, cap_syms_dev,
                           coded ? nullptr : cap_bits_dev,
                           // the IDFT runs in receive_and_decode only (core/lte_receiver.py:318-333): the SIMO
                           // MRC receiver (core/ofdm_core.py:1340-1534) never de-precodes
                           (d.sc_fdm && d.chain == LTE_CHAIN_UNCODED) ? 1 : 0, zn ? zn_nv<R>(p) : nullptr));
  }
  if (coded && do_rx) {
    {
      Timer t(p, KN_DEMATCH);
      if (zn)
        LCHK(launch_dematch_zn<R>(s, zn_z<R>(p), zn_nv<R>(p), p->n_re_bits / d.bps, p->Nd, d.bps, B, p->rx_map.p,
                                  p->n_layers, c.blk_ptrs.p, p->rows_dev.p, turbo_plan_ch(p)));
      else
        LCHK(launch_dematch<R>(s, c.llr.p, p->n_re_bits, B, p->rx_map.p, p->n_layers, c.blk_ptrs.p, p->rows_dev.p,
                                 turbo_plan_ch(p)));
    }
    const int G = (B + 63) / 64;
    std::vector<TurboJob> jobs(p->C);
    for (int r = 0; r < p->C; ++r) {
      const CbInfo& cb = p->cbs[r];
      jobs[r] = TurboJob{c.blk[r].p, c.ckpt[r].p, p->decb[r].p, cb.K, cb.f1, cb.f2, G, turbo_plan_ch(p)};
    }
    {
      Timer t(p, KN_TURBO);
      LCHK(launch_turbo_jobs(s, jobs.data(), p->C, d.turbo_iters, TM_DEC1, sizeof(R) == 8 ? 1 : 0));
    }
    {
      Timer t(p, KN_CRC);
      LCHK(launch_crc_count(s, p->cbi.p, p->C, p->dec_ptrs.p, p->kw_dev.p, B, p->pw.p, p->PW, d.n_bits,
                            p->frame_err.p, p->frame_crc.p, cap_bits_dev, 0, inj_bits ? nullptr : p->fid.p,
                            a->seed));
    }
  }
  if (do_rx) {
    Timer t(p, KN_ACC);
    LCHK(launch_accumulate(s, B, coded ? 1 : 0, d.n_bits, n_snr, p->snr_idx.p, p->frame_err.p, p->frame_crc.p,
                           p->counts.p));
  }
  // results
  std::vector<unsigned long long> hc((size_t)4 * n_snr);
  HIPCHK(hipMemcpyAsync(hc.data(), p->counts.p, hc.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
  if (a->frame_errors)
    HIPCHK(hipMemcpyAsync(a->frame_errors, p->frame_err.p, B * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  std::vector<uint32_t> crc;
  if (a->frame_crc_ok && coded) {
    crc.resize(B);
    HIPCHK(hipMemcpyAsync(crc.data(), p->frame_crc.p, B * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  }
  if (a->cap_signal_tx)
    HIPCHK(hipMemcpyAsync(a->cap_signal_tx, c.x.p, (size_t)B * p->L * sizeof(V), hipMemcpyDeviceToHost, s));
  if (a->cap_signal_rx) {
    DBuf<V> tmp;
    if (tmp.alloc((size_t)B * rx * p->L)) return fail(LTE_ENOMEM, "capture");
    {
      Timer t(p, KN_CAP);
      hipLaunchKernelGGL(k_cap_rx<R>, dim3(((p->L + 255) / 256) * B, rx), dim3(256), 0, s, p->L, rx, B, ysrc, yrs, yfs,
                         c.npow.p, p->fid.p, a->seed, inj_z, inj_z_stride, tmp.p);
      LCHK((int)hipGetLastError());
    }
    HIPCHK(hipMemcpyAsync(a->cap_signal_rx, tmp.p, (size_t)B * rx * p->L * sizeof(V), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    tmp.release();
  }
  if (a->cap_data_syms)
    HIPCHK(hipMemcpyAsync(a->cap_data_syms, cap_syms_dev, (size_t)B * p->n_sym * p->Nd * sizeof(V),
                          hipMemcpyDeviceToHost, s));
  if (a->cap_H)
    HIPCHK(hipMemcpyAsync(a->cap_H, c.H.p, (size_t)B * rx * p->n_grp * d.N * sizeof(V), hipMemcpyDeviceToHost, s));
  if (a->cap_pilot_stats)
    HIPCHK(hipMemcpyAsync(a->cap_pilot_stats, c.pstats.p, (size_t)B * rx * p->n_grp * 2 * sizeof(R),
                          hipMemcpyDeviceToHost, s));
  if (a->cap_bits_rx)
    HIPCHK(hipMemcpyAsync(a->cap_bits_rx, cap_bits_dev, (size_t)B * d.n_bits, hipMemcpyDeviceToHost, s));
  if (a->cap_llr && coded)
    HIPCHK(hipMemcpyAsync(a->cap_llr, c.llr.p, (size_t)B * p->n_re_bits * sizeof(R), hipMemcpyDeviceToHost, s));
  if (a->cap_tx_syms && do_tx)
    HIPCHK(hipMemcpyAsync(a->cap_tx_syms, c.captx.p, (size_t)B * p->n_sym * p->Nd * sizeof(V), hipMemcpyDeviceToHost,
                          s));
  if (a->cap_noise_power)
    HIPCHK(hipMemcpyAsync(a->cap_noise_power, c.npow.p, (size_t)B * rx * sizeof(R), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (p->timing) collect_timing(p);
  if (a->counts)
    for (size_t i = 0; i < hc.size(); ++i) a->counts[i] += hc[i];
  if (a->frame_crc_ok && coded)
    for (int b = 0; b < B; ++b) a->frame_crc_ok[b] = (uint8_t)crc[b];
  return LTE_OK;
}

extern "C" {

int lte_run(lte_plan* p, const lte_run_args* a) {
  if (!p || !a) return fail(LTE_EINVAL, "null argument");
  const lte_plan_desc& d = p->d;
  const int B = a->n_frames;
  if (B < 1 || B > d.max_frames) return fail(LTE_EINVAL, "n_frames out of range (1..max_frames)");
  if (!a->snr_db) return fail(LTE_EINVAL, "snr_db required");
  const int n_snr = std::max(1, a->n_snr);
  hipStream_t s = p->stream;
  if (p->counts.alloc((size_t)4 * n_snr)) return fail(LTE_ENOMEM, "counts");
  // per-frame parameters
  std::vector<double> sl(B);
  std::vector<int32_t> si(B, 0);
  std::vector<uint64_t> fid(B);
  for (int b = 0; b < B; ++b) {
    sl[b] = std::pow(10.0, a->snr_db[b] / 10.0);   // snr_linear = 10 ** (snr_db / 10) (channel.py:32), float64
    if (a->snr_index) {
      si[b] = a->snr_index[b];
      if (si[b] < 0 || si[b] >= n_snr) return fail(LTE_EINVAL, "snr_index out of range");
    }
    fid[b] = a->frame_ids ? a->frame_ids[b] : a->frame_id0 + (uint64_t)b;
  }
  HIPCHK(hipMemcpyAsync(p->snr_idx.p, si.data(), B * sizeof(int32_t), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(p->fid.p, fid.data(), B * sizeof(uint64_t), hipMemcpyHostToDevice, s));
  // payload injection (packed MSB-first)
  const uint32_t* inj_bits = nullptr;
  int64_t inj_bits_stride = 0;
  if (a->bits) {   // one uint8 per bit from the caller, packed MSB-first on the device
    const int nf = a->bits_stride ? B : 1;
    const int nwd = (d.n_bits + 31) / 32;
    const size_t nb = a->bits_stride ? (size_t)(nf - 1) * a->bits_stride + d.n_bits : (size_t)d.n_bits;
    if (p->inj_bytes.alloc(nb) || p->inj_bits.alloc((size_t)nf * nwd)) return fail(LTE_ENOMEM, "inj bits");
    HIPCHK(hipMemcpyAsync(p->inj_bytes.p, a->bits, nb, hipMemcpyHostToDevice, s));
    LCHK(launch_pack_bits(s, p->inj_bytes.p, a->bits_stride, d.n_bits, nwd, nf, p->inj_bits.p));
    inj_bits = p->inj_bits.p;
    inj_bits_stride = a->bits_stride ? nwd : 0;
  }
  HIPCHK(hipMemsetAsync(p->counts.p, 0, 4 * n_snr * sizeof(unsigned long long), s));
  HIPCHK(hipMemsetAsync(p->frame_err.p, 0, B * sizeof(uint32_t), s));
  const int stages = a->stages ? a->stages : LTE_STAGE_ALL;
  if (!(stages & LTE_STAGE_TX) && !a->in_signal) return fail(LTE_EINVAL, "in_signal required when the TX stage is skipped");
  p->evuse.clear();
  if (logmap_on() && (d.chain == LTE_CHAIN_CODED || d.chain == LTE_CHAIN_SFBC_CODED) && !p->f64)
    return fail(LTE_EUNSUP, "exact log-MAP decoding runs in float64 plans only");
  if (!p->mimo && !p->bf) {
    const int e = p->f64 ? run_siso<double>(p, a, B, n_snr, sl, inj_bits, inj_bits_stride)
                         : run_siso<float>(p, a, B, n_snr, sl, inj_bits, inj_bits_stride);
    HIPCHK(hipStreamSynchronize(s));
    return e;
  }
  if (stages != LTE_STAGE_ALL) return fail(LTE_EUNSUP, "multi-antenna chains run all stages");
  if (p->mimo)
    return p->f64 ? run_mimo<double>(p, a, B, n_snr, sl, inj_bits, inj_bits_stride)
                  : run_mimo<float>(p, a, B, n_snr, sl, inj_bits, inj_bits_stride);
  // beamforming chain: noise scale sqrt(noise_variance / 2), noise_variance =
  // 10 ** (-snr_db / 10) (core/ofdm_core.py:2397-2399)
  std::vector<double> sig(B);
  for (int b = 0; b < B; ++b) sig[b] = std::sqrt(std::pow(10.0, -a->snr_db[b] / 10.0) / 2.0);
  return p->f64 ? run_bf<double>(p, a, B, n_snr, sig, inj_bits, inj_bits_stride)
                : run_bf<float>(p, a, B, n_snr, sig, inj_bits, inj_bits_stride);
}

// ------------------------------------------------------------------ stage entry points
}  // extern "C"

// Stage entry points (host in / out, the chains' device kernels), R = float / double.
template <class R>
static int stage_grid(int N, TableSet& t, Grid& g) {
  g = Grid{};
  g.N = N;
  g.log2N = ilog2(N);
  if (sizeof(R) == 8) {
    if (upload(t.tw64, make_twiddles64(N))) return -1;
    g.tw64 = t.tw64.p;
  } else {
    if (upload(t.tw, make_twiddles(N))) return -1;
    g.tw = t.tw.p;
  }
  return 0;
}

template <class R>
static int fft_host(int N, int inverse, int64_t batch, const R* in, R* out) {
  if (N < 8 || N > 2048 || (N & (N - 1)) || batch < 0 || (!in && batch) || (!out && batch))
    return fail(LTE_EINVAL, "bad fft arguments");
  if (batch == 0) return LTE_OK;
  if (N < 64) return fail(LTE_EUNSUP, "N < 64");
  TableSet t;
  Grid g;
  if (stage_grid<R>(N, t, g)) return fail(LTE_ENOMEM, "tables");
  DBuf<cx<R>> di, dout;
  if (di.alloc(batch * N) || dout.alloc(batch * N)) { t.release(); return fail(LTE_ENOMEM, "fft buffers"); }
  int rc = LTE_OK;
  if (hipMemcpy(di.p, in, batch * N * sizeof(cx<R>), hipMemcpyHostToDevice) != hipSuccess ||
      launch_fft<R>(nullptr, g, inverse, batch, di.p, dout.p) != 0 || hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(out, dout.p, batch * N * sizeof(cx<R>), hipMemcpyDeviceToHost) != hipSuccess)
    rc = fail(LTE_EHIP, "fft failed");
  di.release(); dout.release(); t.release();
  return rc;
}

template <class R>
static int dft_host(int M, int inverse, int64_t batch, const R* in, R* out) {
  if (M < 1 || M > 1024 || batch < 0 || (!in && batch) || (!out && batch)) return fail(LTE_EINVAL, "bad dft arguments");
  if (batch == 0) return LTE_OK;
  int N = 64;
  while (N < 2 * M - 1) N <<= 1;
  TableSet t;
  Grid g;
  bool bad = stage_grid<R>(N, t, g) != 0;
  if (!bad && sizeof(R) == 8) {
    std::vector<double2> ch, bh;
    make_bluestein64(N, M, ch, bh);
    bad = upload(t.chirp64, ch) || upload(t.bhat64, bh);
    g.chirp64 = t.chirp64.p;
    g.bhat64 = t.bhat64.p;
  } else if (!bad) {
    std::vector<float2> ch, bh;
    make_bluestein(N, M, ch, bh);
    bad = upload(t.chirp, ch) || upload(t.bhat, bh);
    g.chirp = t.chirp.p;
    g.bhat = t.bhat.p;
  }
  if (bad) { t.release(); return fail(LTE_ENOMEM, "tables"); }
  g.Nd = M;
  DBuf<cx<R>> di, dout;
  if (di.alloc(batch * M) || dout.alloc(batch * M)) { t.release(); return fail(LTE_ENOMEM, "dft buffers"); }
  int rc = LTE_OK;
  if (hipMemcpy(di.p, in, batch * M * sizeof(cx<R>), hipMemcpyHostToDevice) != hipSuccess ||
      launch_dft<R>(nullptr, g, inverse, batch, di.p, dout.p) != 0 || hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(out, dout.p, batch * M * sizeof(cx<R>), hipMemcpyDeviceToHost) != hipSuccess)
    rc = fail(LTE_EHIP, "dft failed");
  di.release(); dout.release(); t.release();
  return rc;
}

template <class R>
static int llr_host(int bps, int64_t n, const R* syms, const R* nv, R* llr) {
  if ((bps != 2 && bps != 4 && bps != 6) || n < 0) return fail(LTE_EINVAL, "bad llr arguments");
  if (n == 0) return LTE_OK;
  DBuf<cx<R>> ds;
  DBuf<R> dn, dl;
  if (ds.alloc(n) || dn.alloc(n) || dl.alloc(n * bps)) return fail(LTE_ENOMEM, "llr buffers");
  int rc = LTE_OK;
  if (hipMemcpy(ds.p, syms, n * sizeof(cx<R>), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(dn.p, nv, n * sizeof(R), hipMemcpyHostToDevice) != hipSuccess ||
      launch_llr<R>(nullptr, bps, n, ds.p, dn.p, dl.p) ||
      hipMemcpy(llr, dl.p, n * bps * sizeof(R), hipMemcpyDeviceToHost) != hipSuccess)
    rc = fail(LTE_EHIP, "llr failed");
  ds.release(); dn.release(); dl.release();
  return rc;
}

template <class R>
static int hard_host(int bps, int64_t n, const R* syms, uint8_t* bits) {
  if ((bps != 2 && bps != 4 && bps != 6) || n < 0) return fail(LTE_EINVAL, "bad hard arguments");
  if (n == 0) return LTE_OK;
  DBuf<cx<R>> ds;
  DBuf<uint8_t> db;
  if (ds.alloc(n) || db.alloc(n * bps)) return fail(LTE_ENOMEM, "buffers");
  int rc = LTE_OK;
  if (hipMemcpy(ds.p, syms, n * sizeof(cx<R>), hipMemcpyHostToDevice) != hipSuccess ||
      launch_hard<R>(nullptr, bps, n, ds.p, db.p) ||
      hipMemcpy(bits, db.p, n * bps, hipMemcpyDeviceToHost) != hipSuccess)
    rc = fail(LTE_EHIP, "hard failed");
  ds.release(); db.release();
  return rc;
}

// QAMModulator.bits_to_symbols (core/modulator.py:61-88) on n whole symbols
static int qam_map_host(int bps, int64_t n, const uint8_t* bits, double* out) {
  if ((bps != 2 && bps != 4 && bps != 6) || n < 0 || (n && (!bits || !out)))
    return fail(LTE_EINVAL, "bad qam map arguments");
  if (n == 0) return LTE_OK;
  DBuf<uint8_t> db;
  DBuf<double2> dout;
  if (db.alloc((size_t)n * bps) || dout.alloc(n)) return fail(LTE_ENOMEM, "qam map buffers");
  int rc = LTE_OK;
  if (hipMemcpy(db.p, bits, (size_t)n * bps, hipMemcpyHostToDevice) != hipSuccess ||
      launch_qam_map(nullptr, bps, n, db.p, dout.p) || hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(out, dout.p, (size_t)n * 16, hipMemcpyDeviceToHost) != hipSuccess)
    rc = fail(LTE_EHIP, "qam map failed");
  db.release(); dout.release();
  return rc;
}

// QAMModulator.symbols_to_bits (core/modulator.py:90-112), the reference's
// own distance and argmin
static int hard_argmin_host(int bps, int64_t n, const double* syms, uint8_t* bits) {
  if ((bps != 2 && bps != 4 && bps != 6) || n < 0 || (n && (!syms || !bits)))
    return fail(LTE_EINVAL, "bad decision arguments");
  if (n == 0) return LTE_OK;
  DBuf<double2> ds;
  DBuf<uint8_t> db;
  if (ds.alloc(n) || db.alloc((size_t)n * bps)) return fail(LTE_ENOMEM, "decision buffers");
  const bool ok = hipMemcpy(ds.p, syms, (size_t)n * 16, hipMemcpyHostToDevice) == hipSuccess &&
                  launch_hard_argmin(nullptr, bps, n, ds.p, db.p) == 0 && hipDeviceSynchronize() == hipSuccess &&
                  hipMemcpy(bits, db.p, (size_t)n * bps, hipMemcpyDeviceToHost) == hipSuccess;
  ds.release(); db.release();
  return ok ? LTE_OK : fail(LTE_EHIP, "decisions failed");
}

// LTEChannelEstimator.estimate_channel + _interpolate_channel
// (core/lte_receiver.py:40-133) on batch received grids of N subcarriers
static int chest_host(int N, int P, const int32_t* pidx, const double* known, int64_t batch, const double* Y,
                      double* H, double* hp, double* stats) {
  if (N < 1 || P < 1 || P > 4096 || batch < 0 || !pidx || !known || (batch && (!Y || !H)))
    return fail(LTE_EINVAL, "bad channel estimation arguments");
  for (int p = 0; p < P; ++p)
    if (pidx[p] < 0 || pidx[p] >= N || (p && pidx[p] <= pidx[p - 1]))
      return fail(LTE_EINVAL, "pilot indices must be ascending and inside [0, N)");
  if (batch == 0) return LTE_OK;
  DBuf<int32_t> dp;
  DBuf<double2> dk, dy, dh, dhp;
  DBuf<double> dst;
  const size_t ny = (size_t)batch * N;
  if (dp.alloc(P) || dk.alloc(P) || dy.alloc(ny) || dh.alloc(ny) || (hp && dhp.alloc((size_t)batch * P)) ||
      (stats && dst.alloc((size_t)batch * 2)))
    return fail(LTE_ENOMEM, "channel estimation buffers");
  bool ok = hipMemcpy(dp.p, pidx, (size_t)P * 4, hipMemcpyHostToDevice) == hipSuccess &&
            hipMemcpy(dk.p, known, (size_t)P * 16, hipMemcpyHostToDevice) == hipSuccess &&
            hipMemcpy(dy.p, Y, ny * 16, hipMemcpyHostToDevice) == hipSuccess &&
            launch_chest(nullptr, N, P, dp.p, dk.p, batch, dy.p, dh.p, hp ? dhp.p : nullptr,
                         stats ? dst.p : nullptr) == 0 &&
            hipDeviceSynchronize() == hipSuccess && hipMemcpy(H, dh.p, ny * 16, hipMemcpyDeviceToHost) == hipSuccess;
  if (ok && hp) ok = hipMemcpy(hp, dhp.p, (size_t)batch * P * 16, hipMemcpyDeviceToHost) == hipSuccess;
  if (ok && stats) ok = hipMemcpy(stats, dst.p, (size_t)batch * 2 * 8, hipMemcpyDeviceToHost) == hipSuccess;
  dp.release(); dk.release(); dy.release(); dh.release(); dhp.release(); dst.release();
  return ok ? LTE_OK : fail(LTE_EHIP, "channel estimation failed");
}

// LTEEqualizerZF.equalize (core/lte_receiver.py:154-180): Y / (H + reg)
static int zf_host(int64_t n, const double* Y, const double* H, double reg, double* out) {
  if (n < 0 || (n && (!Y || !H || !out))) return fail(LTE_EINVAL, "bad equalizer arguments");
  if (n == 0) return LTE_OK;
  DBuf<double2> dy, dh, dout;
  if (dy.alloc(n) || dh.alloc(n) || dout.alloc(n)) return fail(LTE_ENOMEM, "equalizer buffers");
  const bool ok = hipMemcpy(dy.p, Y, (size_t)n * 16, hipMemcpyHostToDevice) == hipSuccess &&
                  hipMemcpy(dh.p, H, (size_t)n * 16, hipMemcpyHostToDevice) == hipSuccess &&
                  launch_zf(nullptr, n, dy.p, dh.p, reg, dout.p) == 0 && hipDeviceSynchronize() == hipSuccess &&
                  hipMemcpy(out, dout.p, (size_t)n * 16, hipMemcpyDeviceToHost) == hipSuccess;
  dy.release(); dh.release(); dout.release();
  return ok ? LTE_OK : fail(LTE_EHIP, "equalizer failed");
}

extern "C" {

int lte_qam_map_host64(int bps, int64_t n, const uint8_t* bits, double* out) {
  return qam_map_host(bps, n, bits, out);
}
int lte_nearest_host64(int bps, int64_t n, const double* syms, uint8_t* bits) {
  return hard_argmin_host(bps, n, syms, bits);
}
int lte_chest_host64(int N, int n_pilots, const int32_t* pilot_idx, const double* known, int64_t batch,
                     const double* Y, double* H, double* pilot_ls, double* stats) {
  return chest_host(N, n_pilots, pilot_idx, known, batch, Y, H, pilot_ls, stats);
}
int lte_zf_host64(int64_t n, const double* Y, const double* H, double regularization, double* out) {
  return zf_host(n, Y, H, regularization, out);
}
int lte_rsc_encode_host(int64_t n, const uint8_t* bits, int termination, uint8_t* systematic, uint8_t* parity) {
  if (n < 0 || (n && !bits) || !systematic || !parity) return fail(LTE_EINVAL, "bad rsc arguments");
  const int64_t m = n + (termination ? 3 : 0);
  if (m == 0) return LTE_OK;
  DBuf<uint8_t> du, ds, dp;
  if (du.alloc(n ? n : 1) || ds.alloc(m) || dp.alloc(m)) return fail(LTE_ENOMEM, "rsc buffers");
  const bool ok = (n == 0 || hipMemcpy(du.p, bits, n, hipMemcpyHostToDevice) == hipSuccess) &&
                  launch_rsc(nullptr, n, du.p, termination ? 1 : 0, ds.p, dp.p) == 0 &&
                  hipMemcpy(systematic, ds.p, m, hipMemcpyDeviceToHost) == hipSuccess &&
                  hipMemcpy(parity, dp.p, m, hipMemcpyDeviceToHost) == hipSuccess;
  du.release(); ds.release(); dp.release();
  return ok ? LTE_OK : fail(LTE_EHIP, "rsc failed");
}

int lte_fft_host(int N, int inverse, int64_t batch, const float* in, float* out) {
  return fft_host<float>(N, inverse, batch, in, out);
}
int lte_fft_host64(int N, int inverse, int64_t batch, const double* in, double* out) {
  return fft_host<double>(N, inverse, batch, in, out);
}
int lte_dft_host(int M, int inverse, int64_t batch, const float* in, float* out) {
  return dft_host<float>(M, inverse, batch, in, out);
}
int lte_dft_host64(int M, int inverse, int64_t batch, const double* in, double* out) {
  return dft_host<double>(M, inverse, batch, in, out);
}
int lte_llr_host(int bps, int64_t n, const float* syms, const float* nv, float* llr) {
  return llr_host<float>(bps, n, syms, nv, llr);
}
int lte_llr_host64(int bps, int64_t n, const double* syms, const double* nv, double* llr) {
  return llr_host<double>(bps, n, syms, nv, llr);
}
int lte_hard_host(int bps, int64_t n, const float* syms, uint8_t* bits) { return hard_host<float>(bps, n, syms, bits); }
int lte_hard_host64(int bps, int64_t n, const double* syms, uint8_t* bits) {
  return hard_host<double>(bps, n, syms, bits);
}

int lte_crc_host(int64_t n, const uint8_t* bits, uint32_t poly, int len, uint32_t* crc) {
  if (n < 0 || !crc || (n && !bits)) return fail(LTE_EINVAL, "bad crc arguments");
  if ((poly != 0x1864CFBu && poly != 0x1800063u) || len != 24) {
    // any other CRC (CRC-16 0x11021, crc.py:187-209): the serial device kernel
    if (len < 1 || len > 31 || (poly >> len) != 1u)
      return fail(LTE_EUNSUP, "CRC length 1..31 with the x^len term in poly");
    DBuf<uint8_t> db;
    DBuf<uint32_t> dout;
    if (db.alloc(n ? n : 1) || dout.alloc(1)) return fail(LTE_ENOMEM, "buffers");
    const bool ok = (n == 0 || hipMemcpy(db.p, bits, n, hipMemcpyHostToDevice) == hipSuccess) &&
                    launch_crc_serial(nullptr, n, db.p, poly & ((1u << len) - 1u), len, dout.p) == 0 &&
                    hipMemcpy(crc, dout.p, 4, hipMemcpyDeviceToHost) == hipSuccess;
    db.release(); dout.release();
    return ok ? LTE_OK : fail(LTE_EHIP, "crc failed");
  }
  const int nw = (int)((n + 24 + 31) / 32) + 1;
  std::vector<uint32_t> w(nw, 0);
  pack_bits(bits, (int)n, w.data(), nw);
  DBuf<uint32_t> dpw, dinj;
  DBuf<uint64_t> dfid;
  if (dpw.alloc(nw) || dinj.alloc(nw) || dfid.alloc(1)) return fail(LTE_ENOMEM, "buffers");
  int rc = LTE_OK;
  std::vector<uint32_t> o(nw);
  if (hipMemcpy(dinj.p, w.data(), nw * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(dfid.p, 0, 8) != hipSuccess ||
      launch_payload(nullptr, dpw.p, nw, (int)n, (int)(poly & 0xFFFFFFu), dfid.p, 0, 1, dinj.p, 0) ||
      hipMemcpy(o.data(), dpw.p, nw * 4, hipMemcpyDeviceToHost) != hipSuccess)
    rc = fail(LTE_EHIP, "crc failed");
  if (rc == LTE_OK) {
    uint32_t v = 0;
    for (int t = 0; t < 24; ++t) {
      const int64_t q = n + t;
      v = (v << 1) | ((o[q >> 5] >> (31 - (q & 31))) & 1u);
    }
    *crc = v;
  }
  dpw.release(); dinj.release(); dfid.release();
  return rc;
}

int lte_turbo_encode_host(int K, int64_t ncb, const uint8_t* bits, uint8_t* out) {
  int f1, f2;
  if (!qpp_lookup(K, &f1, &f2)) return fail(LTE_EINVAL, "Invalid code block size K=" + std::to_string(K));
  if (ncb < 0 || (ncb && (!bits || !out))) return fail(LTE_EINVAL, "bad arguments");
  if (ncb == 0) return LTE_OK;
  const int PW = (K + 31) / 32 + 1, KW = PW, EW = (K + 6 + 31) / 32;
  std::vector<uint32_t> w((size_t)ncb * PW);
  for (int64_t c = 0; c < ncb; ++c) pack_bits(bits + c * K, K, &w[c * PW], PW);
  CbInfo ci{K, 0, K, 0, 0, f1, f2, 3 * K + 12};
  DBuf<uint32_t> dpw, denc;
  DBuf<CbInfo> dci;
  DBuf<uint16_t> dqm;
  std::vector<CbInfo> vci{ci};
  std::vector<uint16_t> qm(K + 32);
  encode_qmask(&ci, 1, K + 32, qm.data());
  if (dpw.alloc(w.size()) || denc.alloc((size_t)ncb * 3 * EW) || upload(dci, vci) || upload(dqm, qm)) {
    dpw.release(); denc.release(); dci.release(); dqm.release();
    return fail(LTE_ENOMEM, "buffers");
  }
  std::vector<uint32_t> e((size_t)ncb * 3 * EW);
  int rc = LTE_OK;
  if (hipMemcpy(dpw.p, w.data(), w.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      launch_encode(nullptr, dpw.p, PW, KW, denc.p, EW, dci.p, 1, (int)ncb, dqm.p, K + 32) ||
      hipMemcpy(e.data(), denc.p, e.size() * 4, hipMemcpyDeviceToHost) != hipSuccess)
    rc = fail(LTE_EHIP, "encode failed");
  if (rc == LTE_OK) {
    for (int64_t c = 0; c < ncb; ++c) {
      const uint32_t* d0 = &e[c * 3 * EW];
      const uint32_t* d1 = d0 + EW;
      const uint32_t* d2 = d1 + EW;
      auto gb = [](const uint32_t* w, int i) -> uint8_t { return (w[i >> 5] >> (31 - (i & 31))) & 1u; };
      uint8_t* o = out + c * (3 * K + 12);
      for (int k = 0; k < K; ++k) { o[3 * k] = gb(d0, k); o[3 * k + 1] = gb(d1, k); o[3 * k + 2] = gb(d2, k); }
      for (int t = 0; t < 3; ++t) {
        o[3 * K + t] = gb(d0, K + t);
        o[3 * K + 3 + t] = gb(d1, K + t);
        o[3 * K + 6 + t] = gb(d0, K + 3 + t);
        o[3 * K + 9 + t] = gb(d2, K + t);
      }
    }
  }
  dpw.release(); denc.release(); dci.release(); dqm.release();
  return rc;
}

}  // extern "C"

// Host-side layout conversion [ncb][3K+12] -> decoder rows, shared by the
// turbo entry points.  T = float (fast mode) / double (the reference's precision).
template <class T>
static int turbo_host_run(int K, int iters, int64_t ncb, const T* llr, const T* ls, const T* lp, const T* la,
                          int mode, uint8_t* bits, T* app) {
  int f1, f2;
  if (!qpp_lookup(K, &f1, &f2)) return fail(LTE_EINVAL, "Invalid interleaver size K=" + std::to_string(K));
  if (ncb < 0) return fail(LTE_EINVAL, "bad ncb");
  if (ncb == 0) return LTE_OK;
  const int f64 = sizeof(T) == 8;
  const int G = (int)((ncb + 63) / 64);
  const int ch = turbo_chunk(G);   // fewer than TURBO_CH groups: contiguous blocks, no padding
  const int64_t rows = turbo_rows(K);
  std::vector<T> h((size_t)turbo_galloc(G) * rows * 64, (T)0);
  auto at = [&](int64_t c, int64_t row) -> T& { return h[turbo_elem_ch(ch, rows, c / 64, row) + (c % 64)]; };
  // decoder rows hold LLR/2 (exact; lte_decoder.hip gam)
  auto put = [&](int64_t c, int64_t row, T v) { at(c, row) = (T)0.5 * v; };
  for (int64_t c = 0; c < ncb; ++c) {
    if (mode == TM_APP) {
      const T* s = ls + c * (K + 3);
      const T* q = lp + c * (K + 3);
      const T* A = la + c * (K + 3);
      for (int k = 0; k < K + 3; ++k) { put(c, trow_ls(K, k), s[k]); put(c, trow_lp(K, 1, k), q[k]); }
      for (int k = 0; k < K; ++k) put(c, trow_le(K, k), A[k]);
    } else {
      const T* l = llr + c * (3 * K + 12);
      for (int k = 0; k < K; ++k) {
        put(c, trow_ls(K, k), l[3 * k]);
        put(c, trow_lp(K, 1, k), l[3 * k + 1]);
        put(c, trow_lp(K, 2, k), l[3 * k + 2]);
      }
      for (int t = 0; t < 3; ++t) {
        put(c, trow_ls(K, K + t), l[3 * K + t]);
        put(c, trow_lp(K, 1, K + t), l[3 * K + 3 + t]);
        put(c, trow_ls2t(K, t), l[3 * K + 6 + t]);
        put(c, trow_lp(K, 2, K + t), l[3 * K + 9 + t]);
      }
    }
  }
  DBuf<T> db, dck;
  DBuf<uint32_t> dbits;
  const int KW = turbo_kw(K);
  if (db.alloc(h.size()) || dck.alloc((size_t)turbo_galloc(G) * turbo_nwin(K) * turbo_ck_rows(f64) * 64) ||
      dbits.alloc((size_t)G * KW * 64))
    return fail(LTE_ENOMEM, "turbo buffers");
  int rc = LTE_OK;
  std::vector<uint32_t> hb((size_t)G * KW * 64);
  if (hipMemcpy(db.p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess ||
      launch_turbo(nullptr, db.p, dck.p, dbits.p, K, f1, f2, iters, G, mode, f64, ch) ||
      hipDeviceSynchronize() != hipSuccess)
    rc = fail(LTE_EHIP, std::string("turbo failed: ") + hipGetErrorString(hipGetLastError()));
  if (rc == LTE_OK) {
    if (mode == TM_APP) {
      if (hipMemcpy(h.data(), db.p, h.size() * sizeof(T), hipMemcpyDeviceToHost) != hipSuccess)
        rc = fail(LTE_EHIP, "copy");
      for (int64_t c = 0; c < ncb && rc == LTE_OK; ++c)
        for (int k = 0; k < K; ++k) app[c * K + k] = at(c, trow_le(K, k));
    } else {
      if (hipMemcpy(hb.data(), dbits.p, hb.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) rc = fail(LTE_EHIP, "copy");
      for (int64_t c = 0; c < ncb && rc == LTE_OK; ++c)
        for (int k = 0; k < K; ++k) {
          const uint32_t w = hb[((c / 64) * KW + (k >> 5)) * 64 + (c % 64)];
          bits[c * K + k] = (w >> (31 - (k & 31))) & 1u;
        }
    }
  }
  db.release(); dck.release(); dbits.release();
  return rc;
}

extern "C" {

int lte_turbo_decode_host(int K, int iters, int64_t ncb, const float* llr, uint8_t* bits) {
  if (iters < 0 || (ncb > 0 && (!llr || !bits))) return fail(LTE_EINVAL, "bad arguments");
  if (logmap_on()) return fail(LTE_EUNSUP, "exact log-MAP runs in float64 only (the f32 decoder is max-log)");
  return turbo_host_run<float>(K, iters, ncb, llr, nullptr, nullptr, nullptr, TM_DEC1, bits, nullptr);
}

int lte_turbo_decode_host64(int K, int iters, int64_t ncb, const double* llr, uint8_t* bits) {
  if (iters < 0 || (ncb > 0 && (!llr || !bits))) return fail(LTE_EINVAL, "bad arguments");
  return turbo_host_run<double>(K, iters, ncb, llr, nullptr, nullptr, nullptr, TM_DEC1, bits, nullptr);
}

int lte_bcjr_host(int K, int64_t ncb, const float* ls, const float* lp, const float* la, float* app) {
  if (ncb > 0 && (!ls || !lp || !la || !app)) return fail(LTE_EINVAL, "bad arguments");
  if (logmap_on()) return fail(LTE_EUNSUP, "exact log-MAP runs in float64 only (the f32 decoder is max-log)");
  return turbo_host_run<float>(K, 0, ncb, nullptr, ls, lp, la, TM_APP, nullptr, app);
}

int lte_bcjr_host64(int n, int64_t ncb, const double* ls, const double* lp, const double* la, double* app) {
  if (n < 0 || ncb < 0 || (n > 0 && ncb > 0 && (!ls || !lp || !la || !app))) return fail(LTE_EINVAL, "bad arguments");
  if (ncb == 0 || n == 0) return LTE_OK;   // K = 0: empty decisions and LLRs, like the reference
  const size_t sz = (size_t)ncb * n;
  DBuf<double> dls, dlp, dla, dal, dapp;
  if (dls.alloc(sz) || dlp.alloc(sz) || dla.alloc(sz) || dal.alloc(sz * 8) || dapp.alloc(sz))
    return fail(LTE_ENOMEM, "bcjr buffers");
  int rc = LTE_OK;
  if (hipMemcpy(dls.p, ls, sz * 8, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(dlp.p, lp, sz * 8, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(dla.p, la, sz * 8, hipMemcpyHostToDevice) != hipSuccess ||
      launch_bcjr64(nullptr, dls.p, dlp.p, dla.p, n, (int)ncb, dal.p, dapp.p) ||
      hipDeviceSynchronize() != hipSuccess || hipMemcpy(app, dapp.p, sz * 8, hipMemcpyDeviceToHost) != hipSuccess)
    rc = fail(LTE_EHIP, std::string("bcjr failed: ") + hipGetErrorString(hipGetLastError()));
  dls.release(); dlp.release(); dla.release(); dal.release(); dapp.release();
  return rc;
}

}  // extern "C"
