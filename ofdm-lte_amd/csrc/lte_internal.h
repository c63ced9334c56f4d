// Internal (non-ABI) declarations shared by the kernel TUs and the C-ABI TU.
#pragma once
#include <vector>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/lte_phy.h"
#include "lte_common.h"

namespace lte {

// Per code-block-slot description (one entry per CB index r of a frame).
struct CbInfo {
  int K, F, info, off, crc;   // segmentation.py:74-263
  int f1, f2;                 // QPP (turbo_encoder.py:34-73)
  int E;                      // rate-matched length
};

struct Grid {                 // device pointers + numerology for one plan
  int N, log2N, Nc, cp, Nd, Np, bps, n_sym, L, n_grp;
  const int32_t* data_idx;    // [Nd]
  const int32_t* pilot_idx;   // [Np]
  const float2* pilots;       // [Np]
  const int32_t* seg;         // [N]  left pilot of the interpolation segment
  const float* inv_gap;       // [Np] 1/(p_{i+1}-p_i)
  const float2* tw;           // [N]
  const float2* constel;      // [M]
  float qscale;               // sqrt(2) / sqrt(10) / sqrt(42)
  // SC-FDM (M = Nd point DFT by Bluestein's chirp-z on N-point FFTs, Nd < N/2):
  const float2* chirp;        // [Nd] exp(-i pi n^2 / Nd)
  const float2* bhat;         // [N]  FFT_N(exp(+i pi m^2 / Nd), circular) / (N sqrt(Nd))
  int no_eq;                  // uncoded SISO: slice the raw FFT output (enable_equalization=False)
  // float64 copies of the tables for the f64 chain (null in f32 plans)
  const double2* pilots64;
  const double* inv_gap64;
  const double2* tw64;
  const double2* chirp64;
  const double2* bhat64;
  // per-subcarrier role for the wave-private receivers: data ordinal j >= 0,
  // pilot ordinal p as -(p + 2), -1 guard / DC  [N]
  const int32_t* kinfo;
};
// precision-selected table accessors (R = float / double)
template <class R> struct GridT;
template <> struct GridT<float> {
  __host__ __device__ static const float2* tw(const Grid& g) { return g.tw; }
  __host__ __device__ static const float2* pilots(const Grid& g) { return g.pilots; }
  __host__ __device__ static const float* inv_gap(const Grid& g) { return g.inv_gap; }
  __host__ __device__ static const float2* chirp(const Grid& g) { return g.chirp; }
  __host__ __device__ static const float2* bhat(const Grid& g) { return g.bhat; }
};
template <> struct GridT<double> {
  __host__ __device__ static const double2* tw(const Grid& g) { return g.tw64; }
  __host__ __device__ static const double2* pilots(const Grid& g) { return g.pilots64; }
  __host__ __device__ static const double* inv_gap(const Grid& g) { return g.inv_gap64; }
  __host__ __device__ static const double2* chirp(const Grid& g) { return g.chirp64; }
  __host__ __device__ static const double2* bhat(const Grid& g) { return g.bhat64; }
};

// launchers (return hipError_t as int)
constexpr int CRC24A_POLY = 0x864CFB, CRC24B_POLY = 0x800063;   // crc.py polynomials without x^24
// crc: CRC polynomial to append (0: none)
int launch_payload(hipStream_t s, uint32_t* pw, int PW, int n_bits, int crc, const uint64_t* fid,
                   uint64_t seed, int B, const uint32_t* inj, int64_t inj_stride);
// qmask: encode_qmask(cbs, C, qstride) on the host, C x qstride uint16, qstride >= max K + 32 and a
// multiple of 2 (the kernel reads whole 32-entry rows as uint32 pairs; entries past K are zero)
void encode_qmask(const CbInfo* cbs, int C, int qstride, uint16_t* out);
int launch_encode(hipStream_t s, const uint32_t* pw, int PW, int KWmax, uint32_t* enc, int EW,
                  const CbInfo* cbi_dev, int C, int B, const uint16_t* qmask, int qstride);
// Signal-chain launchers, R = double (the reference's precision, default) or
// float (fast mode); explicit instances in lte_kernels.hip.
template <class R>
int launch_ofdm_tx(hipStream_t s, const Grid& g, int coded, const uint32_t* pw, int PW, const uint32_t* enc,
                   int enc_words, const int32_t* tx_map, cx<R>* x, int B, cx<R>* cap_syms = nullptr,
                   int sc_fdm = 0);
template <class R>
int launch_fading(hipStream_t s, int B, int num_rx, int n_paths, const R* gains_dev, const uint64_t* fid,
                  uint64_t seed, const R* inj_ph, int64_t inj_stride, R* phases, cx<R>* coef);
template <class R>
int launch_channel(hipStream_t s, const Grid& g, int B, int num_rx, int rayleigh, int n_paths,
                   const int32_t* delays_dev, const R* gains_dev, R fD, R fs, const R* phases, const cx<R>* coef,
                   const cx<R>* x, cx<R>* y, R* pow_part, int nblk, int max_delay);
template <class R>
int launch_npow(hipStream_t s, int B, int num_rx, const R* pow_part, int nblk, int L, const R* snr_lin, R* npow);
int channel_nblk(int L);   // power partials per (frame, rx) written by launch_channel
// OFDM TX with the static-tap multipath channel fused in (SISO, fD = 0, every
// delay <= CP, N >= 512): k_ofdm_tx<.., CH> writes the received stream outside
// each symbol's CP (the only samples the receiver reads) and the power of the
// channel output over the symbol's samples [max_delay, N + cp); k_chan_fix adds
// the power of the first max_delay samples, which need the previous symbol's
// tail (kept per symbol in xh).  pow_part then holds n_sym partials per frame.
constexpr int TXCH_MAXP = 8;
template <class R>
struct TxChannelT {
  int n_paths, max_delay;
  int num_rx;          // receive antennas (SIMO: independent taps per RX, y / coef / pow_part per RX)
  int delays[TXCH_MAXP];
  const cx<R>* coef;   // [B][num_rx][n_paths]
  cx<R>* y;            // [B][num_rx][L]
  cx<R>* xh;           // [B][n_sym][2 * max_delay]: first / last max_delay TX samples of each symbol
  R* pow_part;         // [B][num_rx][n_sym]
  // fD != 0: per-symbol Taylor sets of every path [B][num_rx][n_paths][n_sym][mimo_ncf<R>()]
  // (k_jakes_sets); null for static taps (coef)
  const cx<R>* tcoef;
  // static taps, SIMO into the paired receiver (k_rx_frame_simo2<.., XIN>):
  // non-null, the TX writes each symbol's N time samples here [B][n_sym][N]
  // (f64 scaled as ifft * sqrt(N), f32 unscaled with the scale in the taps)
  // instead of num_rx received streams; the receiver applies the taps
  cx<R>* x_out;
};
bool txch_supported(const Grid& g, int n_paths, int max_delay);
// host payload bits (one uint8 per bit, frames `stride` bytes apart) already on
// the device -> packed MSB-first words [nf][nwd]
int launch_pack_bits(hipStream_t s, const uint8_t* bits, int64_t stride, int n_bits, int nwd, int nf, uint32_t* out);
// the Philox mode's raw streams: per (frame, counter) the 4 outputs of rng4 and
// the unit normal pairs of gauss2<double> / gauss2<float> (any pointer may be null)
int launch_philox_draws(hipStream_t s, uint64_t seed, const uint64_t* fid, int nf, uint32_t stream, int64_t n_ctr,
                        uint32_t* u, double* g64, float* g32);
// per-OFDM-symbol Taylor sets of the SISO paths from k_fading's phases (the
// fused TX channel at fD != 0): [B][n_paths][n_sym][mimo_ncf<R>()]
template <class R>
int launch_jakes_sets(hipStream_t s, int B, int n_paths, int n_sym, int sym_len, const R* phases, const R* gains,
                      double fD, double fs, cx<R>* tcoef);
template <class R>
int launch_ofdm_tx_ch(hipStream_t s, const Grid& g, int coded, const uint32_t* pw, int PW, const uint32_t* enc,
                      int enc_words, const int32_t* tx_map, int B, cx<R>* cap_syms, const TxChannelT<R>& ch,
                      int sc_fdm = 0);
template <class R>
int launch_chan_fix(hipStream_t s, const Grid& g, int B, const TxChannelT<R>& ch);
// coded TX + channel with one slot per frame (the frame's coded streams staged
// in LDS once); same outputs as launch_ofdm_tx_ch(coded = 1).  txf_map / txf_re
// (both or neither): the bank-aware lane order of plan_txf_lane_order --
// [n_sym][N/2][bps] sources and [n_sym][N/2] RE of each slot.
template <class R>
int launch_ofdm_txf(hipStream_t s, const Grid& g, const uint32_t* enc, int enc_words, const int32_t* tx_map,
                    const int32_t* txf_map, const int32_t* txf_re, int B, cx<R>* cap_syms,
                    const TxChannelT<R>& ch);
// wave-private f64 coded TX + static taps (lte_wave.hip), N = 2048, SISO, four
// paths with every delay <= 64: launch_ofdm_txf's outputs; it dispatches to
// it with LTE_TX_WAVE=1 (off by default)
bool txf_w_supported(const Grid& g, int f64, int n_paths, int max_delay, int num_rx, int tv);
int tx_wave_enabled();
int launch_ofdm_txf_w(hipStream_t s, const Grid& g, const uint32_t* enc, int enc_words, const int32_t* tx_map, int B,
                      double2* cap_syms, const TxChannelT<double>& ch);
// the lane order: for each OFDM symbol a permutation of its Nd data REs over
// the N/2 TX slots, greedy per 32-slot group (one ds_read_b32 lane group) so
// that each of the bps coded-bit gathers sees as few distinct words per LDS
// bank (word mod 32) as it can, and each 8-slot group (one ds_write_b128 lane
// group) distinct RE positions mod 8.  tx_map [n_sym][Nd][bps]; returns the
// modelled extra LDS cycles per 32-lane gather before / after in model[2].
void plan_txf_lane_order(const std::vector<int32_t>& tx_map, const std::vector<int32_t>& data_idx, int n_sym,
                         int Nd, int bps, int slots, std::vector<int32_t>& txf_map, std::vector<int32_t>& txf_re,
                         double model[2]);
template <class R>
int launch_rx_chest(hipStream_t s, const Grid& g, int B, int num_rx, const cx<R>* y, int64_t y_rx_stride,
                    int64_t y_frame_stride, const R* npow, const uint64_t* fid, uint64_t seed, const R* inj_z,
                    int64_t inj_stride, cx<R>* H, R* pstats);
// coded: nv_out set -> llr takes z (cx<R> per RE), nv_out sigma^2_eff
template <class R>
int launch_rx_data(hipStream_t s, const Grid& g, int chain, int rayleigh, int B, int num_rx, const cx<R>* y,
                   int64_t y_rx_stride, int64_t y_frame_stride, const cx<R>* H, const R* npow, const R* snr_lin,
                   const uint64_t* fid, uint64_t seed, const R* inj_z, int64_t inj_stride, const uint32_t* pw, int PW,
                   int n_bits, uint32_t* frame_err, R* llr, cx<R>* cap_syms, uint8_t* cap_bits, int sc_fdm = 0,
                   R* nv_out = nullptr);
// Fused SISO receiver (estimation + data path, one slot per frame): coded or
// uncoded, one RX, no SC-FDM.  nv_out set: llr takes z per RE and nv_out
// sigma^2_eff per (frame, group, data subcarrier); H / pstats: optional captures.
bool rx_frame_supported(const Grid& g, int chain, int num_rx, int sc_fdm);
// wave-private f64 coded receiver (lte_wave.hip): k_rx_frame's outputs (ZN demap:
// equalised symbols zo + sigma^2_eff nv_out) for N = 2048; launch_rx_frame
// dispatches to it with LTE_RX_WAVE=1 (off by default)
bool rx_frame_w_supported(const Grid& g, int chain, int f64);
int rx_wave_enabled();
int launch_rx_frame_w(hipStream_t s, const Grid& g, int rayleigh, int B, const double2* y, int64_t y_frame_stride,
                      const double* npow, const double* snr_lin, const uint64_t* fid, uint64_t seed,
                      const double* inj_z, int64_t inj_stride, double* zo, double* nv_out, double2* cap_syms,
                      double2* H, double* pstats);
template <class R>
int launch_rx_frame(hipStream_t s, const Grid& g, int chain, int rayleigh, int B, const cx<R>* y,
                    int64_t y_frame_stride, const R* npow, const R* snr_lin, const uint64_t* fid, uint64_t seed,
                    const R* inj_z, int64_t inj_stride, const uint32_t* pw, int PW, int n_bits, uint32_t* frame_err,
                    R* llr, cx<R>* cap_syms, uint8_t* cap_bits, R* nv_out, cx<R>* H, R* pstats);
// Fused SIMO MRC receiver (uncoded, 2..RXS_MAXRX RX): one slot per frame walks
// its symbols, every RX's estimate in registers; H / pstats: optional captures
// [B][num_rx][n_grp][N] / [B][num_rx][n_grp][2].
constexpr int RXS_MAXRX = 4;
bool rx_frame_simo_supported(const Grid& g, int num_rx);
template <class R>
int launch_rx_frame_simo(hipStream_t s, const Grid& g, int B, int num_rx, const cx<R>* y, int64_t y_rx_stride,
                         int64_t y_frame_stride, const R* npow, const uint64_t* fid, uint64_t seed, const R* inj_z,
                         int64_t inj_stride, const uint32_t* pw, int PW, int n_bits, uint32_t* frame_err,
                         cx<R>* cap_syms, uint8_t* cap_bits, cx<R>* H, R* pstats,
                         const TxChannelT<R>* xc = nullptr);
// the paired SIMO receiver applies (N = 1024, an even RX count, no H / pilot
// statistics capture); xc->x_out (the TX's symbol handoff) needs it
bool rx_simo2_ok(const Grid& g, int num_rx, bool H, bool pstats);
// Rate dematch into the decoder rows (rows of R: float / double).  rx_map
// [n_layers][T]: layer 0 assigns, layers 1.. add in order (E > N_cb
// repetition, rate_matching.py:433-436).  g0: first 64-frame group.
// ch: chunk width of the decoder rows (turbo_chunk of their capacity in groups)
template <class R>
int launch_dematch(hipStream_t s, const R* llr, int T, int B, const int32_t* rx_map, int n_layers, R* const* blk,
                   const int64_t* rows, int ch, int g0 = 0);
// dematch with the soft demapper fused in: reads the equalised symbols z
// ([B][n_re]) and their noise variances ([B][n_grp][nd] per data subcarrier,
// from the receivers' nv_out mode; nv_pairs: [B][n_sym][nd / 2] per Alamouti
// RE pair, k_det_sfbc's) instead of LLRs; same decoder rows as
// launch_dematch (bps 4 / 6)
template <class R>
int launch_dematch_zn(hipStream_t s, const cx<R>* z, const R* nv, int n_re, int nd, int bps, int B,
                      const int32_t* rx_map, int n_layers, R* const* blk, const int64_t* rows, int ch, int g0 = 0,
                      int nv_pairs = 0);
// f64 != 0: the float64 decoder (bit-exact with the reference), blk / ckpt hold doubles
int launch_turbo(hipStream_t s, void* blk, void* ckpt, uint32_t* bits, int K, int f1, int f2, int iters,
                 int G, int mode, int f64, int ch);
struct TurboJob {           // one CB slot of a batch: G groups of 64 code blocks of size K
  void* blk;                // float / double rows (lte_decoder.hip)
  void* ck;
  uint32_t* bits;
  int K, f1, f2, G;
  int ch;                   // chunk width of blk / ck (turbo_chunk of their capacity); one per launch
};
constexpr int TURBO_MAX_JOBS = 16;
struct TurboJobs {
  TurboJob j[TURBO_MAX_JOBS];
  int n;
  int prefix[TURBO_MAX_JOBS + 1];
};
int launch_turbo_jobs(hipStream_t s, const TurboJob* jobs, int n, int iters, int mode, int f64);
// rate_dematching_turbo for any E (repeats summed in order): llr [ncb][E] -> out [ncb][n_out]
int launch_rate_dematch(hipStream_t s, const double* llr, int E, int Ncb, int n_out, const int32_t* src0, int64_t ncb,
                        double* out);
// exact log-MAP (set_decoder_mode(False)) for the float64 decoders; default max-log-MAP
void set_logmap(int on);
int logmap_on();
// one float64 BCJR pass of any length n (LogMAPDecoder.decode): app [ncb][n];
// alpha_scratch n * ncb * 8 doubles
int launch_bcjr64(hipStream_t s, const double* ls, const double* lp, const double* la, int n, int ncb,
                  double* alpha_scratch, double* app);
int launch_crc_count(hipStream_t s, const CbInfo* cbi_dev, int C, uint32_t* const* dec, const int* KW, int B,
                     const uint32_t* pw, int PW, int n_bits, uint32_t* frame_err, uint32_t* frame_crc,
                     uint8_t* cap_bits, int b0 = 0, const uint64_t* fid = nullptr, uint64_t seed = 0);
// (fid given: the transmitted words are re-drawn from k_payload's Philox counters instead of read from pw)
int launch_accumulate(hipStream_t s, int B, int coded, int n_bits, int n_snr, const int32_t* snr_idx,
                      const uint32_t* frame_err, const uint32_t* frame_crc, unsigned long long* counts);
template <class R>
int launch_fft(hipStream_t s, const Grid& g, int inverse, int64_t batch, const cx<R>* in, cx<R>* out);
template <class R>
int launch_dft(hipStream_t s, const Grid& g, int inverse, int64_t batch, const cx<R>* in, cx<R>* out);
template <class R>
int launch_llr(hipStream_t s, int bps, int64_t n, const cx<R>* syms, const R* nv, R* llr);
template <class R>
int launch_hard(hipStream_t s, int bps, int64_t n, const cx<R>* syms, uint8_t* bits);
// building-block stage kernels (lte_blocks.hip, float64, NumPy's operation order)
int launch_qam_map(hipStream_t s, int bps, int64_t n, const uint8_t* bits, double2* out);
int launch_hard_argmin(hipStream_t s, int bps, int64_t n, const double2* y, uint8_t* bits);
int launch_chest(hipStream_t s, int N, int P, const int32_t* pidx, const double2* known, int64_t batch,
                 const double2* Y, double2* H, double2* hp, double* stats);
int launch_zf(hipStream_t s, int64_t n, const double2* Y, const double2* H, double reg, double2* out);
int launch_crc_serial(hipStream_t s, int64_t n, const uint8_t* bits, uint32_t poly_low, int len, uint32_t* out);
int launch_rsc(hipStream_t s, int64_t n, const uint8_t* u, int term, uint8_t* sys, uint8_t* par);

// ---------------------------------------------------------------- multi-antenna chains
// SFBC 2xN (configs 4 / simulate_miso / simulate_mimo) and TM4 spatial
// multiplexing (config 5 and its generalisation).  lte_mimo.hip.
enum { MIMO_SFBC = 0, MIMO_SPATIAL = 1 };
// terms per fading coefficient set: h(c + d) = sum_k c_k d^k, d in samples from
// the set's centre (f32: degree 2; f64: degree 5, remainder under float64 rounding)
template <class R> constexpr int mimo_ncf() { return sizeof(R) == 8 ? 6 : 3; }
// f64 expands the Jakes sum per coefficient set when |w_max| * half-span <= 2.7e-3
// (degree-5 remainder < 1e-17); otherwise it evaluates it per sample (exact_jakes)
inline bool mimo_taylor_ok(double fD, double fs, int span) {
  return 6.283185307179586 * (fD < 0 ? -fD : fD) / fs * (0.5 * span) <= 2.7e-3;
}
// f32's per-symbol quadratic: truncation (|w| S / 2)^3 / 6 under float32's
// half ulp (6e-8) while |w| S / 2 <= 7e-3 (~20 km/h at 20 MHz); past it the
// per-sample sum (exact_jakes) in float64 arithmetic, rounded to float
inline bool mimo_taylor_ok_prec(bool f64, double fD, double fs, int span) {
  return f64 ? mimo_taylor_ok(fD, fs, span) : 6.283185307179586 * (fD < 0 ? -fD : fD) / fs * (0.5 * span) <= 7e-3;
}
struct MimoGrid {
  int mode, num_tx, num_rx;
  int res;                 // QAM symbols per OFDM symbol: SFBC Nd&~1, spatial Nd
  int n_dsc;               // data SCs that carry data: SFBC Nd&~1, spatial ceil(Nd/num_tx)
  int maxP;                // pilot stride of the per-TX tables
  int n_est;               // channel estimates per frame (SFBC: one per 14-symbol group; spatial: every symbol)
  int n_cs;                // fading coefficient sets per link path (1 if fD == 0 or exact Jakes, else n_sym)
                           // each of mimo_ncf<R>() terms: f32 A + B d + C d^2, f64 the degree-5 Taylor
  const int32_t* np_tx;    // [num_tx] pilots of each TX
  const int32_t* ppos;     // [num_tx][maxP] pilot subcarriers of TX t
  const float2* pval;      // [num_tx][maxP] pilot symbols of TX t
  const float* pig;        // [num_tx][maxP] 1/(gap to the next pilot of TX t)
  const int32_t* pseg;     // [num_tx][n_dsc] left pilot (within TX t's set) of data SC j; -1 / >= np-1: edge hold
  int rank, det;           // spatial: layers, LTE_DET_*
  const double* W;         // spatial: [4][4] complex (re, im) precoder, entry (t, c) at (t*4 + c)*2
  // float64 plans: the pilot tables in float64, and for fD != 0 the exact
  // Jakes sum per sample (jakes_fading, rayleighchannel.py:20-42): jw[m] =
  // (2 pi fD) cos(alpha_m) as the reference forms it, the 16 phases of every
  // link path in the channel kernels' `phases` buffer
  const double2* pval64;
  const double* pig64;
  int exact_jakes;
  double jw[16];
};
template <class R> struct MGT;
template <> struct MGT<float> {
  __host__ __device__ static const float2* pval(const MimoGrid& m) { return m.pval; }
  __host__ __device__ static const float* pig(const MimoGrid& m) { return m.pig; }
};
template <> struct MGT<double> {
  __host__ __device__ static const double2* pval(const MimoGrid& m) { return m.pval64; }
  __host__ __device__ static const double* pig(const MimoGrid& m) { return m.pig64; }
};
// Multi-antenna launchers, R = double (the reference's complex128, default)
// or float (fast mode); explicit instances in lte_mimo.hip.
// transmit_mimo's link power made by the TX kernel (part = null: not asked for):
// per link and OFDM symbol the power of the link's faded signal (static taps)
template <class R>
struct TxLinkPower {
  const int32_t* delays;   // [n_paths] (device)
  const cx<R>* coef;       // [B][num_rx][num_tx][n_paths][mimo_ncf<R>()] (n_cs = 1)
  R* part;                 // [B][num_rx][num_tx][nblk]
  int n_paths, max_delay, nblk;
  // k_ofdm_txch_sfbc only, 1: the merged link noise -- part's two entries per
  // RX are the links' powers summed and the RX stream's power
  int merged;
};
template <class R>
int launch_ofdm_tx_mimo(hipStream_t s, const Grid& g, const MimoGrid& m, int coded, const uint32_t* pw, int PW,
                        const uint32_t* enc, int enc_words, const int32_t* tx_map, cx<R>* x, int B,
                        const TxLinkPower<R>& lp);
// per link path: f32 h(n) = A + B d + C d^2 around the centre of n's OFDM
// symbol (fD != 0), or A (fD == 0); f64 A (fD == 0) or the phases (exact Jakes)
template <class R>
int launch_fading_mimo(hipStream_t s, const Grid& g, const MimoGrid& m, int B, int rayleigh, int n_paths,
                       const R* gains, double fD, double fs, const uint64_t* fid, uint64_t seed,
                       const R* inj_ph, int64_t inj_ph_stride, const R* inj_h, int64_t inj_h_stride,
                       cx<R>* coef, R* phases);
// TX + flat (AWGN) channel in one pass per (frame, symbol, RX): y [B][num_rx][L]
// and pow_part [B][num_rx][nblk] (per OFDM symbol); coef from launch_fading_mimo
template <class R>
int launch_ofdm_txch_flat(hipStream_t s, const Grid& g, const MimoGrid& m, int coded, const uint32_t* pw, int PW,
                          const uint32_t* enc, int enc_words, const int32_t* tx_map, const cx<R>* coef, cx<R>* y,
                          R* pow_part, int nblk, int B);
// config 4: SFBC TX + static-tap Rayleigh links in one pass per frame (y gets
// the faded RX signals, lp.part one power per link); then the link sigmas, the
// combined link noise added to y and the RX power partials pow_part
// [B][num_rx][*pow_nblk] (*pow_nblk = 1: one per frame and RX)
template <class R>
bool sfbc_txch_supported(const Grid& g, const MimoGrid& m, int n_paths, int max_delay);
template <class R>
int launch_ofdm_txch_sfbc(hipStream_t s, const Grid& g, const MimoGrid& m, int coded, const uint32_t* pw, int PW,
                          const uint32_t* enc, int enc_words, const int32_t* tx_map, const TxLinkPower<R>& lp,
                          cx<R>* y, int B);
// config 4's merged link noise (Philox mode, full chain, no capture of the
// received streams or noise powers): instead of adding the RX's 100 dB link
// noise to y0_r (k_link_noise_pairs) and measuring the noisy power, the RX's
// one noise draw in the receiver carries both, per RX (from the two partials
// k_ofdm_txch_sfbc<.., MRG> writes: sum_t sum_n |y0_rt|^2 and sum_n |y0_r|^2)
//   s2 = ((sum_t p_rt / L) / 1e10) / 2   (the links' sigma^2 per component),
//   P = sum_n |y0_r|^2 / L + 2 s2        (the link noise's power in expectation),
//   npow_awgn = (P / num_tx) / snr,  npow_eff = 2 s2 + npow_awgn,
// and k_rx_sfbc draws sqrt(npow_eff / 2) per component: the same distribution
// as the two draws (independent Gaussians add) with P's link-noise term
// (~1e-10 of P) in expectation.  oracle/philox.sfbc_draws(merged=True).
template <class R>
int launch_npow_sfbc_merged(hipStream_t s, int B, int num_rx, int num_tx, const R* link_part, int L, const R* snr_lin,
                            R* npow);
template <class R>
int launch_link_noise_add(hipStream_t s, const Grid& g, const MimoGrid& m, int B, const R* link_part, R* link_sigma,
                          cx<R>* y, const uint64_t* fid, uint64_t seed, R* pow_part, int* pow_nblk);
// phases / gains: exact-Jakes mode (m.exact_jakes) only
template <class R>
int launch_channel_mimo(hipStream_t s, const Grid& g, const MimoGrid& m, int B, int n_paths, const int32_t* delays,
                        const cx<R>* coef, const R* phases, const R* gains, double fs, const cx<R>* x, cx<R>* y,
                        int link_noise, const uint64_t* fid, uint64_t seed, const R* inj_lz, int64_t inj_lz_stride,
                        R* link_part, R* link_sigma, R* pow_part, int nblk, int link_part_done = 0);
// OFDM symbols (blocks of N + cp samples) of a stream: the power partials per
// (frame, rx) the multi-antenna channel passes write
int mimo_channel_nblk(int L, int sym_len);
// per link [mean|x|^2, mean|y|^2, Re, Im mean(y conj x)] of the link's output
// y (with its 100 dB link noise when link_sigma is set)
template <class R>
int launch_link_stats(hipStream_t s, const Grid& g, const MimoGrid& m, int B, int n_paths, const int32_t* delays,
                      const cx<R>* coef, const R* phases, const R* gains, double fs, const cx<R>* x,
                      const R* link_sigma, const uint64_t* fid, uint64_t seed, const R* inj_lz, int64_t inj_lz_stride,
                      R* part, int nblk, R* stats);
// noise power per RX: ((P / div) / snr): div = num_tx (transmit_mimo) or 1 (spatial)
template <class R>
int launch_npow_mimo(hipStream_t s, int B, int num_rx, const R* pow_part, int nblk, int L, const R* snr_lin,
                     double div, R* npow);
// wave-private f64 RX FFT + CRS pilot estimates (lte_wave.hip), N = 2048, the
// pilot-estimate handoff: launch_rx_fft_mimo's outputs; it dispatches to it
// unless LTE_MIMO_RX_WAVE=0
bool rx_fft_mimo_w_supported(const Grid& g, const MimoGrid& m, int f64, int h_pilots);
int mimo_rx_wave_enabled();
bool rx_simo_w_supported(const Grid& g, int num_rx, int f64, bool H, bool pstats, bool xin);
int simo_rx_wave_enabled();
bool tx_simo_w_supported(const Grid& g, int f64, int coded, int sc_fdm, const TxChannelT<double>& ch);
int simo_tx_wave_enabled();
bool tx_simo_w_fuses_fix(const Grid& g, int coded, int sc_fdm, const TxChannelT<double>& ch);
int launch_ofdm_tx_simo_w(hipStream_t s, const Grid& g, const uint32_t* pw, int PW, int B, double2* cap_syms,
                          const TxChannelT<double>& ch);
int launch_rx_frame_simo_w(hipStream_t s, const Grid& g, int B, int num_rx, const double2* y, int64_t y_rx_stride,
                           int64_t y_frame_stride, const double* npow, const uint64_t* fid, uint64_t seed,
                           const double* inj_z, int64_t inj_stride, const uint32_t* pw, int PW, int n_bits,
                           uint32_t* frame_err, double2* cap_syms, uint8_t* cap_bits);
int launch_rx_fft_mimo_w(hipStream_t s, const Grid& g, const MimoGrid& m, int B, const double2* y, const double* npow,
                         const uint64_t* fid, uint64_t seed, const double* inj_z, int64_t inj_stride, double2* Y,
                         double2* H);
template <class R>
// h_pilots: H receives the LS pilot estimates [b][rx][e][tx][maxP] instead of
// the interpolated [b][rx][e][tx][n_dsc] (launch_det_spatial's h_pilots
// interpolates them per RE with the same mimo_interp)
int launch_rx_fft_mimo(hipStream_t s, const Grid& g, const MimoGrid& m, int B, const cx<R>* y, const R* npow,
                       const uint64_t* fid, uint64_t seed, const R* inj_z, int64_t inj_stride, cx<R>* Y, cx<R>* H,
                       int h_pilots = 0);
// config 4's receiver + SFBC detector in one pass per frame (k_rx_sfbc): the
// outputs of launch_rx_fft_mimo + launch_det_sfbc (zn handoff or bit errors)
// without Y / H in HBM
template <class R>
bool rx_sfbc_supported(const Grid& g, const MimoGrid& m);
template <class R>
int launch_rx_sfbc(hipStream_t s, const Grid& g, const MimoGrid& m, int coded, int B, const cx<R>* y, const R* npow,
                   const uint64_t* fid, uint64_t seed, const R* snr_lin, const uint32_t* pw, int PW, int n_bits,
                   uint32_t* frame_err, cx<R>* zo, R* nvo);
template <class R>
// coded: LLRs to llr, or (zo != null) the combined symbols to zo [B][n_sym][res]
// and sigma^2_eff per RE pair to nvo [B][n_sym][res / 2] for launch_dematch_zn
int launch_det_sfbc(hipStream_t s, const Grid& g, const MimoGrid& m, int coded, int rayleigh, int B, const cx<R>* Y,
                    const cx<R>* H, const R* snr_lin, const uint32_t* pw, int PW, int n_bits, uint32_t* frame_err,
                    R* llr, cx<R>* cap_syms, uint8_t* cap_bits, cx<R>* zo = nullptr, R* nvo = nullptr);
template <class R>
int launch_det_spatial(hipStream_t s, const Grid& g, const MimoGrid& m, int B, const cx<R>* Y, const cx<R>* H,
                       const double* nvar, const uint32_t* pw, int PW, int n_bits, uint32_t* frame_err,
                       cx<R>* cap_syms, uint8_t* cap_bits, int h_pilots = 0);
// SFBCAlamouti.encode (decode = 0: a = symbols -> o0 = TX0, o1 = TX1) / .decode
// (decode = 1: a = rx, h0 / h1 the per-SC estimates -> o0), float64 [n] complex, n even
int launch_sfbc_stage(hipStream_t s, int decode, int64_t n, const double* a, const double* h0, const double* h1,
                      double reg, double* o0, double* o1);
int launch_det_stage(hipStream_t s, int det, int NR, int NT, int R, int bps, int64_t n, const double* y,
                     const double* H, const double* W, double s2, double* out);

// ---------------------------------------------------------------- beamforming (lte_bf.hip)
constexpr int LTE_BF_MAX_TX = 8, LTE_BF_MAX_RX = 8;
// per frame: channel, precoder, effective channel, 1/||H_eff||^2, PMI, gain;
// R = double (the default) / float (fast mode)
template <class R>
struct BfFrameT {
  cx<R> H[LTE_BF_MAX_RX][LTE_BF_MAX_TX];
  cx<R> W[LTE_BF_MAX_TX];
  cx<R> He[LTE_BF_MAX_RX];
  R inv_p;
  int pmi;
  double gain_db;
};
// sigma: per frame noise scale sqrt(10^(-SNR/10) / 2) (core/ofdm_core.py:2397-2399)
template <class R>
int launch_bf(hipStream_t s, int B, int n_sym, int Nd, int bps, int num_tx, int num_rx, int adaptive, int ncb,
              const double* cb, const uint64_t* fid, uint64_t seed, const R* inj_h, int64_t inj_h_stride,
              BfFrameT<R>* fr, const R* sigma, const uint32_t* pw, int PW, int n_bits, const R* inj_z,
              int64_t inj_z_stride, uint32_t* frame_err, cx<R>* cap_syms, uint8_t* cap_bits);

// turbo modes
enum { TM_DEC1 = 0, TM_DEC2 = 1, TM_DECODE = 2, TM_APP = 3, TM_FINAL = 4 };  // TM_DECODE: full decode (iterations + decisions)
// turbo geometry: rows of one (r, group) block = 4K+12: LS (sys + sys1 tail,
// K + 3), LP1 (K + 3), LP2 (K + 3), LS2T (decoder 2's sys tail, 3), LE (K);
// placement: trow_* below
__host__ __device__ inline int64_t turbo_rows(int K) { return 4LL * K + 12; }
// Row of each decoder input / the extrinsic within a block (LTE_TURBO_ILV):
//  3: all four rows of step k side by side -- [4k] LS, [4k+1] LE, [4k+2] LP1,
//    [4k+3] LP2 -- then the LS, LP1, LP2 tails and LS2T (3 each);
//  2 (default): decoder 1's three rows of step k side by side -- [3k] LS(k),
//    [3k+1] LE(k), [3k+2] LP1(k) for k < K -- so its step reads one contiguous
//    1.5 KB span (f64) and decoder 2's step at pi(k) a 1 KB LS / LE span;
//    then LS tail (3), LP1 tail (3), LP2 (K + 3), LS2T (3);
//  1: [2k] LS(k), [2k+1] LE(k); LS tail, LP1, LP2, LS2T;
//  0: sequential LS, LP1, LP2, LS2T, LE.
// A/B on MI355X (f64 decoder, 65 536 frames): see DESIGN.md §5.
#ifndef LTE_TURBO_ILV
#define LTE_TURBO_ILV 1
#endif
__host__ __device__ inline int64_t trow_ls(int K, int k) {   // k in [0, K + 3)
  if (LTE_TURBO_ILV == 3) return k < K ? 4LL * k : 4LL * K + (k - K);
  if (LTE_TURBO_ILV == 2) return k < K ? 3LL * k : 3LL * K + (k - K);
  if (LTE_TURBO_ILV == 1) return k < K ? 2LL * k : (int64_t)K + k;
  return k;
}
__host__ __device__ inline int64_t trow_le(int K, int k) {   // k in [0, K)
  return LTE_TURBO_ILV == 3 ? 4LL * k + 1 : LTE_TURBO_ILV == 2 ? 3LL * k + 1 : LTE_TURBO_ILV == 1 ? 2LL * k + 1
                                                                                           : 3LL * K + 12 + k;
}
__host__ __device__ inline int64_t trow_lp(int K, int dec, int k) {   // dec 1 / 2, k in [0, K + 3)
  if (LTE_TURBO_ILV == 3) return k < K ? 4LL * k + 1 + dec : 4LL * K + 3 * dec + (k - K);
  if (LTE_TURBO_ILV == 2) return dec == 1 ? (k < K ? 3LL * k + 2 : 3LL * K + 3 + (k - K)) : 3LL * K + 6 + k;
  if (LTE_TURBO_ILV == 1) return (dec == 1 ? 2LL * K + 3 : 3LL * K + 6) + k;
  return (dec == 1 ? (int64_t)K + 3 : 2LL * K + 6) + k;
}
__host__ __device__ inline int64_t trow_ls2t(int K, int j) { return (LTE_TURBO_ILV ? 4LL * K + 9 : 3LL * K + 9) + j; }
__host__ __device__ inline int turbo_nwin(int K) { return K / 8 + 1; }  // checkpoint windows (>= 8 steps each)
// alpha checkpoint rows per window: f32 states 1..7 (state 0 is 0 after
// normalisation); f64 all 8 states (unnormalised, as the reference)
constexpr int TURBO_CK_ROWS_F32 = 7;
constexpr int TURBO_CK_ROWS_F64 = 8;
__host__ __device__ inline int turbo_ck_rows(int f64) { return f64 ? TURBO_CK_ROWS_F64 : TURBO_CK_ROWS_F32; }
constexpr int TURBO_RS = 64;   // decoder row stride (elements): 64 code blocks per wave
// Block arrays (decoder rows, checkpoints) are chunked over frame groups:
// [chunk][row][CH groups][64 lanes], so the rows of CH waves that run side by
// side share DRAM pages and TLB entries.  CH = TURBO_CH for arrays of at least
// TURBO_CH groups (which then allocate whole chunks); arrays of fewer groups
// (small plans, the host entry points) take CH = 1, each group's block
// contiguous, and allocate exactly their groups (turbo_chunk / turbo_galloc of
// the array's capacity in groups).  Every launch on an array passes its CH.
#ifndef LTE_TURBO_CH
#define LTE_TURBO_CH 32
#endif
constexpr int TURBO_CH = LTE_TURBO_CH;
__host__ __device__ inline int turbo_chunk(int64_t G) { return G < TURBO_CH ? 1 : TURBO_CH; }
__host__ __device__ inline int64_t turbo_galloc(int64_t G) {
  return turbo_chunk(G) == 1 ? G : (G + TURBO_CH - 1) / TURBO_CH * TURBO_CH;
}
// element offset of lane 0 of (group g, row) in a block array of `rows` rows per group
template <int CH = TURBO_CH>
__host__ __device__ inline int64_t turbo_elem(int64_t rows, int64_t g, int64_t row) {
  return (((g / CH) * rows + row) * CH + g % CH) * TURBO_RS;
}
// the same for a runtime chunk width (1 or TURBO_CH)
__host__ __device__ inline int64_t turbo_elem_ch(int ch, int64_t rows, int64_t g, int64_t row) {
  return ch == 1 ? turbo_elem<1>(rows, g, row) : turbo_elem<TURBO_CH>(rows, g, row);
}
__host__ __device__ inline int turbo_kw(int K) { return (K + 31) / 32; }

}  // namespace lte
