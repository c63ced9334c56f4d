/*
 * lte_phy.h -- C ABI of liblte_hip.so, the gfx950 (MI355X) LTE PHY link engine.
 *
 * The reference (Darioxavierl/OFDM-LTE) is pure Python/NumPy and has no FFI;
 * its drop-in boundary is the Python class API (ofdm_module.py:32-207,
 * core/ofdm_core.py:42-2486).  This header is the native boundary underneath
 * the Python mirror of that API (ofdm-lte_amd/lte_phy/): plain C, plain
 * pointers and sizes, no torch or C++ types.  Each entry point names the
 * reference function(s) whose work it replaces.
 *
 * Conventions: every function returns LTE_OK (0) or a negative LTE_E* code;
 * lte_strerror() / lte_last_error() describe it.  Host buffers are owned by
 * the caller; device memory is owned by the library (one plan = one device
 * workspace).  All calls are synchronous at return.  One plan per thread.
 */
#ifndef LTE_PHY_H
#define LTE_PHY_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  LTE_OK = 0,
  LTE_EINVAL = -1,  /* bad argument (mirrors the reference's ValueError)      */
  LTE_EHIP = -2,    /* HIP runtime / launch failure                             */
  LTE_ENOMEM = -3,  /* device allocation failed                                 */
  LTE_ENODEV = -4,  /* no gfx950 device                                         */
  LTE_EUNSUP = -5   /* configuration outside what the GPU path implements       */
};

/* Chain kinds: which reference simulate_* method a plan runs. */
enum {
  LTE_CHAIN_UNCODED = 0, /* OFDMSimulator.simulate_siso      core/ofdm_core.py:660-737   */
  LTE_CHAIN_CODED = 1,   /* OFDMSimulator.simulate_siso_coded core/ofdm_core.py:925-1338 */
  LTE_CHAIN_SIMO = 2,    /* OFDMSimulator.simulate_simo (MRC) core/ofdm_core.py:1536-1679 */
  /* SFBC Alamouti 2 x num_rx, uncoded: simulate_miso / simulate_mimo
   * (core/ofdm_core.py:1850-2258) with the estimator fix of SURVEY Q19 */
  LTE_CHAIN_SFBC = 3,
  /* config 4: the SISO coding chain (simulate_siso_coded TX/RX coding,
   * core/ofdm_core.py:1003-1299) around SFBC 2 x num_rx */
  LTE_CHAIN_SFBC_CODED = 4,
  /* TM4 spatial multiplexing, 2 / 4 TX x 1-4 RX, rank 1-4, codebook precoder,
   * MMSE / ZF / SIC / MRC detection: simulate_spatial_multiplexing
   * core/ofdm_core.py:2489-2815 (config 5 = 4x4, rank 4, PMI 0, MMSE) */
  LTE_CHAIN_SPATIAL = 5,
  /* beamforming, frequency domain only as in the reference: flat H per frame,
   * rank-1 codebook PMI feedback, static codebook or adaptive MRT precoder, MRC:
   * OFDMSimulator.simulate_beamforming core/ofdm_core.py:2260-2477.  num_tx
   * 2 / 4 / 8, num_rx 1-8; L = n_sym * Nd REs per antenna (noise layout). */
  LTE_CHAIN_BEAMFORMING = 6
};
/* MIMODetector.detector_type (core/mimo_detector.py:116-133); IRC == MMSE */
enum { LTE_DET_MMSE = 0, LTE_DET_ZF = 1, LTE_DET_SIC = 2, LTE_DET_MRC = 3 };
enum { LTE_CH_AWGN = 0, LTE_CH_RAYLEIGH = 1 }; /* core/channel.py:10-245 */

/* Arithmetic type of a plan's signal chain and turbo decoder.  DEFAULT =
 * float64 for every chain (the reference computes in float64 / complex128
 * throughout); F32 is the opt-in fast mode.  ABI version 2 (lte_version):
 * in version 1 DEFAULT meant float32 for the multi-antenna and beamforming
 * chains -- their real / complex captures and in_signal are now float64 /
 * complex128 unless LTE_PREC_F32 is asked for ("ABI
 * versions"). */
enum { LTE_PREC_DEFAULT = 0, LTE_PREC_F32 = 32, LTE_PREC_F64 = 64 };

/* ABI version this header describes; lte_version() returns the library's.
 * A client checks lte_version() == LTE_ABI_VERSION once before any other call
 * (lte_abi_check(LTE_ABI_VERSION) does exactly that).  History (INTEGRATION.md "ABI versions"):
 *   1  LTE_PREC_DEFAULT = float32 for the multi-antenna / beamforming chains
 *   2  LTE_PREC_DEFAULT = float64 for every chain; cap_bf_gain double
 *   3  lte_run_args.snr_db is double (the reference's float64 SNR in dB) */
#define LTE_ABI_VERSION 3

#define LTE_MAX_PATHS 16
enum { LTE_STAGE_TX = 1, LTE_STAGE_CHANNEL = 2, LTE_STAGE_RX = 4, LTE_STAGE_ALL = 7 };

/* Plan descriptor.  Numerology follows LTEConfig (config.py:101-130); the
 * resource grid (guards, DC, pilot every 6th SC) is derived from N, Nc exactly
 * as LTEResourceGrid (core/resource_mapper.py:57-93). */
typedef struct {
  int32_t N, Nc, cp_len;   /* FFT size, useful SCs, CP samples                   */
  int32_t bps;             /* 2 / 4 / 6  (QPSK / 16-QAM / 64-QAM)                */
  int32_t n_sym;           /* OFDM symbols per frame (uncoded/SIMO); coded: 0=auto */
  int32_t chain;           /* LTE_CHAIN_*                                        */
  int32_t channel;         /* LTE_CH_*                                           */
  int32_t num_rx;          /* 1 for SISO, >=1 for SIMO                           */
  int32_t n_paths;         /* Rayleigh taps                                      */
  int32_t delays[LTE_MAX_PATHS]; /* integer sample delays round(tau*fs)          */
  double gains[LTE_MAX_PATHS];   /* linear amplitudes as RayleighChannel holds them */
  double fD;               /* max Doppler (Hz); 0 -> static taps                 */
  double fs;               /* sample rate (Hz)                                   */
  int32_t n_bits;          /* payload bits per frame (uncoded) / TB size (coded) */
  int32_t turbo_iters;     /* coded: decoder iterations (reference passes 8)     */
  int32_t max_frames;      /* workspace capacity (frames per lte_run call)       */
  int32_t cell_id;         /* pilot PN seed (PilotPattern cell_id), normally 0   */
  int32_t num_tx;          /* TX antennas: 1 (SISO/SIMO), 2 (SFBC), 4 (spatial).
                            * Multi-antenna gains: SFBC as RayleighChannel holds
                            * them; spatial links convert once more (Q2).  The
                            * multi-antenna chains use one link per (rx, tx).   */
  /* spatial chain only (LTE_CHAIN_SPATIAL): */
  int32_t rank;            /* layers, 1..min(num_tx, num_rx, 4); 0 -> num_tx with W = I */
  int32_t detector;        /* LTE_DET_*                                          */
  double precoder[32];     /* W [num_tx][rank] (LTECodebook.get_precoder, core/codebook_lte.py:
                            * 317-330): entry (t, c) at [(t*4 + c)*2] re, [+1] im */
  /* SC-FDM (enable_sc_fdm, core/dft_precoding.py): the uncoded SISO / SIMO
   * transmitters DFT-precode each symbol's Nd QAM symbols (core/modulator.py:
   * 232-236); the uncoded SISO receiver applies the IDFT after ZF
   * (core/lte_receiver.py:318-333).  As in the reference, the SIMO receiver
   * does not de-precode and the coded chain ignores the flag. */
  int32_t sc_fdm;
  /* beamforming chain: 0 = update_mode 'static' (the CSI-feedback codebook
   * vector), 1 = 'adaptive' (MRT, AdaptiveBeamforming) */
  int32_t bf_adaptive;
  /* uncoded SISO receiver without ZF (OFDMSimulator / OFDMReceiver
   * enable_equalization=False: receive_and_decode slices the raw FFT output,
   * core/lte_receiver.py:294-299; the CRS estimate still runs) */
  int32_t no_equalization;
  int32_t precision;       /* LTE_PREC_*                                         */
} lte_plan_desc;

typedef struct lte_plan lte_plan;

/* Per-call arguments of lte_run.  Frame b (0 <= b < n_frames) is one
 * independent (SNR, trial) unit.  Randomness: Philox4x32-10 keyed by
 * (seed, frame_id, stream, index); any non-NULL inject pointer replaces the
 * corresponding Philox draws (ref-compat mode: the host supplies the numbers
 * the reference's global NumPy RNG would draw).  *_stride = elements between
 * consecutive frames (0 = the same data broadcast to every frame). */
typedef struct {
  int32_t n_frames;
  /* host [n_frames] SNR in dB, float64 as the reference holds it; the library
   * forms 10 ** (snr_db / 10) (core/channel.py:32,191) and the detectors'
   * noise variances 1 / 10 ** (snr_db / 10) (core/ofdm_core.py:1224) or
   * 10 ** (-snr_db / 10) (:2397, :2737) from it in float64.  (ABI <= 2: float) */
  const double *snr_db;
  const int32_t *snr_index;    /* host [n_frames] row in counts (NULL -> 0)        */
  int32_t n_snr;               /* rows of counts                                   */
  uint64_t seed;
  const uint64_t *frame_ids;   /* host [n_frames] (NULL -> frame_id0 + b)          */
  uint64_t frame_id0;
  /* injection (host, optional) */
  const uint8_t *bits; int64_t bits_stride;     /* [.][n_bits] values 0/1          */
  const double *phases; int64_t phases_stride;  /* [.][num_rx][n_paths][16] rad
                                                   (multi-antenna: [.][num_rx][num_tx][n_paths][16]) */
  const double *noise; int64_t noise_stride;    /* [.][num_rx][2][L] unit normals  */
  /* outputs */
  uint64_t *counts;            /* host [n_snr][4] += {bit_err, bits, blk_err, blks} */
  uint32_t *frame_errors;      /* host [n_frames] optional                         */
  uint8_t *frame_crc_ok;       /* host [n_frames] optional (coded)                 */
  /* stage selection (LTE_STAGE_* bitmask, 0 = all).  Without LTE_STAGE_TX the
   * time-domain TX signal comes from in_signal; without LTE_STAGE_CHANNEL,
   * in_signal is taken as the already-received signal (no fading, no noise). */
  int32_t stages;
  /* in_signal and the real / complex captures below hold the plan's
   * arithmetic type (lte_plan_precision): float / complex64 (interleaved
   * float pairs) in f32 plans, double / complex128 in f64 plans. */
  const void *in_signal; int64_t in_signal_stride; /* [.][L] complex (stride in real elements) */
  /* captures (host, optional; used by the single-call Python API) */
  void *cap_signal_tx;         /* [n_frames][L] complex ([n_frames][num_tx][L] multi-antenna) */
  void *cap_signal_rx;         /* [n_frames][num_rx][L] complex (noisy)             */
  void *cap_data_syms;         /* [n_frames][n_sym*Nd] complex (ZF / MRC / SFBC / MMSE output;
                                  multi-antenna: n_sym*res, res = Nd&~1 SFBC, Nd spatial) */
  void *cap_H;                 /* [n_frames][num_rx][n_grp][N] complex              */
  void *cap_pilot_stats;       /* [n_frames][num_rx][n_grp][2] real (P, noise)      */
  uint8_t *cap_bits_rx;        /* [n_frames][n_bits]                                */
  void *cap_llr;               /* [n_frames][n_sym*Nd*bps] real (coded, RE order)   */
  void *cap_noise_power;       /* [n_frames][num_rx] real                           */
  void *cap_tx_syms;           /* [n_frames][n_sym*Nd] complex TX data REs          */
  /* multi-antenna injection (optional): link noise of transmit_mimo's 100 dB
   * per-link channels [.][num_rx][num_tx][2][L] unit normals; flat spatial
   * link gains [.][num_rx][num_tx][2] (re, im of h ~ CN(0,1)) */
  const double *link_noise; int64_t link_noise_stride;
  const double *link_h; int64_t link_h_stride;
  /* multi-antenna capture: per link [n_frames][num_rx][num_tx][4] = mean|x_tx|^2,
   * mean|y_link|^2, Re and Im of mean(y_link conj(x_tx)) -- the statistics
   * transmit_mimo reports its channel_matrix from (core/ofdm_core.py:505-516);
   * real, the plan's arithmetic type */
  void *cap_link_stats;
  /* beamforming capture: per frame PMI (CSIFeedback) and beamforming gain (dB);
   * cap_H holds H [n_frames][num_rx][num_tx] for this chain */
  int32_t *cap_pmi;
  double *cap_bf_gain;         /* [n_frames] beamforming gain (dB), float64 (ABI 2; float in ABI 1) */
} lte_run_args;

/* Library / device. */
const char *lte_strerror(int code);
const char *lte_last_error(void);
int lte_device_init(int device);            /* select + check gfx950 */
int lte_version(void);                     /* ABI version: LTE_ABI_VERSION (3) */
/* Call once as lte_abi_check(LTE_ABI_VERSION): LTE_OK when the loaded library
 * implements the ABI of the header the caller was compiled against, LTE_EUNSUP
 * (with lte_last_error() naming both versions) otherwise. */
int lte_abi_check(int abi_version);

/* Plans. */
int lte_plan_create(const lte_plan_desc *desc, lte_plan **out);
int lte_plan_destroy(lte_plan *plan);
/* Geometry derived by the plan: [L, n_sym, Nd, Np, n_grp, n_cb, coded_bits, n_re_bits] */
int lte_plan_info(const lte_plan *plan, int64_t *info8);
/* Arithmetic type the plan runs in: LTE_PREC_F32 or LTE_PREC_F64. */
int lte_plan_precision(const lte_plan *plan);
/* Run the full chain (TX -> channel -> RX (-> turbo)) for one batch of frames. */
int lte_run(lte_plan *plan, const lte_run_args *args);
/* Per-kernel device time accumulated by lte_run while timing is on (HIP events
 * on the plan's stream).  names: comma-separated kernel names; ms/launches per
 * kernel in the same order.  n_max entries. */
int lte_timing_enable(lte_plan *plan, int on);
int lte_timing_read(lte_plan *plan, char *names, int names_len, double *ms, int64_t *launches, int n_max);
int lte_timing_reset(lte_plan *plan);

/* ---- stage entry points (parity tests; host in/out, same device kernels) ---- */
/* IFFT*sqrt(N) / FFT/sqrt(N): core/modulator.py:242 / core/lte_receiver.py:487 */
int lte_fft_host(int N, int inverse, int64_t batch, const float *in, float *out);
int lte_fft_host64(int N, int inverse, int64_t batch, const double *in, double *out);
/* Pilots: PilotPattern.generate_pilots core/resource_mapper.py:137-152 (MT19937 seed(cell_id) + choice([1,-1])) */
int lte_pilots(int cell_id, int n, double *out_re_im);
/* The Philox mode's device random streams (the draws that replace the
 * reference's np.random.randint / rand / normal: core/rayleighchannel.py:31,
 * core/channel.py:227-228): for each frame f and counter c < n_ctr,
 * Philox4x32-10 of counter (c, stream, frame_id lo, hi), key (seed lo, hi).
 * out_u32 [n_frames][n_ctr][4] the four outputs; out_gauss64 / out_gauss32
 * [n_frames][n_ctr][4] the unit normal pairs the noise kernels form from
 * outputs (x, y) and (z, w) (float64 / float32 Box-Muller).  Any output may
 * be NULL. */
int lte_philox_host(uint64_t seed, int n_frames, const uint64_t *frame_ids, uint32_t stream, int64_t n_ctr,
                    uint32_t *out_u32, double *out_gauss64, float *out_gauss32);
/* SC-FDM DFT / IDFT of size M (<= 1024): DFTPrecodifier.precoding /
 * IDFTDecodifier.decoding core/dft_precoding.py:66-118, 199-226 (unitary,
 * 1/sqrt(M)); in / out [batch][M] complex64.  Bluestein on the device. */
int lte_dft_host(int M, int inverse, int64_t batch, const float *in, float *out);
int lte_dft_host64(int M, int inverse, int64_t batch, const double *in, double *out);
/* Soft demap: _calculate_llrs_* core/ofdm_core.py:791-923 (bps 2/4/6) */
int lte_llr_host(int bps, int64_t n, const float *syms, const float *noise_var, float *llr);
int lte_llr_host64(int bps, int64_t n, const double *syms, const double *noise_var, double *llr);
/* QAM map: QAMModulator.bits_to_symbols core/modulator.py:61-88 -- bits [n][bps]
 * (0 / 1 bytes, MSB first per symbol) -> n complex128 points of the
 * natural-binary index (level * (1 / sqrt(2 | 10 | 42)), NumPy's divide) */
int lte_qam_map_host64(int bps, int64_t n, const uint8_t *bits, double *out);
/* Channel estimation: LTEChannelEstimator.estimate_channel + _interpolate_channel
 * core/lte_receiver.py:40-133 -- for each of batch received grids Y [batch][N]
 * (complex128): LS Y[p] / X[p] at the n_pilots ascending pilot_idx (known X
 * complex128), np.linspace between consecutive pilots, edges held -> H
 * [batch][N]; pilot_ls [batch][n_pilots] the LS values (or NULL); stats
 * [batch][2] = mean |Y_p|^2, mean |Y_p - X_p|^2 (pairwise sums, or NULL) */
int lte_chest_host64(int N, int n_pilots, const int32_t *pilot_idx, const double *known, int64_t batch,
                     const double *Y, double *H, double *pilot_ls, double *stats);
/* ZF equalizer: LTEEqualizerZF.equalize core/lte_receiver.py:154-180 --
 * out = Y / (H + regularization), n complex128 (NumPy's complex divide) */
int lte_zf_host64(int64_t n, const double *Y, const double *H, double regularization, double *out);
/* Nearest point as the reference decides it: QAMModulator.symbols_to_bits
 * core/modulator.py:90-112 -- np.abs(c - y) over the constellation (NumPy's
 * complex absolute) and np.argmin (first minimum), also on exact decision
 * boundaries; n complex128 in, n * bps MSB-first bits out */
int lte_nearest_host64(int bps, int64_t n, const double *syms, uint8_t *bits);
/* Hard decision (the chains' per-axis slicer, ties -> lower level; equal to
 * lte_nearest_host64 off the decision boundaries):
 * QAMModulator.symbols_to_bits core/modulator.py:90-112 */
int lte_hard_host(int bps, int64_t n, const float *syms, uint8_t *bits);
int lte_hard_host64(int bps, int64_t n, const double *syms, uint8_t *bits);
/* RSC constituent encoder: rsc_encode core/channel_coding/turbo_encoder.py:137-211
 * -- n bits in; systematic (the feedback bit a_k) and parity out, n (+ 3
 * termination steps when termination != 0) bytes each */
int lte_rsc_encode_host(int64_t n, const uint8_t *bits, int termination, uint8_t *systematic, uint8_t *parity);
/* Turbo encode: turbo_encode core/channel_coding/turbo_encoder.py:214-313 */
int lte_turbo_encode_host(int K, int64_t ncb, const uint8_t *bits, uint8_t *out /*[ncb][3K+12]*/);
/* Turbo decode: turbo_decode core/channel_coding/turbo_decoder.py:338-450 */
int lte_turbo_decode_host(int K, int iters, int64_t ncb, const float *llr /*[ncb][3K+12]*/, uint8_t *bits);
/* One max-log BCJR pass, a-posteriori output: LogMAPDecoder.decode turbo_decoder.py:181-278 */
int lte_bcjr_host(int K, int64_t ncb, const float *ls, const float *lp, const float *la, float *app);
/* float64 turbo decode, bit-exact with turbo_decode (core/channel_coding/turbo_decoder.py:338-450):
 * the reference's unnormalised max-log recursion in its own operation order. */
int lte_turbo_decode_host64(int K, int iters, int64_t ncb, const double *llr /*[ncb][3K+12]*/, uint8_t *bits);
/* float64 single BCJR pass of any length n, a-posteriori output for every step:
 * LogMAPDecoder.decode (turbo_decoder.py:181-278) with return_extrinsic=False.
 * n = 0 is valid (nothing written), like the reference's zero-step recursion. */
int lte_bcjr_host64(int n, int64_t ncb, const double *ls, const double *lp, const double *la, double *app);
/* CRC: _calculate_crc core/channel_coding/crc.py:89-134 (MSB-first, zero init);
 * poly 0x1864CFB (CRC-24A, calculate_crc24a :137-159) or 0x1800063 (CRC-24B,
 * calculate_crc24b :162-184), len 24; any other poly with its x^len term and
 * len 1..31 (CRC-16 0x11021, calculate_crc16 :187-209) by a serial kernel */
int lte_crc_host(int64_t n, const uint8_t *bits, uint32_t poly, int len, uint32_t *crc);
/* Channel on an arbitrary-length stream: ChannelSimulator.transmit (core/channel.py:
 * 334-345) = RayleighChannel.filter (rayleighchannel.py:44-58) + measured-power
 * AWGN (channel.py:34-68, 203-234).  x [L] complex64 -> y [num_rx][L] complex64.
 * phases [num_rx][n_paths][16] (NULL -> Philox(seed)), noise [num_rx][2][L]
 * unit normals (NULL -> Philox(seed)). */
int lte_channel_host(int64_t L, int num_rx, int channel, int n_paths, const int32_t *delays, const double *gains,
                     double fD, double fs, double snr_db, uint64_t seed, const float *x, const double *phases,
                     const double *noise, float *y, float *noise_power);
/* the same in float64: x [L] complex128 -> y [num_rx][L] complex128 */
int lte_channel_host64(int64_t L, int num_rx, int channel, int n_paths, const int32_t *delays, const double *gains,
                       double fD, double fs, double snr_db, uint64_t seed, const double *x, const double *phases,
                       const double *noise, double *y, double *noise_power);
/* Multi-antenna channel on arbitrary streams.
 * mode 0: OFDMChannel.transmit_mimo (core/ofdm_core.py:434-543) -- AWGN links
 *   h = exp(j tx pi/2); Rayleigh links each a 100 dB ChannelSimulator (fading +
 *   link noise); RX noise (P_rx / num_tx) / SNR.
 * mode 1: ChannelSimulator.transmit_spatial_multiplexing (core/channel.py:
 *   397-493) -- AWGN links h ~ CN(0,1) (link_h); Rayleigh links with the given
 *   gains and fD (time-varying Jakes); RX noise P_rx / SNR.
 * x [num_tx][L] complex64 -> y [num_rx][L] complex64; link_stats (optional)
 * [num_rx][num_tx][4] = mean|x|^2, mean|y_link|^2, Re / Im mean(y_link conj(x)).
 * phases [num_rx][num_tx][n_paths][16], link_noise [num_rx][num_tx][2][L],
 * link_h [num_rx][num_tx][2], noise [num_rx][2][L]: NULL -> Philox(seed). */
int lte_channel_mimo_host(int64_t L, int num_tx, int num_rx, int mode, int channel, int n_paths,
                          const int32_t *delays, const double *gains, double fD, double fs, double snr_db,
                          uint64_t seed, const float *x, const double *phases, const double *link_noise,
                          const double *link_h, const double *noise, float *y, float *link_stats,
                          float *noise_power);
/* the same in float64 (complex128 streams; fD != 0 evaluates the Jakes sum of
 * rayleighchannel.py:20-42 exactly per sample instead of the float32 path's
 * per-symbol expansion) */
int lte_channel_mimo_host64(int64_t L, int num_tx, int num_rx, int mode, int channel, int n_paths,
                            const int32_t *delays, const double *gains, double fD, double fs, double snr_db,
                            uint64_t seed, const double *x, const double *phases, const double *link_noise,
                            const double *link_h, const double *noise, double *y, double *link_stats,
                            double *noise_power);
/* TM4 detection: MIMODetector.detect (core/mimo_detector.py:55-369) per
 * subcarrier, float64 on the device.  y [num_rx][n_sc] complex128, H
 * [num_rx][num_tx][n_sc] complex128, W [num_tx][rank] complex128 (row-major),
 * detector LTE_DET_*; bps 2/4/6 is SIC's constellation (0: none -> SIC uses
 * MMSE, :225-228) -> out [rank][n_sc] complex128.  num_rx, num_tx <= 4. */
int lte_mimo_detect_host(int detector, int num_rx, int num_tx, int rank, int bps, int64_t n_sc, const double *y,
                         const double *H, const double *W, double sigma2, double *out);
/* SFBC Alamouti on host arrays, float64 [n] complex128 (interleaved re, im),
 * n even (LTE_EINVAL with the reference's ValueError text otherwise; n = 0
 * writes nothing).  encode: SFBCAlamouti.encode (core/sfbc_alamouti.py:45-78),
 * per pair TX0 [s0, -conj(s1)], TX1 [s1, conj(s0)].  decode:
 * SFBCAlamouti.decode (:80-163) with per-subcarrier estimates H0 / H1 and the
 * caller's regularization (the reference's default 1e-10) -- the combiner the
 * chains' SFBC detector runs. */
int lte_sfbc_encode_host64(int64_t n, const double *syms, double *tx0, double *tx1);
int lte_sfbc_decode_host64(int64_t n, const double *rx, const double *H0, const double *H1, double regularization,
                           double *out);
/* Rate dematching map: rate_dematching_turbo core/channel_coding/rate_matching.py:374-489
 * src[j] = index into the E rate-matched LLRs feeding output j of [3K+12], -1 = zero. */
int lte_rate_dematch_map(int K, int E, int rv_idx, int32_t *src);
/* rate_dematching_turbo (core/channel_coding/rate_matching.py:374-489) for any
 * E, on the device: llr [ncb][E] float64 -> out [ncb][3K+12]; punctured
 * positions 0.0, repeats (E > N_cb) summed in order onto 0.0 (:433-436).
 * E = 0 (all punctured) writes zeros without a launch, as the reference returns. */
int lte_rate_dematch_host64(int K, int E, int rv_idx, int64_t ncb, const double *llr, double *out);
/* QPP interleaver pi(i) = (f1 i + f2 i^2) mod K: qpp_interleave
 * core/channel_coding/turbo_encoder.py:76-103 (out[i] = in[perm[i]]). */
int lte_qpp_perm(int K, int32_t *perm);
/* Sub-block interleaver index map (32 columns, <NULL>s removed):
 * sub_block_interleaver core/channel_coding/rate_matching.py:25-94 (out[i] = in[perm[i]]). */
int lte_subblock_perm(int n, int32_t *perm);
/* set_decoder_mode (core/channel_coding/turbo_decoder.py:35-54): 1 = max-log-MAP
 * (the reference default), 0 = exact log-MAP (log_sum_exp max*, :64-88) for
 * every float64 decode (entry points and f64 plans); float32 decoders refuse
 * exact log-MAP with LTE_EUNSUP. */
int lte_set_decoder_mode(int use_max_log_map);

#ifdef __cplusplus
}
#endif
#endif /* LTE_PHY_H */
