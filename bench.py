"""Headline benchmark: LTE subframes/s through the full coded chain
(config 2: 20 MHz, 64-QAM, Rayleigh ITU Pedestrian-A, turbo max-log-MAP x8,
TB 27 760 bits = 5 code blocks = 14 OFDM symbols), BER sweep SNR 0:2:30 dB,
in float64 (the reference's arithmetic; `--precision f32` is the fast mode).
`--config 3|4|5` runs BASELINE.json's other GPU configs through the same
harness (config 5 is the one BASELINE names for the 8-GPU sharded grid).

One step = one batch of `--frames` subframes per GPU pushed TX -> channel ->
RX (+ turbo); all inputs (Philox bits / fading / noise) are generated on the
device.  N>1: one process per GPU (torch.distributed, RCCL); frames are
partitioned by global frame id (weak scaling, no data-path collective); the
only collectives are the SUM of the BER counters and the MAX of the step time.

BER match: the `cpu_baseline` leg runs the float64 oracle on the bench's own
frames -- frame ids from both ends of rank 0's first timed step, with the
oracle's restatement of the device's Philox draws (oracle/philox.py) -- and
after the timed region rank 0 runs the same frame ids through the same plan:
`ber_match` reports how many frames agree bit for bit and the largest BER gap
over the sample's SNR points.

`python bench.py --gpus N` with no launcher environment starts N ranks itself
(torch.distributed.run on 127.0.0.1, before anything touches the GPU) and
exits with their status; under a launcher WORLD_SIZE must equal --gpus.

usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5] [--frames F]
                       [--precision f64|f32] [--velocity KMH] [--channel awgn|rayleigh_mp]
"""
import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, 'ofdm-lte_amd')):
    if p not in sys.path:
        sys.path.insert(0, p)

METRIC = "LTE subframes/sec (20 MHz, 64-QAM, Rayleigh+turbo) at 1/2/4/8 GPU; BER match"
SNRS = np.arange(0, 31, 2, dtype=np.float64)
SEED = 0x5EED
TB = 27760
HBM_PEAK_GBS = 8000.0
CPU_PER_GPU = 16     # host cores per GPU on the box (its CPU share)
# compulsory stage-boundary bytes of one config-2 coded subframe
# (TX map+IFFT, channel, FFT, estimation/equalisation/LLR, dematch+decode, CRC),
# quoted for 4-B reals; the f64 chain moves 8-B reals at the same boundaries
B_SF_F32 = 2_116_904
# Non-packed vector ALU peaks of one MI355X (add / max, 1 op per lane per
# instruction; 256 CUs x 4 SIMD-32 x 2.4 GHz):
#  * f32: a wave64 instruction every 2 cycles per SIMD with several waves
#    resident (MI355X_MICROARCH.md: SIMD-32, 2 cycles per wave64 VALU op)
#    = 32 lane-ops/cycle/SIMD -> 78.6 T op/s (half the 157.3 TFLOPS FMA spec)
#  * f64: 16 lane-ops/cycle/SIMD (the 78.6 TFLOPS f64 vector FMA spec / 2)
#    -> 39.3 T op/s; scripts/valu_peak_bench.hip measures both on the box
VALU_PEAK_OPS = {'f32': 256 * 4 * 32 * 2.4e9, 'f64': 256 * 4 * 16 * 2.4e9}

# BASELINE.json's GPU configs: the workload, the default batch per GPU (sized to
# the 288 GB of HBM and to fill the decoder's 1 024 resident waves several
# times over), and the per-frame payload
WORKLOADS = {
    2: {'short': '20 MHz, 64-QAM, Rayleigh+turbo', 'frames': 65536, 'coded': True, 'n_bits': TB,
        'desc': 'config 2: SISO 20 MHz (N=2048) 64-QAM, Rayleigh ITU Pedestrian-A, turbo max-log-MAP 8 it., '
                'TB 27760 (5 CBs, 14 OFDM symbols), SNR 0:2:30 dB'},
    3: {'short': 'config 3: SIMO 1x4 MRC, 10 MHz, 16-QAM, Rayleigh VehA', 'frames': 65536, 'coded': False,
        'n_bits': 14 * 499 * 4,
        'desc': 'config 3: SIMO 1x4 MRC, 10 MHz (N=1024) 16-QAM, Rayleigh ITU Vehicular-A per RX antenna, '
                '14 OFDM symbols (27944 bits) uncoded, SNR 0:2:30 dB'},
    4: {'short': 'config 4: SFBC 2x2 + turbo, 20 MHz, 64-QAM, Rayleigh', 'frames': 65536, 'coded': True,
        'n_bits': TB,
        'desc': 'config 4: Tx diversity 2x2 Alamouti SFBC + turbo max-log-MAP 8 it., 20 MHz 64-QAM, Rayleigh ITU '
                'Pedestrian-A per link (transmit_mimo), TB 27760, SNR 0:2:30 dB'},
    5: {'short': 'config 5: spatial 4x4 MMSE, 20 MHz, 64-QAM', 'frames': 32768, 'coded': False,
        'n_bits': 14 * 999 * 6,
        'desc': 'config 5: spatial multiplexing 4x4, rank 4, TM4 PMI 0 (W = I4), MMSE, 20 MHz 64-QAM, '
                '14 OFDM symbols (83916 bits) uncoded, SNR 0:2:30 dB'},
}


def _cpu_worker(job):
    """One host core: the float64 oracle on the bench's own frames (its
    restatement of the device's Philox draws), frame after frame from `ids`,
    for `seconds`; returns ([(id, bit_errors, crc_ok)], elapsed)."""
    config, seconds, ids, channel = job
    from oracle import lte_oracle as O, philox as P
    O.lib()
    f = P.BENCH_FRAMES[config]
    kw = {'channel': channel} if config == 5 and channel else {}
    res, t0 = [], time.perf_counter()
    for i in ids:
        e, c = f(int(i), **kw)
        res.append((int(i), e, c))
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return res, time.perf_counter() - t0


def _cpu_model():
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or 'unknown'


def sample_ids(F, procs):
    """Frame ids of rank 0's first timed step ([0, F)) taken alternately from
    both ends, dealt round-robin to the workers."""
    h = (F + 1) // 2
    order = np.empty(2 * h, dtype=np.int64)
    order[0::2] = np.arange(h)
    order[1::2] = F - 1 - np.arange(h)
    order = order[:F]
    return [order[i::procs].tolist() for i in range(procs)]


def _cpu_pool(config, F, seconds, procs, channel):
    """`procs` single-threaded oracle worker processes on the bench's frames for
    `seconds`: (frames/s summed over workers, [(id, errors, crc)], wall s)."""
    import multiprocessing as mp
    jobs = [(config, seconds, ids, channel) for ids in sample_ids(F, procs)]
    # close() + join(), not the context manager's terminate(): the workers exit
    # on their own (under rocprofv3 a terminate() leaves SIGTERM stack dumps)
    pool = mp.get_context('spawn').Pool(procs)
    try:
        res = pool.map(_cpu_worker, jobs)
        pool.close()
    except BaseException:
        pool.terminate()
        raise
    finally:
        pool.join()
    value = sum(len(r[0]) / r[1] for r in res)
    frames = sorted(x for r in res for x in r[0])
    return value, frames, max(r[1] for r in res)


def cpu_baseline(config=2, F=65536, seconds=15.0, procs=None, channel=None, single_seconds=None):
    """Time the oracle (float64 CPU restatement: NumPy front end + C turbo
    decoder, bit-exact with the reference) on this host's cores on a bounded
    sample of the bench's own frames, as BASELINE.md's CPU timing asks: one
    single-threaded worker process per core (frames are independent) over the
    box's CPU share (16 cores per GPU: `value`, `gpu_share`), and one process
    alone (`single_process`, `single_seconds`, default 8 s; 0 skips it).
    `all_cores` is the per-core rate x the host's CPUs, an extrapolation: the
    pool's rules size worker pools to the CPU share, not the whole machine
    (scripts/cpu_baseline_scaling.py measures 1 .. all cores where that is
    allowed; profiles/r6_cpu_baseline_scaling.json).  Runs before the GPU is
    initialised (spawned processes).  The per-frame results feed `ber_match`."""
    procs = procs or max(1, min(CPU_PER_GPU, os.cpu_count() or 1))
    for v in ('OMP_NUM_THREADS', 'OPENBLAS_NUM_THREADS', 'MKL_NUM_THREADS'):
        os.environ[v] = '1'
    value, frames, wall = _cpu_pool(config, F, seconds, procs, channel)
    n = len(frames)
    single_seconds = min(8.0, seconds) if single_seconds is None else single_seconds
    single = None
    if single_seconds > 0:
        v1, f1, w1 = _cpu_pool(config, F, single_seconds, 1, channel)
        single = {'value': v1, 'cores': 1, 'frames': len(f1), 'seconds': round(w1, 1)}
    host = os.cpu_count() or procs
    per_core = value / procs
    return {'value': value, 'unit': 'subframes/s', 'cores': procs, 'kind': 'port', 'host_cores': host,
            'per_core': per_core, 'cpu_model': _cpu_model(),
            'gpu_share': {'value': value, 'cores': procs, 'frames': n, 'seconds': round(wall, 1)},
            'single_process': single,
            'all_cores': {'value': per_core * host, 'cores': host, 'measured': False,
                          'what': 'per-core rate of the gpu_share pool x the host CPUs (linear: the frames are '
                                  'independent); not run here -- worker pools on the box are sized to its CPU '
                                  'share. Measured 1 .. all cores of another host: '
                                  'profiles/r6_cpu_baseline_scaling.json'},
            'sample': f'{n} of the bench\'s own config-{config} frames (ids from both ends of rank 0\'s first '
                      f'timed step, the oracle\'s restatement of the device Philox draws) over SNR 0:2:30 dB, '
                      f'{wall:.1f} s on {procs} host cores, one single-threaded process each '
                      f'(oracle: NumPy + C, float64)' +
                      (f'; single process: {single["frames"]} frames in {single["seconds"]} s' if single else ''),
            'frames': frames}


def ber_match(plan, cpu, coded):
    """Rank 0, after the timed region: the oracle's sample frames through the
    bench's own plan (same seed, SNR by frame id); per-frame equality and the
    largest |BER_gpu - BER_oracle| over the SNR points of the sample."""
    fr = cpu.get('frames') if cpu else None
    if not fr:
        return None
    ids = np.array([f[0] for f in fr], dtype=np.uint64)
    e_or = np.array([f[1] for f in fr], dtype=np.int64)
    S = len(SNRS)
    e_gpu = np.zeros(len(ids), dtype=np.int64)
    c_gpu = np.zeros(len(ids), dtype=bool)
    for i in range(0, len(ids), plan.max_frames):
        chunk = ids[i:i + plan.max_frames]
        si = (chunk % np.uint64(S)).astype(np.int32)
        out = plan.run(SNRS[si], snr_index=si, n_snr=S, seed=SEED, frame_ids=chunk)
        e_gpu[i:i + len(chunk)] = out['frame_errors']
        if coded:
            c_gpu[i:i + len(chunk)] = out['crc_ok'].astype(bool)
    si = (ids % np.uint64(S)).astype(np.int64)
    nb = WORKLOADS[cpu['config']]['n_bits']
    dber = 0.0
    per = {}
    for s in np.unique(si):
        m = si == s
        d = abs(e_gpu[m].sum() - e_or[m].sum()) / (m.sum() * nb)
        per[f'{SNRS[s]:g}'] = int(m.sum())
        dber = max(dber, float(d))
    out = {'frames': int(len(ids)), 'frames_identical': int(np.sum(e_gpu == e_or)),
           'max_abs_dber': dber, 'frames_per_snr_db': per,
           'what': 'the oracle (float64, cpu_baseline leg) and the GPU plan on the same bench frame ids: per-frame '
                   'bit-error equality and max over SNR points of |BER_gpu - BER_oracle| on the sample'}
    if coded:
        c_or = np.array([bool(f[2]) for f in fr])
        out['crc_identical'] = int(np.sum(c_gpu == c_or))
    return out


def load_profile(name):
    """A committed rocprofv3 --pmc summary (profiles/<name>), or None."""
    p = os.path.join(ROOT, 'profiles', name)
    if os.path.exists(p):
        try:
            return json.load(open(p))
        except Exception:
            return None
    return None


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv):
    """--gpus N without a launcher: time the CPU baseline here (this process
    never touches the GPU; 16 host cores per GPU of the node), then run N ranks
    under torch.distributed.run as a child process and return its status.
    Rank 0 reads the baseline from LTE_BENCH_CPU_JSON (a file path), so the
    N > 1 line carries it too."""
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    if cpu_seconds(args) > 0:
        procs = max(1, min(CPU_PER_GPU * args.gpus, os.cpu_count() or 1))
        cpu = cpu_baseline(args.config, args.frames, cpu_seconds(args), procs, args.channel)
        cpu['config'] = args.config
        path = os.path.join(os.environ.get('TMPDIR', '/tmp'), f'lte_bench_cpu_{os.getpid()}.json')
        with open(path, 'w') as f:
            json.dump(cpu, f)
        env['LTE_BENCH_CPU_JSON'] = path
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={args.gpus}',
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), os.path.abspath(__file__)] + argv
    rc = subprocess.call(cmd, env=env)
    if env.get('LTE_BENCH_CPU_JSON'):
        try:
            os.remove(env['LTE_BENCH_CPU_JSON'])
        except OSError:
            pass
    return rc


def cpu_seconds(args):
    """--cpu-seconds, or 15 s (0 under --dry-run unless given)."""
    if args.no_cpu:
        return 0.0
    if args.cpu_seconds is not None:
        return float(args.cpu_seconds)
    return 0.0 if args.dry_run else 15.0


def decoder_row_bytes(K, esz, iters):
    """Compulsory HBM bytes of one code block through the exact lane-per-code-
    block decoder (k_turbo64 / k_turbo): a step of the unnormalised
    recursion needs the three rows (Ls, Lp, La) of its step in the forward
    sweep and again in the backward sweep (beta at k depends on every input
    after k, the LLR on alpha and beta; a code block's working set cannot stay
    on chip), plus the extrinsic store: 7 rows of esz bytes per step and pass.
    The first pass has no a priori (5 rows), the final a-posteriori pass stores
    packed decisions instead of an extrinsic (6 rows + K/8 B).  The two tail
    rows (Ls, Lp) of the 3 termination steps are read once per pass.  The alpha
    checkpoint rows are NOT counted: they are this implementation's choice (its
    measured traffic shows them)."""
    passes = 2 * iters + 1
    rows = 5 + (passes - 2) * 7 + 6 if iters >= 1 else 6
    return K * rows * esz + 3 * 2 * passes * esz + K / 8


def shape_bytes(K, iters=8):
    """(all bytes, store bytes) one 64-frame wave of the decoder's access-shape
    microbenchmark moves for a code block of K (scripts/turbo_shape_bench.hip
    wave_bytes: 512-B rows; forward + backward row loads, tails, extrinsic
    stores, checkpoint stores and loads)."""
    nsub = K // 8
    nsw = (nsub + 2) // 3
    rows = stores = 0
    for p in range(2 * iters + 1):
        per = 2 if p == 0 else 3
        rows += per * K * 2 + 6 + K + ((nsub + 2) // 3) * 8 + nsw * 8
        stores += K + ((nsub + 2) // 3) * 8
    return rows * 512, stores * 512


def shape_store_share(iters=8):
    """Share of the decoder shape's bytes that are stores (extrinsic +
    checkpoint rows), from the shape bench's own byte counts."""
    from lte_phy.channel_coding import segmentation_sizes
    tot = [shape_bytes(K, iters) for K in segmentation_sizes(TB + 24)]
    return sum(t[1] for t in tot) / sum(t[0] for t in tot)


def turbo_roofline(prec, tim, F, iters=8):
    """Turbo decoder (the dominant kernel of configs 2 and 4).  `bound` is the
    measured limiter: the exact lane-per-code-block recursion streams its rows
    through HBM (a code block's working set cannot stay on chip), so
    achieved / peak / frac price the compulsory row stream of that algorithm
    (decoder_row_bytes per launch / the mean launch time) against 8 TB/s, and
    `traffic` is the PMC-measured HBM bytes per launch (hbm_frac = its rate /
    8 TB/s).  Beside it SURVEY §8(d)'s K7 figure, `valu_frac`: sum(K+3) x 17
    passes x ~100 add/max ops per subframe against the non-packed f64 (f32)
    vector peak, and the SQ-counted VALU issue occupancy."""
    from lte_phy.channel_coding import segmentation_sizes
    t_ms, t_n = tim.get('turbo', (0.0, 0))
    avg_s = t_ms / max(t_n, 1) * 1e-3
    Fp = ((F + 63) // 64) * 64            # frames padded to whole 64-frame decoder groups
    esz = 8 if prec == 'f64' else 4
    Ks = segmentation_sizes(TB + 24)
    ops_sf = sum(K + 3 for K in Ks) * (2 * iters + 1) * 100
    row_bytes = sum(Fp * decoder_row_bytes(K, esz, iters) for K in Ks)
    stage_bytes = sum(Fp * ((3 * K + 12) * esz + K / 8) for K in Ks)
    peak = VALU_PEAK_OPS[prec]
    achieved_T = ops_sf * F / avg_s / 1e12 if t_n else 0.0
    traffic = load_profile(f'pmc_turbo_traffic_{prec}.json')
    sq = load_profile(f'pmc_turbo_sq_{prec}.json')
    shape = load_profile('r3_turbo_shape_microbench.json')
    gbs = row_bytes / avg_s / 1e9 if t_n else 0.0
    tr = traffic['bytes_per_frame'] * Fp if traffic else None
    tr_gbs = tr / avg_s / 1e9 if tr and t_n else None
    busy = (sq['valu_wave_instr_per_frame'] * Fp * sq['issue_cycles_per_instr'] / (avg_s * 2.4e9 * 1024)
            if sq and t_n else None)
    ceil = shape.get(f'ceiling_GBs_{prec}') if shape else None
    limiter = 'hbm' if busy is None or (tr_gbs or gbs) / HBM_PEAK_GBS >= busy else 'valu'
    valu_frac = round(achieved_T * 1e12 / peak, 4) if t_n else 0.0
    if limiter == 'hbm':
        head = {'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                'frac': round(gbs / HBM_PEAK_GBS, 4) if t_n else 0.0}
        what = ('compulsory row stream of the exact recursion (decoder_row_bytes: per code-block step 7 rows of '
                f'{esz} B -- Ls, Lp, La forward and backward + the extrinsic store -- over 2 it. + 1 passes) x '
                'frames / mean launch time, against 8 TB/s; traffic = PMC-measured HBM bytes per launch '
                '(gfx950-corrected)')
    else:
        head = {'achieved': round(achieved_T, 3), 'peak': round(peak / 1e12, 2), 'unit': 'Top/s', 'frac': valu_frac}
        what = (f'SURVEY §8(d) K7: sum(K+3) x (2 it. + 1) passes x 100 add/max ops per subframe ({ops_sf} op) x '
                f'frames / mean launch time, against the non-packed {prec} vector peak')
    out = {'bound': limiter, 'kernel': 'k_turbo64' if prec == 'f64' else 'k_turbo'}
    out.update(head)
    out.update({
        'traffic': round(tr) if tr else None,
        'hbm_frac': round(tr_gbs / HBM_PEAK_GBS, 4) if tr_gbs else None,
        'valu_frac': valu_frac,
        'what': what,
        'bound_basis': 'bound = the measured limiter: the PMC traffic rate as a share of 8 TB/s (hbm_frac) against '
                       'the SQ-counted VALU issue occupancy (issued_valu_busy_frac), whichever is higher.  SURVEY '
                       "§8(d) names VALU as K7's roofline; that figure is valu_frac (the reference recursion has "
                       '103 add/max per trellis step and pass -- gamma 6, alpha 24, beta 24, a-posteriori 47, '
                       'extrinsic 2 -- which §8(d) rounds to 100)',
        'valu': {'achieved': round(achieved_T, 3), 'peak': round(peak / 1e12, 2), 'unit': 'Top/s',
                 'frac': valu_frac, 'ops_per_subframe': ops_sf,
                 'what': f'SURVEY §8(d) K7: sum(K+3) x (2 it. + 1) passes x 100 add/max ops per subframe x frames / '
                         f'mean launch time, against the non-packed {prec} vector peak'},
        'ops_per_subframe': ops_sf,
        'avg_launch_ms': round(avg_s * 1e3, 3), 'launches': t_n, 'frames_per_launch': F,
        'issued_valu_busy_frac': round(busy, 4) if busy is not None else None,
        'valu_wave_instr_per_frame': sq['valu_wave_instr_per_frame'] if sq else None,
        'measured_limiter': limiter,
        'hbm_row_stream': {
            'achieved_GBs': round(gbs, 1), 'peak_GBs': HBM_PEAK_GBS,
            'frac_row_stream': round(gbs / HBM_PEAK_GBS, 4),
            'alg_bytes_per_launch': int(row_bytes),
            'alg_bytes': 'exact-recursion row stream: per code-block step 7 rows (Ls, Lp, La forward and '
                         'backward + extrinsic store) x esz B x 17 passes (first pass 5, final 6 + K/8 B decisions)',
            'traffic_over_alg': round(tr / row_bytes, 3) if tr else None,
            'traffic_GBs': round(tr_gbs, 1) if tr_gbs else None,
            'traffic_frac': round(tr_gbs / HBM_PEAK_GBS, 4) if tr_gbs else None,
            'shape_ceiling': ({'GBs': ceil, 'traffic_frac_of_ceiling': round(tr_gbs / ceil, 4) if tr_gbs else None,
                               'source': 'profiles/r3_turbo_shape_microbench.json (another box: +-5 %)'}
                              if ceil else None),
            # the decoder's access shape with and without its stores (extrinsic +
            # checkpoint rows): a STORED reference time from round 3, replaced by
            # this box's own measurement when the shape bench runs after the timed
            # region (same_box_shape_ceiling); the byte share is the shape's own count
            'store_cost': {'shape_ms_full': 319.5, 'shape_ms_reads_only': 237.4,
                           'store_share_of_time': round(1 - 237.4 / 319.5, 3),
                           'store_share_of_bytes': round(shape_store_share(iters), 4),
                           'measured_in_this_run': False,
                           'source': 'stored: profiles/r3_turbo_shape_layouts.jsonl run shape4, variants aux3 / '
                                     'a3nost, CH 32 (65 536 frames), another box; byte share: shape_bytes'}},
        'stage_bytes': {'bytes_per_launch': int(stage_bytes),
                        'achieved_GBs': round(stage_bytes / avg_s / 1e9, 2) if t_n else 0.0,
                        'frac': round(stage_bytes / avg_s / 1e9 / HBM_PEAK_GBS, 5) if t_n else 0.0,
                        'what': 'SURVEY §8(d) stage boundary: rate-dematched input LLRs + decoded bits'}})
    return out


def stage_bytes_per_frame(config, plan, prec):
    """Algorithmic HBM bytes per frame of each timed stage of the bench's
    default path (the kernels lte_run launches for it with every LTE_* knob at
    its default), from the streams those kernels must read and write
    (complex = 2 x esz B, packed bits).  Stage -> (kernels, bytes, what); the
    kernel names are the keys of the committed PMC summaries (PMC_FILES), so
    each stage's measured traffic sits beside its algorithmic bytes.
    * The fused transmitters (configs 2/3: static taps; configs 4/5) write the
      received streams without their CP samples where the receiver never reads
      them (SISO / SIMO: k_chan_fix rebuilds the stream's first samples);
      configs 4/5 keep the CP (the link power is measured over it).
    * The receivers read n_sym x N samples per RX (the CP is stripped).
    * Config 5 (spatial, no H capture): k_rx_fft_mimo(_w) hands the detector the
      LS pilot estimates, nr x n_est x nt x pilots-per-TX (LTE_SPATIAL_HP),
      not the interpolated H.
    * Flat links (config 5 'awgn'): TX and links are one pass
      (k_ofdm_txch_flat); the 'channel' timer then covers only k_npow_mimo's
      per-RX power (partials in, one noise power out)."""
    esz = 8 if prec == 'f64' else 4
    c = 2 * esz
    L, n_sym, bits = plan.L, plan.n_sym, plan.n_bits / 8
    N, nr = plan.N, plan.num_rx
    sym = n_sym * N * c                       # one antenna's symbols without CP
    rows = 0
    if config in (2, 4):                      # decoder rows: 3K + 12 per code block
        from lte_phy.channel_coding import segmentation_sizes
        rows = sum(3 * K + 12 for K in segmentation_sizes(plan.n_bits + 24))
    if config in (2, 3):
        # config 3, float64: the wave-private TX (k_ofdm_tx_simo_w, the default; LTE_SIMO_TX_WAVE=0: k_ofdm_tx)
        simo_tw = prec == 'f64' and N == 1024 and os.environ.get('LTE_SIMO_TX_WAVE', '1') != '0'
        ctx = {2: 'k_ofdm_txf', 3: 'k_ofdm_tx_simo_w' if simo_tw else 'k_ofdm_tx'}[config]
        # config 3, float64: the wave-private receiver (k_rx_frame_simo_w, the default; LTE_SIMO_RX_WAVE=0 the
        # block kernel k_rx_frame_simo2)
        simo_w = prec == 'f64' and N == 1024 and os.environ.get('LTE_SIMO_RX_WAVE', '1') != '0'
        crx = {2: 'k_rx_frame', 3: 'k_rx_frame_simo_w' if simo_w else 'k_rx_frame_simo2'}[config]
        tx_in = plan.coded_bits / 8 if config == 2 else bits
        out = {'ofdm_tx': ([ctx], tx_in + nr * sym, 'payload / coded bits in, each RX stream (no CP) out'),
               'rx_data': ([crx], nr * sym + (0 if config == 2 else bits),
                           'each RX stream (no CP) in' + (', payload bits in for the error count' if config == 3
                                                           else ''))}
        if plan.channel == 1:   # static taps: coefficients, then the first-samples power fix-up + noise power
            D, P = plan.max_delay, plan.n_paths
            out['fading'] = (['k_fading'], nr * P * c, 'one tap coefficient per (RX, path) out')
            if config == 3 and simo_tw:   # the wave TX forms the head samples' power itself (k_chan_fix skipped)
                out['channel'] = (['k_npow'], nr * n_sym * esz + nr * esz,
                                  'the power partials in, the noise power out')
            else:
                out['channel'] = (['k_chan_fix', 'k_npow'], n_sym * 2 * D * c + nr * P * c + 3 * nr * n_sym * esz,
                                  "each symbol's head / previous tail (2 x max delay) and the taps in, the power "
                                  'partials updated, the noise power out')
        if config == 2:   # equalised symbols + sigma^2_eff per (group, data SC) to k_dematch_zn
            out['rx_data'] = ([crx], nr * sym + n_sym * plan.Nd * c + plan.n_grp * plan.Nd * esz,
                              'the RX stream (no CP) in; equalised symbols + sigma^2_eff per data SC out')
            out['dematch'] = (['k_dematch_zn'], n_sym * plan.Nd * c + plan.n_grp * plan.Nd * esz + rows * esz,
                              'symbols + sigma^2_eff in, the decoder rows (3K + 12 per CB) out')
        return out
    nt = plan.num_tx
    stream = L * c                            # one antenna's stream with CP
    if config == 4:
        res = plan.res
        # the merged link noise (default: LTE_SFBC_LINK_MERGE) folds the link noise into the receiver's draw:
        # the 'channel' stage is then the per-RX noise powers from the TX's power partials
        merged = os.environ.get('LTE_SFBC_LINK_MERGE', '1') != '0'
        chan = ((['k_npow_sfbc_merged'], 2 * nr * esz + nr * esz + esz,
                 'per RX the links\' and the stream\'s power partials and the SNR in, the noise power out') if merged else
                (['k_link_noise_pairs'], 2 * nr * stream, 'each RX stream in and out (+ link noise)'))
        return {'ofdm_tx': (['k_ofdm_txch_sfbc'], plan.coded_bits / 8 + nr * stream,
                            'coded bits in, each RX antenna\'s faded stream (with CP) out'),
                'channel': chan,
                'rx_chest': (['k_rx_sfbc'], nr * sym + n_sym * res * c + n_sym * (res // 2) * esz,
                             'each RX stream (no CP) in; combined symbols + sigma^2_eff per RE pair out'),
                'dematch': (['k_dematch_zn'], n_sym * res * c + n_sym * (res // 2) * esz + rows * esz,
                            'symbols + sigma^2_eff in, the decoder rows out')}
    y = n_sym * nr * plan.n_dsc * c           # data-SC values per RX and symbol
    hp = nr * plan.n_est * nt * plan.pilots_per_tx * c   # LS pilot estimates
    flat = plan.channel == 0
    # float64: the wave-private receiver (k_rx_fft_mimo_w, the default; LTE_MIMO_RX_WAVE=0 the block kernel)
    wave = prec == 'f64' and plan.N == 2048 and os.environ.get('LTE_MIMO_RX_WAVE', '1') != '0'
    out = {'rx_chest': (['k_rx_fft_mimo_w' if wave else 'k_rx_fft_mimo'], nr * sym + y + hp,
                        'each RX stream (no CP) in; data-SC values + LS pilot estimates out'),
           'rx_data': (['k_det_spatial'], y + hp + bits, 'data-SC values + pilot estimates + payload bits in')}
    if flat:
        out['ofdm_tx'] = (['k_ofdm_txch_flat'], bits + nr * stream, 'payload bits in, each RX stream (with CP) out')
        out['fading'] = (['k_fading_mimo'], nr * nt * c, 'the flat link gains out')
        out['channel'] = (['k_npow_mimo'], nr * (n_sym + 1) * esz, 'per-symbol power partials in, noise power out')
    else:
        out['ofdm_tx'] = (['k_ofdm_tx_mimo'], bits + nt * stream, 'payload bits in, each TX stream (with CP) out')
        out['channel'] = (['k_channel_tay', 'k_npow_mimo'], (nt + nr) * stream,
                          'each TX stream in, each RX stream out')
    return out


# the committed rocprofv3 --pmc summary of each config's bench step (the
# traffic beside each stage's algorithmic bytes; tests/test_roofline_pmc.py)
PMC_FILES = {2: 'r5_pmc_c2_final.json', 3: 'r6_pmc_c3_wave4.json', 4: 'r6_pmc_c4_merged.json',
             5: 'r6_pmc_c5.json'}


def pmc_stage_bytes(pmc, kernels):
    """HBM bytes per frame of a stage's kernels in a PMC summary (the instance
    '<name><template args>' that ran, the longest if several): None when the
    first (main) kernel is absent; a later helper kernel the summary does not
    list (k_npow: a few hundred bytes) counts 0."""
    if not pmc:
        return None
    ks = pmc['kernels']
    tot = 0.0
    for i, name in enumerate(kernels):
        hits = [v for k, v in ks.items() if k == name or k.startswith(name + '<')]
        if not hits:
            if i == 0:
                return None
            continue
        tot += max(hits, key=lambda v: v.get('ms', 0))['hbm_bytes_per_frame']
    return tot


def stage_table(config, plan, prec, tim, F, steps):
    """Every timed stage that has an algorithmic byte count: its kernels, its
    algorithmic bytes per frame, the committed PMC bytes per frame of the same
    kernels (PMC_FILES) and both rates against the 8 TB/s peak."""
    sb = stage_bytes_per_frame(config, plan, prec)
    pmc = load_profile(PMC_FILES[config]) if prec == 'f64' else None
    out = {}
    for k, (ms, n) in tim.items():
        if k not in sb or not n:
            continue
        kern, b, what = sb[k]
        st_s = ms / steps * 1e-3
        gbs = b * F / st_s / 1e9
        tb = pmc_stage_bytes(pmc, kern)
        out[k] = {'kernels': kern, 'ms_per_step': round(st_s * 1e3, 3), 'alg_bytes_per_frame': round(b),
                  'alg_GBs': round(gbs, 1), 'frac': round(gbs / HBM_PEAK_GBS, 4), 'what': what,
                  'pmc_bytes_per_frame': round(tb) if tb else None,
                  'traffic_GBs': round(tb * F / st_s / 1e9, 1) if tb else None,
                  'traffic_frac': round(tb * F / st_s / 1e9 / HBM_PEAK_GBS, 4) if tb else None}
    return out


def hbm_roofline(config, plan, prec, tim, F, steps):
    """Uncoded configs: the dominant timed stage against the HBM roofline --
    its algorithmic bytes per frame x frames / its time per step (HIP events
    on the plan stream), the committed PMC bytes of the same kernels as
    `traffic`, every other stage beside it (stage_table)."""
    st = stage_table(config, plan, prec, tim, F, steps)
    if not st:
        return None
    dom = max(st, key=lambda k: st[k]['ms_per_step'])
    d = st[dom]
    tb = d['pmc_bytes_per_frame']
    # the dominant kernel's SQ counters from the same PMC summary: with HBM well
    # under its peak, these say where the rest of the time goes
    sq = None
    pmc = load_profile(PMC_FILES[config]) if prec == 'f64' else None
    if pmc:
        hits = [v for k, v in pmc['kernels'].items() if k == d['kernels'][0] or k.startswith(d['kernels'][0] + '<')]
        if hits:
            h = max(hits, key=lambda v: v.get('ms', 0))
            sq = {'valu_wave_instr_per_frame': h.get('valu_wave_instr_per_frame'),
                  'wave_cycles': h.get('wave_cycles'), 'share_of_active_issue': h.get('share_of_active_issue'),
                  'what': 'SQ counters of the dominant kernel (fractions of wave cycles: active issue, waiting); '
                          'HBM far under 8 TB/s with VALU most of the issue and waits the rest means latency-bound '
                          'f64 VALU work (the Box-Muller noise), DESIGN.md section 5'}
    return {'bound': 'hbm', 'kernel': ' + '.join(d['kernels']), 'stage': dom, 'achieved': d['alg_GBs'],
            'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': d['frac'],
            'traffic': round(tb * F) if tb else None,
            'hbm_frac': d['traffic_frac'],
            'alg_bytes_per_frame': d['alg_bytes_per_frame'], 'stage_ms_per_step': d['ms_per_step'],
            'launches': tim[dom][1], 'steps': steps, 'frames_per_step': F,
            'what': 'algorithmic bytes of the kernels the default path launches (stage_bytes_per_frame: the streams '
                    'they must read / write) x frames / the stage time per step (HIP events on the plan stream); '
                    'traffic = the same kernels\' HBM bytes per frame in the committed PMC summary ('
                    + PMC_FILES[config] + ') x frames per launch; hbm_frac = that traffic\'s rate / 8 TB/s',
            'pmc_source': 'profiles/' + PMC_FILES[config],
            'sq_counters': sq,
            'other_stages': {k: v for k, v in st.items() if k != dom}}


def roofline(config, prec, tim, steps, F, el, value, world, iters=8, plan=None):
    if config in (2, 4):
        roof = turbo_roofline(prec, tim, F, iters)
        t_ms = tim.get('turbo', (0.0, 0))[0]
        roof['turbo_share_of_step'] = round(t_ms / (el * 1e3) if el > 0 else 0, 3)
        if plan is not None:
            roof['front_end'] = front_end(prec, tim, F, config, plan, steps)
        if config == 2:
            esz = 8 if prec == 'f64' else 4
            # SURVEY §8(d)'s whole-chain view: compulsory stage-boundary bytes per subframe
            roof['pipeline_hbm'] = {'bytes_per_subframe': B_SF_F32 * esz // 4,
                                    'achieved_GBs': round(B_SF_F32 * esz / 4 * value / world / 1e9, 2),
                                    'frac': round(B_SF_F32 * esz / 4 * value / world / 1e9 / HBM_PEAK_GBS, 5)}
    else:
        roof = hbm_roofline(config, plan, prec, tim, F, steps) if plan is not None else None
        if roof is None:
            return None
    roof['kernel_ms_per_step'] = {k: round(v[0] / steps, 3) for k, v in tim.items() if v[1]}
    return roof


def same_box_shape_ceiling(hrs, F):
    """The decoder's access-shape ceiling measured on this box after the timed
    region (scripts/turbo_shape_bench, built with -DLTE_SHAPE_AUX=3, run as a
    child process): replaces the stored round-3 ceiling from another box."""
    exe = os.path.join(ROOT, 'scripts', 'turbo_shape_bench')
    if not os.path.exists(exe) or F % 64:
        return
    try:
        r = subprocess.run([exe, str(F), 'decoder'], capture_output=True, text=True, timeout=180)
        d = json.loads(r.stdout.strip().splitlines()[-1])
    except (subprocess.SubprocessError, ValueError, IndexError, OSError):
        return
    dl = d['decoder_layout']
    ceil = dl['GBs_best']
    tr = hrs.get('traffic_GBs')
    hrs['shape_ceiling'] = {'GBs': ceil, 'traffic_frac_of_ceiling': round(tr / ceil, 4) if tr else None,
                            'shape_ms': {k: dl[k] for k in ('ms_1wps', 'ms_2wps', 'ms_free')},
                            'source': 'same box, same call: scripts/turbo_shape_bench F decoder after the timed region'}
    if 'ms_1wps_reads_only' in dl:
        full, ro = dl['ms_1wps'], dl['ms_1wps_reads_only']
        share = (d['bytes_per_launch_stores'] / d['bytes_per_launch_ckpt'] if d.get('bytes_per_launch_stores')
                 else shape_store_share())
        hrs['store_cost'] = {'shape_ms_full': full, 'shape_ms_reads_only': ro,
                             'store_share_of_time': round(1 - ro / full, 3), 'store_share_of_bytes': round(share, 4),
                             'measured_in_this_run': True,
                             'source': 'same box, same call: the shape at one wave per SIMD with and without its '
                                       'extrinsic / checkpoint stores (scripts/turbo_shape_bench F decoder)'}


def merge_timers(all_tim):
    """Per stage, the rank whose mean launch time is the largest (the roofline
    prices the slowest rank's kernels, like the step time)."""
    out = {}
    for tim in all_tim:
        for k, (ms, n) in (tim or {}).items():
            if n and (k not in out or ms / n > out[k][0] / out[k][1]):
                out[k] = (ms, n)
    return out


def front_end(prec, tim, F, config, plan, steps):
    """Coded configs (2, 4): every front-end stage's algorithmic bytes
    (stage_bytes_per_frame) and committed PMC traffic beside its HIP-event
    time (stage_table), plus the VALU / LDS shares of active issue of its first
    kernel from the same PMC passes (what bounds the FFT / noise kernels, which
    are not HBM-bound)."""
    st = stage_table(config, plan, prec, tim, F, steps)
    pmc = load_profile(PMC_FILES[config]) if prec == 'f64' else None
    for k, v in st.items():
        if pmc:
            hits = [r for n, r in pmc['kernels'].items() if n == v['kernels'][0] or n.startswith(v['kernels'][0] + '<')]
            if hits:
                share = max(hits, key=lambda r: r.get('ms', 0)).get('share_of_active_issue', {})
                v['valu_share'], v['lds_share'] = share.get('valu'), share.get('lds')
        v['pmc_source'] = 'profiles/' + PMC_FILES[config] if pmc else None
    return st


def dry_run_counts(ids, S, n_bits=TB):
    """--dry-run: a deterministic per-frame statistic in place of the GPU chain
    (exercises the launcher, sharding and reductions without a device)."""
    from lte_phy import dist as D
    si = D.snr_index(ids, S)
    c = np.zeros((S, 4), dtype=np.uint64)
    np.add.at(c[:, 0], si, ids % np.uint64(7))
    np.add.at(c[:, 1], si, np.uint64(n_bits))
    np.add.at(c[:, 2], si, (ids % np.uint64(3) == 0).astype(np.uint64))
    np.add.at(c[:, 3], si, np.uint64(1))
    return c


# --dry-run: each config's plan geometry (what lte_plan_info reports for the
# bench plan) and synthetic per-stage timers, so the N > 1 rehearsal prices
# the same roofline as a GPU run (the line is marked dry_run)
DRY_GEOM = {
    2: dict(L=14 * 2192, n_sym=14, n_bits=TB, num_rx=1, num_tx=1, N=2048, Nd=999, n_grp=1, n_cb=5,
            coded_bits=83772, channel=1, n_paths=4, max_delay=13),
    3: dict(L=14 * 1096, n_sym=14, n_bits=14 * 499 * 4, num_rx=4, num_tx=1, N=1024, Nd=499, n_grp=1, channel=1,
            n_paths=6, max_delay=39),
    4: dict(L=14 * 2192, n_sym=14, n_bits=TB, num_rx=2, num_tx=2, N=2048, Nd=999, n_grp=1, n_cb=5,
            coded_bits=83772, res=998, n_dsc=998, n_est=1, pilots_per_tx=100, channel=1),
    5: dict(L=14 * 2192, n_sym=14, n_bits=14 * 999 * 6, num_rx=4, num_tx=4, N=2048, Nd=999, n_grp=1, n_dsc=250,
            n_est=14, pilots_per_tx=50, channel=0),
}
DRY_STAGE_SHARE = {2: {'turbo': 0.87, 'ofdm_tx': 0.04, 'rx_data': 0.045, 'dematch': 0.03},
                   3: {'ofdm_tx': 0.3, 'channel': 0.02, 'rx_data': 0.65},
                   4: {'turbo': 0.75, 'ofdm_tx': 0.08, 'channel': 0.001, 'rx_chest': 0.08, 'dematch': 0.03},
                   5: {'ofdm_tx': 0.25, 'fading': 0.001, 'channel': 0.001, 'rx_chest': 0.45, 'rx_data': 0.2}}


def dry_run_timers(config, el, steps, rank):
    """Synthetic kernel timers (ms, launches) of one rank: each stage's share
    of the elapsed time, rank r 1 % slower per rank (exercises the slowest-rank
    gather)."""
    return {k: (f * el * 1e3 * (1 + 0.01 * rank), steps) for k, f in DRY_STAGE_SHARE[config].items()}


def make_plan(config, args):
    """The bench plan of one config (the same builders the drop-in API uses)."""
    import lte_phy
    from lte_phy import _capi as C
    Cfg, Sim = lte_phy.LTEConfig, lte_phy.OFDMSimulator
    F = args.frames
    if config == 2:
        sim = Sim(Cfg(bandwidth=20.0, modulation='64-QAM'), channel_type='rayleigh_mp', itu_profile='Pedestrian_A',
                  velocity_kmh=args.velocity, precision=args.precision)
        return sim._plan(C.CHAIN_CODED, 0, TB, max_frames=F, iters=args.iters)
    if config == 3:
        sim = Sim(Cfg(bandwidth=10.0, modulation='16-QAM'), channel_type='rayleigh_mp', itu_profile='Vehicular_A',
                  velocity_kmh=args.velocity, precision=args.precision)
        return sim._plan(C.CHAIN_SIMO, 14, WORKLOADS[3]['n_bits'], num_rx=4, max_frames=F)
    if config == 4:
        sim = Sim(Cfg(bandwidth=20.0, modulation='64-QAM'), channel_type='rayleigh_mp', itu_profile='Pedestrian_A',
                  velocity_kmh=args.velocity, precision=args.precision)
        return sim._sfbc_plan(0, TB, 2, coded=True, max_frames=F, iters=args.iters)
    from lte_phy.ofdm_core import _spatial_plan
    return _spatial_plan(Cfg(bandwidth=20.0, modulation='64-QAM'), args.channel or 'awgn', 'Pedestrian_A',
                         args.velocity or 3.0, 2.0, 14, WORKLOADS[5]['n_bits'], F, precision=args.precision)[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--config', type=int, choices=sorted(WORKLOADS), default=2,
                    help='BASELINE.json config: 2 (the headline), 3, 4 or 5')
    ap.add_argument('--frames', type=int, default=None, help='subframes per step per GPU (default: per config)')
    ap.add_argument('--iters', type=int, default=8)
    ap.add_argument('--precision', choices=('f64', 'f32'), default='f64')
    ap.add_argument('--velocity', type=float, default=0.0,
                    help='UE speed in km/h (fD = v fc / c at 2 GHz); 0 = the OFDMSimulator default (static taps), '
                         '3 = the GUI default (Jakes fading over the subframe): a secondary line, not the headline')
    ap.add_argument('--channel', choices=('awgn', 'rayleigh_mp'), default=None,
                    help='config 5 only: flat CN(0,1) links (default, simulate_spatial_multiplexing\'s default) '
                         'or PedA Rayleigh at --velocity (3 km/h if 0)')
    ap.add_argument('--cpu-seconds', type=float, default=None)
    ap.add_argument('--no-cpu', action='store_true')
    ap.add_argument('--no-shape-ceiling', action='store_true',
                    help="skip measuring the decoder's access-shape ceiling on this box after the timed region "
                         '(scripts/turbo_shape_bench F decoder, a child process; N = 1, coded configs)')
    ap.add_argument('--dry-run', action='store_true', help='no GPU: launcher / sharding / reductions only (gloo)')
    argv = sys.argv[1:]
    args = ap.parse_args()
    wl = WORKLOADS[args.config]
    args.frames = int(args.frames or wl['frames'])

    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args, argv))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    # the CPU baseline runs first, in spawned worker processes, before anything
    # initialises the GPU: on rank 0 (under an external launcher the other ranks
    # wait for it in the rendezvous), or in the self-launching parent, which
    # hands it over in LTE_BENCH_CPU_JSON
    cpu = None
    if rank == 0 and os.environ.get('LTE_BENCH_CPU_JSON'):
        with open(os.environ['LTE_BENCH_CPU_JSON']) as f:
            cpu = json.load(f)
    elif rank == 0 and cpu_seconds(args) > 0:
        cpu = cpu_baseline(args.config, args.frames, cpu_seconds(args), None, args.channel)
        cpu['config'] = args.config
    import torch
    dist = None
    # LTE_BENCH_BACKEND=gloo: rehearse the N>1 path with several ranks sharing
    # the visible GPUs (device = LOCAL_RANK mod device count); the default is
    # RCCL ('nccl') with one rank per GPU
    backend = 'gloo' if args.dry_run else os.environ.get('LTE_BENCH_BACKEND', 'nccl')
    if backend == 'gloo' and not args.dry_run:
        local = local % max(1, torch.cuda.device_count())
        os.environ['LTE_DEVICE'] = str(local)   # the device lte_phy plans bind to
    if world > 1:
        import torch.distributed as dist
        if backend == 'nccl':
            torch.cuda.set_device(local)
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            if not args.dry_run:
                torch.cuda.set_device(local)
            dist.init_process_group('gloo')
    elif not args.dry_run:
        torch.cuda.set_device(local)

    from lte_phy import dist as D
    S = len(SNRS)
    F = args.frames
    counts = np.zeros((S, 4), dtype=np.uint64)
    prec = args.precision
    geom = None   # the plan's geometry for the uncoded configs' stage bytes
    if args.dry_run:
        import types
        plan = None
        geom = types.SimpleNamespace(**DRY_GEOM[args.config])
        dev_id = f'rank{rank}'
        step = lambda k: dry_run_counts(D.frame_ids(k, rank, world, F), S, wl['n_bits'])   # noqa: E731
    else:
        from lte_phy import _capi as C
        C.device_init(local)
        props = torch.cuda.get_device_properties(local)
        dev_id = f"{getattr(props, 'pci_bus_id', '')}:{getattr(props, 'uuid', local)}"
        plan = make_plan(args.config, args)
        geom = plan
        prec = plan.precision

        def step(k):
            ids = D.frame_ids(k, rank, world, F)
            si = D.snr_index(ids, S)
            return plan.run(SNRS[si], snr_index=si, n_snr=S, seed=SEED, frame_ids=ids)['counts']

    def barrier():
        if not args.dry_run:
            torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        if not args.dry_run:
            torch.cuda.synchronize()

    for w in range(args.warmup):
        step(10_000 + w)
    if plan is not None:
        plan.timing_reset()
        plan.timing(True)
    barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        counts += step(k)
    barrier()
    el = time.perf_counter() - t0
    tim = {}
    if plan is not None:
        plan.timing(False)
        tim = plan.timing_read()
    elif args.dry_run:
        # --dry-run: synthetic per-rank kernel timers (exercise the roofline
        # gather; the line is marked dry_run)
        tim = dry_run_timers(args.config, el, args.steps, rank)

    el = D.allreduce_max(el, dist)
    counts = D.allreduce_counts(counts, dist)
    # kernel timers of every rank: the roofline prices the slowest one
    if dist is not None:
        all_tim = [None] * world
        dist.all_gather_object(all_tim, tim)
        tim = merge_timers(all_tim)
    # distinct devices that took part (not the rank count)
    devs = [dev_id]
    if dist is not None:
        devs = [None] * world
        dist.all_gather_object(devs, dev_id)
    n_dev = len(set(devs))

    total = F * args.steps * world
    value = total / el
    ber = (counts[:, 0] / np.maximum(counts[:, 1], 1)).tolist()
    bler = (counts[:, 2] / np.maximum(counts[:, 3], 1)).tolist()
    workload = wl['desc']
    if args.velocity:
        workload += f' -- SECONDARY line: UE at {args.velocity:g} km/h (Jakes fading over the subframe)'
    if args.config == 5 and args.channel == 'rayleigh_mp':
        workload += f' -- links: Rayleigh PedA at {args.velocity or 3.0:g} km/h'
    metric = METRIC if args.config == 2 else f"LTE subframes/sec ({wl['short']}) at 1/2/4/8 GPU; BER match"
    out = {'metric': metric, 'value': round(value, 1), 'unit': 'subframes/s', 'n_gpus': n_dev,
           'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(el * 1e3 / args.steps, 3),
           'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': prec,
           'data': 'synthetic (Philox4x32-10 payload bits, Jakes phases and AWGN generated on the GPU)',
           'config': {'workload': workload, 'bench_config': args.config, 'velocity_kmh': args.velocity,
                      'frames_per_step_per_gpu': F, 'global_batch': F * world, 'parallelism': f'dp{world}',
                      'ranks': world, 'snr_db': SNRS.tolist()},
           'roofline': (roofline(args.config, prec, tim, args.steps, F, el, value, world, args.iters, geom)
                        if tim else None),
           'ber': [float(f'{b:.4e}') for b in ber], 'bler': [float(f'{b:.4e}') for b in bler]}
    if args.dry_run:
        out['dry_run'] = True
        out['counts'] = counts.tolist()
    if rank == 0:
        # BER match on the oracle's sample of this run's own frames (outside the timed region)
        out['ber_match'] = ber_match(plan, cpu, wl['coded']) if plan is not None else None
        if (not args.no_shape_ceiling and world == 1 and prec == 'f64' and plan is not None and out['roofline']
                and 'hbm_row_stream' in out['roofline']):
            same_box_shape_ceiling(out['roofline']['hbm_row_stream'], F)
        if cpu:
            cpu = {k: v for k, v in cpu.items() if k not in ('frames', 'config')}
            if world > 1:
                cpu['note'] = (f'{cpu["cores"]} single-threaded worker processes, one per core '
                               f'({cpu.get("host_cores", "?")} CPUs visible to the launcher; the CPU share is up to '
                               f'{CPU_PER_GPU} per GPU, {CPU_PER_GPU * world} for {world} GPUs)')
        out['cpu_baseline'] = cpu
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
