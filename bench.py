"""Headline benchmark: LTE subframes/s through the full coded chain
(config 2: 20 MHz, 64-QAM, Rayleigh ITU Pedestrian-A, turbo max-log-MAP x8,
TB 27 760 bits = 5 code blocks = 14 OFDM symbols), BER sweep SNR 0:2:30 dB,
in float64 (the reference's arithmetic; `--precision f32` is the fast mode).

One step = one batch of `--frames` subframes per GPU pushed TX -> channel ->
RX + turbo; all inputs (Philox bits / fading / noise) are generated on the
device.  N>1: one process per GPU (torch.distributed, RCCL); frames are
partitioned by global frame id (weak scaling, no data-path collective); the
only collectives are the SUM of the BER counters and the MAX of the step time.

`python bench.py --gpus N` with no launcher environment starts N ranks itself
(torch.distributed.run on 127.0.0.1, before anything touches the GPU) and
exits with their status; under a launcher WORLD_SIZE must equal --gpus.

usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--frames F] [--precision f64|f32] [--velocity KMH]
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
TB = 27760
HBM_PEAK_GBS = 8000.0
# compulsory stage-boundary bytes of one config-2 coded subframe
# (TX map+IFFT, channel, FFT, estimation/equalisation/LLR, dematch+decode, CRC),
# quoted for 4-B reals; the f64 chain moves 8-B reals at the same boundaries
B_SF_F32 = 2_116_904
# turbo work per subframe = sum(K+3) x 17 passes x ~100 ops
TURBO_OPS_SF = 27_919 * 17 * 100
# Non-packed vector ALU peaks of one MI355X (add / max, 1 op per lane per
# instruction; 256 CUs x 4 SIMD-32 x 2.4 GHz):
#  * f32: a wave64 instruction every 2 cycles per SIMD with several waves
#    resident (MI355X_MICROARCH.md: SIMD-32, 2 cycles per wave64 VALU op)
#    = 32 lane-ops/cycle/SIMD -> 78.6 T op/s (half the 157.3 TFLOPS FMA spec)
#  * f64: 16 lane-ops/cycle/SIMD (the 78.6 TFLOPS f64 vector FMA spec / 2)
#    -> 39.3 T op/s; scripts/valu_peak_bench.hip measures both on the box
VALU_PEAK_OPS = {'f32': 256 * 4 * 32 * 2.4e9, 'f64': 256 * 4 * 16 * 2.4e9}


def _cpu_worker(job):
    """One host core: the oracle's config-2 coded chain on its own frames for
    `seconds`; returns (subframes, elapsed)."""
    seconds, seed = job
    from oracle import lte_oracle as O
    O.lib()
    num = O.Numerology(bandwidth=20.0, modulation='64-QAM')
    L = 14 * (num.N + num.cp)
    rs = np.random.RandomState(seed)
    n, t0 = 0, time.perf_counter()
    while True:
        bits = rs.randint(0, 2, TB)
        d = [{'phases': [2 * np.pi * rs.rand(16) for _ in range(4)], 'z_re': rs.randn(L), 'z_im': rs.randn(L)}]
        O.simulate_siso_coded(num, bits, float(SNRS[n % len(SNRS)]), 'rayleigh_mp', draws=d)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return n, el


def _cpu_model():
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or 'unknown'


def cpu_baseline(seconds=15.0, procs=None):
    """Time the oracle (float64 CPU restatement: NumPy front end + C turbo
    decoder, bit-exact with the reference) on this host's cores on a bounded
    sample of the same workload (config-2 coded subframes cycling over SNRs):
    one single-threaded worker process per core (frames are independent), the
    box's CPU share at most (16 per GPU).  Runs before the GPU is initialised
    (the workers are spawned processes)."""
    import multiprocessing as mp
    procs = procs or max(1, min(16, os.cpu_count() or 1))
    for v in ('OMP_NUM_THREADS', 'OPENBLAS_NUM_THREADS', 'MKL_NUM_THREADS'):
        os.environ[v] = '1'
    with mp.get_context('spawn').Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(seconds, 1234 + i) for i in range(procs)])
    n = sum(r[0] for r in res)
    value = sum(r[0] / r[1] for r in res)
    return {'value': value, 'unit': 'subframes/s', 'cores': procs, 'kind': 'port',
            'per_core': value / procs, 'cpu_model': _cpu_model(),
            'sample': f'{n} config-2 coded subframes (TB {TB}, 8 it.) over SNR 0:2:30 dB, '
                      f'{max(r[1] for r in res):.1f} s on {procs} host cores, one single-threaded '
                      f'process each (oracle: NumPy + C, float64)'}


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
    never touches the GPU), then run N ranks under torch.distributed.run as a
    child process and return its status.  Rank 0 reads the baseline from
    LTE_BENCH_CPU_JSON, so the N > 1 line carries it too."""
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    if not args.no_cpu:
        env['LTE_BENCH_CPU_JSON'] = json.dumps(cpu_baseline(args.cpu_seconds))
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={args.gpus}',
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), os.path.abspath(__file__)] + argv
    return subprocess.call(cmd, env=env)


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


def roofline(prec, tim, steps, F, el, value, world, iters=8):
    """Dominant kernel (the turbo decoder, ~87 % of a step) against the roofline
    that bounds it.  The exact decoder streams its rows: `achieved` = the
    compulsory row bytes of the exact recursion (decoder_row_bytes) per launch
    / the kernel's mean launch time (HIP events on the plan's stream; the max
    over ranks), against the 8 TB/s HBM peak; `traffic` = the PMC-measured HBM
    bytes per launch (profiles/pmc_turbo_traffic_<prec>.json, gfx950-corrected),
    with `shape_ceiling` = the measured streaming rate of the same access shape
    without the arithmetic (profiles/r3_turbo_shape_microbench.json).  Beside
    it: SURVEY §8(d)'s stage-boundary bytes (input LLRs + decoded bits) and its
    VALU view (sum(K+3) x 17 passes x 100 add/max ops per subframe against the
    non-packed vector peak), and the SQ-counted VALU issue occupancy.  `bound`
    is the larger of the measured HBM and VALU occupancies."""
    from lte_phy.channel_coding import segmentation_sizes
    t_ms, t_n = tim.get('turbo', (0.0, 0))
    avg_s = t_ms / max(t_n, 1) * 1e-3
    Fp = ((F + 63) // 64) * 64            # frames padded to whole 64-frame decoder groups
    esz = 8 if prec == 'f64' else 4
    Ks = segmentation_sizes(TB + 24)
    row_bytes = sum(Fp * decoder_row_bytes(K, esz, iters) for K in Ks)
    stage_bytes = sum(Fp * ((3 * K + 12) * esz + K / 8) for K in Ks)
    peak = VALU_PEAK_OPS[prec]
    ops = TURBO_OPS_SF * F
    achieved_T = ops / avg_s / 1e12 if t_n else 0.0
    traffic = load_profile(f'pmc_turbo_traffic_{prec}.json')
    sq = load_profile(f'pmc_turbo_sq_{prec}.json')
    shape = load_profile('r3_turbo_shape_microbench.json')
    gbs = row_bytes / avg_s / 1e9 if t_n else 0.0
    tr = traffic['bytes_per_frame'] * Fp if traffic else None
    tr_gbs = tr / avg_s / 1e9 if tr and t_n else None
    busy = (sq['valu_wave_instr_per_frame'] * Fp * sq['issue_cycles_per_instr'] / (avg_s * 2.4e9 * 1024)
            if sq and t_n else None)
    hbm_occ = (tr_gbs if tr_gbs else gbs) / HBM_PEAK_GBS
    ceil = shape.get(f'ceiling_GBs_{prec}') if shape else None
    roof = {'bound': 'hbm' if busy is None or hbm_occ >= busy else 'valu',
            'kernel': 'k_turbo64' if prec == 'f64' else 'k_turbo',
            'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': round(gbs / HBM_PEAK_GBS, 4),
            # HBM bytes per launch from the committed PMC passes (per-frame bytes,
            # gfx950-corrected, scaled to this launch's frames)
            'traffic': round(tr) if tr else None,
            'alg_bytes_per_launch': int(row_bytes),
            'alg_bytes': 'exact-recursion row stream: per code-block step 7 rows (Ls, Lp, La forward and '
                         'backward + extrinsic store) x esz B x 17 passes (first pass 5, final 6 + K/8 B decisions)',
            'traffic_over_alg': round(tr / row_bytes, 3) if tr else None,
            'traffic_GBs': round(tr_gbs, 1) if tr_gbs else None,
            'traffic_frac': round(tr_gbs / HBM_PEAK_GBS, 4) if tr_gbs else None,
            'shape_ceiling': ({'GBs': ceil, 'traffic_frac_of_ceiling': round(tr_gbs / ceil, 4) if tr_gbs else None,
                               'source': 'profiles/r3_turbo_shape_microbench.json'} if ceil else None),
            'avg_launch_ms': round(avg_s * 1e3, 3), 'launches': t_n, 'frames_per_launch': F,
            'stage_bytes': {'bytes_per_launch': int(stage_bytes), 'achieved_GBs': round(stage_bytes / avg_s / 1e9, 2)
                            if t_n else 0.0, 'frac': round(stage_bytes / avg_s / 1e9 / HBM_PEAK_GBS, 5) if t_n else 0.0,
                            'what': 'SURVEY §8(d) stage boundary: rate-dematched input LLRs + decoded bits'},
            'valu': {'achieved_Tops': round(achieved_T, 3), 'peak_Tops': round(peak / 1e12, 2),
                     'frac': round(achieved_T * 1e12 / peak, 4), 'ops_per_subframe': TURBO_OPS_SF,
                     'issued_busy_frac': round(busy, 4) if busy is not None else None,
                     'wave_instr_per_frame': sq['valu_wave_instr_per_frame'] if sq else None},
            'turbo_share_of_step': round(t_ms / (el * 1e3) if el > 0 else 0, 3),
            'front_end': front_end(prec, tim, F),
            'kernel_ms_per_step': {k: round(v[0] / steps, 3) for k, v in tim.items() if v[1]},
            # SURVEY §8(d)'s whole-chain view: compulsory stage-boundary bytes per subframe
            'pipeline_hbm': {'bytes_per_subframe': B_SF_F32 * esz // 4,
                             'achieved_GBs': round(B_SF_F32 * esz / 4 * value / world / 1e9, 2),
                             'frac': round(B_SF_F32 * esz / 4 * value / world / 1e9 / HBM_PEAK_GBS, 5)}}
    return roof


def merge_timers(all_tim):
    """Per stage, the rank whose mean launch time is the largest (the roofline
    prices the slowest rank's kernels, like the step time)."""
    out = {}
    for tim in all_tim:
        for k, (ms, n) in (tim or {}).items():
            if n and (k not in out or ms / n > out[k][0] / out[k][1]):
                out[k] = (ms, n)
    return out


# front-end stages (bench timers) -> their kernels in the committed PMC summary
FE_KERNELS = {'payload': ['k_payload'], 'encode': ['k_encode'], 'ofdm_tx': ['k_ofdm_txf'],
              'rx_data': ['k_rx_frame'], 'dematch': ['k_dematch_zn'], 'crc_count': ['k_crc_count']}


def front_end(prec, tim, F):
    """Per front-end stage: its HIP-event time per launch, the HBM bytes per
    frame its kernels move (profiles/r3_pmc_<prec>.json, rocprofv3 FETCH_SIZE /
    WRITE_SIZE, gfx950-corrected) and the resulting rate against the 8 TB/s
    peak, plus the VALU / LDS shares of active issue from the same PMC passes
    (what bounds the FFT / noise kernels, which are not HBM-bound)."""
    pmc = load_profile(f'r3_pmc_{prec}.json') or load_profile(f'r2_pmc_{prec}.json')
    if not pmc:
        return None
    ks = pmc['kernels']
    out = {}
    for stage, names in FE_KERNELS.items():
        t_ms, n = tim.get(stage, (0.0, 0))
        if not n or not all(k in ks for k in names):
            continue
        b = sum(ks[k]['hbm_bytes_per_frame'] for k in names)
        gbs = b * F / (t_ms / n * 1e-3) / 1e9
        share = ks[names[0]].get('share_of_active_issue', {})
        out[stage] = {'kernels': names, 'ms': round(t_ms / n, 3), 'hbm_bytes_per_frame': round(b),
                      'achieved_GBs': round(gbs, 1), 'frac': round(gbs / HBM_PEAK_GBS, 3),
                      'valu_share': share.get('valu'), 'lds_share': share.get('lds')}
    return out


def dry_run_counts(ids, S):
    """--dry-run: a deterministic per-frame statistic in place of the GPU chain
    (exercises the launcher, sharding and reductions without a device)."""
    from lte_phy import dist as D
    si = D.snr_index(ids, S)
    c = np.zeros((S, 4), dtype=np.uint64)
    np.add.at(c[:, 0], si, ids % np.uint64(7))
    np.add.at(c[:, 1], si, np.uint64(TB))
    np.add.at(c[:, 2], si, (ids % np.uint64(3) == 0).astype(np.uint64))
    np.add.at(c[:, 3], si, np.uint64(1))
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--frames', type=int, default=65536, help='subframes per step per GPU')
    ap.add_argument('--iters', type=int, default=8)
    ap.add_argument('--precision', choices=('f64', 'f32'), default='f64')
    ap.add_argument('--velocity', type=float, default=0.0,
                    help='UE speed in km/h (fD = v fc / c at 2 GHz); 0 = the OFDMSimulator default (static taps), '
                         '3 = the GUI default (Jakes fading over the subframe): a secondary line, not the headline')
    ap.add_argument('--cpu-seconds', type=float, default=15.0)
    ap.add_argument('--no-cpu', action='store_true')
    ap.add_argument('--dry-run', action='store_true', help='no GPU: launcher / sharding / reductions only (gloo)')
    argv = sys.argv[1:]
    args = ap.parse_args()

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
    if rank == 0 and not args.no_cpu:
        cpu = (json.loads(os.environ['LTE_BENCH_CPU_JSON']) if os.environ.get('LTE_BENCH_CPU_JSON')
               else cpu_baseline(args.cpu_seconds))
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
    F = int(args.frames)
    counts = np.zeros((S, 4), dtype=np.uint64)
    if args.dry_run:
        plan = None
        dev_id = f'rank{rank}'
        step = lambda k: dry_run_counts(D.frame_ids(k, rank, world, F), S)   # noqa: E731
        prec = args.precision
    else:
        import lte_phy
        from lte_phy import _capi as C
        C.device_init(local)
        props = torch.cuda.get_device_properties(local)
        dev_id = f"{getattr(props, 'pci_bus_id', '')}:{getattr(props, 'uuid', local)}"
        sim = lte_phy.OFDMSimulator(lte_phy.LTEConfig(bandwidth=20.0, modulation='64-QAM'),
                                    channel_type='rayleigh_mp', itu_profile='Pedestrian_A',
                                    velocity_kmh=args.velocity, precision=args.precision)
        plan = sim._plan(C.CHAIN_CODED, 0, TB, max_frames=F, iters=args.iters)
        prec = plan.precision

        def step(k):
            ids = D.frame_ids(k, rank, world, F)
            si = D.snr_index(ids, S)
            return plan.run(SNRS[si], snr_index=si, n_snr=S, seed=0x5EED, frame_ids=ids)['counts']

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
        tim = {'turbo': (0.8 * el * 1e3 * (1 + 0.01 * rank), args.steps)}

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
    workload = ('config 2: SISO 20 MHz (N=2048) 64-QAM, Rayleigh ITU Pedestrian-A, '
                'turbo max-log-MAP 8 it., TB 27760 (5 CBs, 14 OFDM symbols), SNR 0:2:30 dB')
    if args.velocity:
        workload += f' -- SECONDARY line: UE at {args.velocity:g} km/h (Jakes fading over the subframe)'
    out = {'metric': METRIC, 'value': round(value, 1), 'unit': 'subframes/s', 'n_gpus': n_dev,
           'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(el * 1e3 / args.steps, 3),
           'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': prec,
           'data': 'synthetic (Philox4x32-10 payload bits, Jakes phases and AWGN generated on the GPU)',
           'config': {'workload': workload, 'velocity_kmh': args.velocity,
                      'frames_per_step_per_gpu': F, 'global_batch': F * world, 'parallelism': f'dp{world}',
                      'ranks': world, 'snr_db': SNRS.tolist()},
           'roofline': roofline(prec, tim, args.steps, F, el, value, world, args.iters) if tim else None,
           'ber': [float(f'{b:.4e}') for b in ber], 'bler': [float(f'{b:.4e}') for b in bler]}
    if args.dry_run:
        out['dry_run'] = True
        out['counts'] = counts.tolist()
    if rank == 0:
        out['cpu_baseline'] = cpu
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
