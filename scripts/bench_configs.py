"""Throughput of every BASELINE.json config on one MI355X (Philox inputs on the
device, SNR cycling over 0:2:30 dB), with the per-kernel breakdown.  The
headline line (config 2) is bench.py's; this script reports the other chains
the same way.  Prints one JSON object per config.

usage: python scripts/bench_configs.py [--frames F] [--steps K] [--only c1,c3,...]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'ofdm-lte_amd'))

SNRS = np.arange(0, 31, 2, dtype=np.float64)


def configs(lte_phy, C):
    O = lte_phy.OFDMSimulator
    Cfg = lte_phy.LTEConfig

    def c1(F):
        s = O(Cfg(bandwidth=1.25, modulation='QPSK'), channel_type='awgn')
        return s._plan(C.CHAIN_UNCODED, 14, 14 * s.Nd * 2, max_frames=F)

    def c2(F):
        s = O(Cfg(bandwidth=20.0, modulation='64-QAM'), channel_type='rayleigh_mp', itu_profile='Pedestrian_A')
        return s._plan(C.CHAIN_CODED, 0, 27760, max_frames=F)

    def c3(F):
        s = O(Cfg(bandwidth=10.0, modulation='16-QAM'), channel_type='rayleigh_mp', itu_profile='Vehicular_A')
        return s._plan(C.CHAIN_SIMO, 14, 14 * s.Nd * 4, num_rx=4, max_frames=F)

    def c4(F):
        s = O(Cfg(bandwidth=20.0, modulation='64-QAM'), channel_type='rayleigh_mp', itu_profile='Pedestrian_A')
        return s._sfbc_plan(0, 27760, 2, coded=True, max_frames=F)

    def c5(chan):
        def f(F):
            from lte_phy.ofdm_core import _spatial_plan, ResourceGrid
            cfg = Cfg(bandwidth=20.0, modulation='64-QAM')
            nd = len(ResourceGrid(cfg.N, cfg.Nc)._data)
            return _spatial_plan(cfg, chan, 'Pedestrian_A', 3, 2.0, 14, 14 * nd * 6, F)[0]
        return f

    def tm4(num_tx, num_rx, rank, det, pmi=0):
        def f(F):
            from lte_phy.ofdm_core import _spatial_plan, ResourceGrid
            from lte_phy.tm4 import DETECTORS, LTECodebook
            cfg = Cfg(bandwidth=20.0, modulation='64-QAM')
            nd = len(ResourceGrid(cfg.N, cfg.Nc)._data)
            W = LTECodebook(num_tx, transmission_mode='TM4', rank=rank).get_precoder(pmi)
            return _spatial_plan(cfg, 'awgn', 'Pedestrian_A', 3, 2.0, 14, 14 * nd * 6, F, num_tx=num_tx,
                                 num_rx=num_rx, rank=rank, detector=DETECTORS[det], W=W)[0]
        return f

    def c2u(F):
        s = O(Cfg(bandwidth=20.0, modulation='64-QAM'), channel_type='rayleigh_mp', itu_profile='Pedestrian_A')
        return s._plan(C.CHAIN_UNCODED, 14, 14 * s.Nd * 6, max_frames=F)

    def scfdm(F):
        s = O(Cfg(bandwidth=20.0, modulation='64-QAM'), channel_type='rayleigh_mp', itu_profile='Pedestrian_A',
              enable_sc_fdm=True)
        return s._plan(C.CHAIN_UNCODED, 14, 14 * s.Nd * 6, max_frames=F)

    def bf(num_tx, num_rx, adaptive):
        def f(F):
            from lte_phy.beamforming import bf_plan
            cfg = Cfg(bandwidth=20.0, modulation='64-QAM')
            s = O(cfg)
            return bf_plan(cfg, 14, 14 * s.Nd * 6, num_tx, num_rx, adaptive, F)
        return f

    return {
        'c1': ('config 1: SISO 1.25 MHz QPSK AWGN, 14 symbols uncoded', c1),
        'c2': ('config 2: SISO 20 MHz 64-QAM PedA + turbo (TB 27760)', c2),
        'c3': ('config 3: SIMO 1x4 MRC 10 MHz 16-QAM VehA, 14 symbols uncoded', c3),
        'c4': ('config 4: SFBC 2x2 Alamouti + turbo, 20 MHz 64-QAM PedA (TB 27760)', c4),
        'c5': ('config 5: spatial 4x4 rank-4 MMSE, 20 MHz 64-QAM, flat CN(0,1) links', c5('awgn')),
        'c5r': ('config 5: spatial 4x4 rank-4 MMSE, 20 MHz 64-QAM, PedA 3 km/h links', c5('rayleigh_mp')),
        'tm4_sic44': ('TM4 4x4 rank-4 SIC (PMI 1), 20 MHz 64-QAM, flat CN(0,1) links', tm4(4, 4, 4, 'SIC', 1)),
        'tm4_zf22': ('TM4 2x2 rank-2 ZF (PMI 1), 20 MHz 64-QAM, flat CN(0,1) links', tm4(2, 2, 2, 'ZF', 1)),
        'tm4_mrc41': ('TM4 4x1 rank-1 MRC (PMI 3), 20 MHz 64-QAM, flat CN(0,1) links', tm4(4, 1, 1, 'MRC', 3)),
        'c2u': ('SISO 20 MHz 64-QAM PedA, 14 symbols uncoded (OFDM, for the SC-FDM comparison)', c2u),
        'scfdm': ('SC-FDM SISO 20 MHz 64-QAM PedA, 14 symbols uncoded (M = 999 DFT)', scfdm),
        'bf81': ('beamforming 8x1 adaptive MRT, 20 MHz 64-QAM, 14 symbols (frequency domain)', bf(8, 1, True)),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--frames', type=int, default=8192)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--only', default='')
    args = ap.parse_args()
    import lte_phy
    from lte_phy import _capi as C
    C.device_init(0)
    want = [w for w in args.only.split(',') if w]
    for key, (desc, mk) in configs(lte_phy, C).items():
        if want and key not in want:
            continue
        F = args.frames
        plan = mk(F)
        S = len(SNRS)

        def step(k):
            ids = np.uint64(k * F) + np.arange(F, dtype=np.uint64)
            si = (ids % np.uint64(S)).astype(np.int32)
            return plan.run(SNRS[si], snr_index=si, n_snr=S, seed=0x5EED, frame_ids=ids)['counts']

        step(1000)
        plan.timing_reset()
        plan.timing(True)
        counts = np.zeros((S, 4), dtype=np.uint64)
        t0 = time.perf_counter()
        for k in range(args.steps):
            counts += step(k)
        el = time.perf_counter() - t0
        plan.timing(False)
        tim = plan.timing_read()
        ber = counts[:, 0] / np.maximum(counts[:, 1], 1)
        print(json.dumps({'config': key, 'workload': desc, 'frames_per_step': F, 'steps': args.steps,
                          'subframes_per_s': round(F * args.steps / el, 1), 'ms_per_step': round(el * 1e3 / args.steps, 3),
                          'kernel_ms_per_step': {k: round(v[0] / args.steps, 3) for k, v in tim.items() if v[1]},
                          'ber_by_snr': [float(f'{b:.3e}') for b in ber]}), flush=True)
        del plan
        from lte_phy import engine
        engine.clear_cache()


if __name__ == '__main__':
    main()
