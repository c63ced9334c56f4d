"""PCIe-inclusive throughput of config 2 through the C-ABI with host buffers
(DESIGN.md §7): the drop-in's single-call shape, where the payload bits come
from and the decoded bits go back to NumPy arrays, next to the resident-input
rate bench.py reports.  Three variants, each timed around lte_run only (the
host arrays are made beforehand):

  resident  Philox payload / fading / noise on the device, counters back (bench.py's value)
  bits      payload bits in (uint8, 27 760 per frame) + decoded bits out
  refcompat bits in / out + the reference's own draws injected: 16 phases per
            path and the unit-normal noise (2 x 30 688 float64 per frame)

usage: python scripts/bench_hostbuf.py [--frames F] [--steps K]   (prints one JSON line)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'ofdm-lte_amd'))

TB = 27760
SNRS = np.arange(0, 31, 2, dtype=np.float64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--frames', type=int, default=8192)
    ap.add_argument('--steps', type=int, default=3)
    args = ap.parse_args()
    import lte_phy
    from lte_phy import _capi as C
    C.device_init(0)
    F = args.frames
    sim = lte_phy.OFDMSimulator(lte_phy.LTEConfig(bandwidth=20.0, modulation='64-QAM'), channel_type='rayleigh_mp',
                                itu_profile='Pedestrian_A')
    plan = sim._plan(C.CHAIN_CODED, 0, TB, max_frames=F)
    rs = np.random.RandomState(0)
    ids = np.arange(F, dtype=np.uint64)
    si = (ids % np.uint64(len(SNRS))).astype(np.int32)
    snr = SNRS[si]
    bits = rs.randint(0, 2, (F, TB)).astype(np.uint8)
    n_paths = len(sim.channels[0].delays)
    phases = 2 * np.pi * rs.rand(F, n_paths, 16)
    noise = rs.randn(F, 2, plan.L)
    variants = {
        'resident': dict(),
        'bits': dict(bits=bits, capture=('bits_rx',)),
        'refcompat': dict(bits=bits, phases=phases, noise=noise, capture=('bits_rx',)),
    }
    out = {'workload': 'config 2 coded subframes (TB 27760), 8 iterations, f64', 'frames_per_call': F,
           'steps': args.steps}
    for name, kw in variants.items():
        plan.run(snr, snr_index=si, n_snr=len(SNRS), seed=0x5EED, frame_ids=ids, **kw)   # warm
        t0 = time.perf_counter()
        for _ in range(args.steps):
            r = plan.run(snr, snr_index=si, n_snr=len(SNRS), seed=0x5EED, frame_ids=ids, **kw)
        el = (time.perf_counter() - t0) / args.steps
        h2d = sum(v.nbytes for k, v in kw.items() if isinstance(v, np.ndarray))
        d2h = sum(r[c].nbytes for c in kw.get('capture', ()))
        out[name] = {'subframes_per_s': round(F / el, 1), 'ms_per_call': round(el * 1e3, 2),
                     'host_to_device_MB': round(h2d / 1e6, 1), 'device_to_host_MB': round(d2h / 1e6, 1)}
        print(json.dumps({name: out[name]}), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
