"""Probe: do two config-2 plans on their own streams overlap one plan's front
end with the other's decoder?  (A/B for a pipelined run; not a product path.)

python scripts/overlap_probe.py [F] [steps]
Prints frames/s for: one plan of F frames; one plan of F/2; two plans of F/2
run from two host threads (each plan has its own HIP stream).
"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'ofdm-lte_amd'))

import numpy as np  # noqa: E402
import bench  # noqa: E402


def main():
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    import torch
    from lte_phy import _capi as C
    from lte_phy import dist as D
    C.device_init(0)
    torch.cuda.set_device(0)

    class A:
        pass
    S = len(bench.SNRS)

    def plan_of(n):
        a = A()
        a.frames, a.velocity, a.precision, a.iters, a.channel = n, 0.0, 'f64', 8, None
        return bench.make_plan(2, a)

    def stepper(plan, n, rank, world):
        def step(k):
            ids = D.frame_ids(k, rank, world, n)
            si = D.snr_index(ids, S)
            return plan.run(bench.SNRS[si], snr_index=si, n_snr=S, seed=bench.SEED, frame_ids=ids)['counts']
        return step

    def timed(fn, nsteps):
        fn(1000)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k in range(nsteps):
            fn(k)
        torch.cuda.synchronize()
        return time.perf_counter() - t

    full = plan_of(F)
    t1 = timed(stepper(full, F, 0, 1), steps)
    print(f'one plan F={F}: {steps * F / t1:.0f} frames/s ({t1 / steps * 1e3:.1f} ms/step)', flush=True)
    del full
    h0, h1 = plan_of(F // 2), plan_of(F // 2)
    s0, s1 = stepper(h0, F // 2, 0, 2), stepper(h1, F // 2, 1, 2)
    th = timed(s0, steps)
    print(f'one plan F/2: {steps * F / 2 / th:.0f} frames/s ({th / steps * 1e3:.1f} ms/step)', flush=True)
    s0(1001), s1(1001)
    torch.cuda.synchronize()
    n2 = 2 * steps
    t = time.perf_counter()
    ths = [threading.Thread(target=lambda f=f: [f(k) for k in range(n2)]) for f in (s0, s1)]
    for x in ths:
        x.start()
    for x in ths:
        x.join()
    torch.cuda.synchronize()
    t2 = time.perf_counter() - t
    print(f'two plans F/2, two threads: {n2 * F / t2:.0f} frames/s ({t2 / n2 * 1e3:.1f} ms per F/2-pair step)',
          flush=True)


if __name__ == '__main__':
    main()
