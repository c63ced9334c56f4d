"""Summarise the FETCH_SIZE / WRITE_SIZE passes of scripts/gpu_full.sh into
profiles/pmc_turbo_traffic.json (read by bench.py for roofline.traffic).

gfx950 corrections (MI355X_MICROARCH.md, HBM / rocprofv3): FETCH_SIZE counts
1/2 of the bytes of wide coalesced streaming reads -> x2; WRITE_SIZE is exact.
Both are in kB (x1024)."""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FRAMES = 8192
TSUB = 2   # alpha checkpoint every 8 * TSUB trellis steps (lte_turbo.hip)


def per_kernel(counter, src):
    tot = defaultdict(float)
    with open(os.path.join(src, f'pmc_{counter}', 'run_counter_collection.csv')) as f:
        for r in csv.DictReader(f):
            name = r['Kernel_Name'].split('(')[0].strip()
            tot[name] += float(r['Counter_Value'])
    return dict(tot)


def main(src=os.path.join(ROOT, 'gpurun_out')):
    fk = per_kernel('FETCH_SIZE', src)
    wk = per_kernel('WRITE_SIZE', src)
    key = [k for k in fk if k.endswith('k_turbo')][0]
    read_b = 2.0 * fk[key] * 1024
    write_b = wk[key] * 1024
    steps, passes = 27919, 17          # sum(K+3) over the 5 CBs of TB 27760; 8 iterations x 2 + final
    ck = 7.0 / (8 * TSUB)
    model_r = steps * passes * 4 * (6 + ck)
    model_w = steps * passes * 4 * (1 + ck)
    out = {
        'kernel': 'k_turbo',
        'frames_per_launch': FRAMES,
        'command': f'rocprofv3 --pmc <C> --kernel-trace --output-format csv -- python3 bench.py --frames {FRAMES} '
                   '--steps 1 --warmup 0 --no-cpu (one pass per counter; scripts/gpu_full.sh)',
        'FETCH_SIZE_kB_raw': fk[key],
        'WRITE_SIZE_kB': wk[key],
        'correction': 'MI355X_MICROARCH.md HBM section: gfx950 FETCH_SIZE reports 1/2 of streaming-read bytes -> '
                      'read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE x 1024 exact.',
        'read_bytes': read_b,
        'write_bytes': write_b,
        'bytes_per_frame': (read_b + write_b) / FRAMES,
        'model_bytes_per_frame': {
            'reads': round(model_r), 'writes': round(model_w),
            'note': f'per CB-step-pass (256-B rows = 4 B per code block): fwd 3 loads + bwd 3 loads + '
                    f'7/{8 * TSUB} ckpt load read; 7/{8 * TSUB} ckpt store + extrinsic store written; '
                    f'x sum(K+3) = {steps} steps x {passes} passes'},
        'per_kernel_kB': {'FETCH_SIZE': fk, 'WRITE_SIZE': wk},
    }
    with open(os.path.join(ROOT, 'profiles', 'pmc_turbo_traffic.json'), 'w') as f:
        json.dump(out, f, indent=1)
    print(f"k_turbo: {out['bytes_per_frame'] / 1e6:.2f} MB/frame measured, "
          f"{(model_r + model_w) / 1e6:.2f} MB/frame model")


if __name__ == '__main__':
    main(*sys.argv[1:])
