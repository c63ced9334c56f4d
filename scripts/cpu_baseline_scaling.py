"""CPU baseline scaling: the float64 oracle (bench.py's cpu_baseline worker) on
the bench's own config-2 frames with 1, 2, 4, ... and all of this host's
cores, one single-threaded process per core ("1 process and
nproc processes").  Run it on a host where a pool of every core is allowed
(not the GPU box, whose worker pools are sized to its 16-core share):

    python scripts/cpu_baseline_scaling.py [--config 2] [--seconds 8] [--out profiles/r6_cpu_baseline_scaling.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'ofdm-lte_amd')):
    if p not in sys.path:
        sys.path.insert(0, p)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', type=int, default=2)
    ap.add_argument('--seconds', type=float, default=8.0)
    ap.add_argument('--out', default=os.path.join(ROOT, 'profiles', 'r6_cpu_baseline_scaling.json'))
    a = ap.parse_args()
    for v in ('OMP_NUM_THREADS', 'OPENBLAS_NUM_THREADS', 'MKL_NUM_THREADS'):
        os.environ[v] = '1'
    host = os.cpu_count() or 1
    counts, p = [], 1
    while p < host:
        counts.append(p)
        p *= 2
    counts.append(host)
    rows = []
    for n in counts:
        value, frames, wall = bench._cpu_pool(a.config, bench.WORKLOADS[a.config]['frames'], a.seconds, n, None)
        rows.append({'procs': n, 'subframes_per_s': round(value, 3), 'per_core': round(value / n, 4),
                     'frames': len(frames), 'seconds': round(wall, 1)})
        print(json.dumps(rows[-1]), flush=True)
    out = {'config': a.config, 'cpu_model': bench._cpu_model(), 'host_cores': host, 'kind': 'port',
           'what': 'the float64 oracle (NumPy front end + C turbo decoder, bit-exact with the reference) on the '
                   "bench's own frames, one single-threaded process per core",
           'single_process': rows[0], 'all_cores': rows[-1], 'rows': rows,
           'scaling_all_over_single': round(rows[-1]['subframes_per_s'] / rows[0]['subframes_per_s'], 2)}
    with open(a.out, 'w') as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ('cpu_model', 'host_cores', 'scaling_all_over_single')}))


if __name__ == '__main__':
    main()
