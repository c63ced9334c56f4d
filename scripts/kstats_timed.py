"""Per-kernel durations of bench.py's timed launches from a rocprofv3
--kernel-trace CSV: the dominant kernel's dispatches in order, split into the
warm-up launches, the K timed launches and whatever follows (the ber_match
re-run), so the trace's average over the timed launches can be set beside the
bench line's roofline.avg_launch_ms (the --stats summary averages all of them).

usage: python scripts/kstats_timed.py <run_kernel_trace.csv> <kernel substring> <warmup> <steps>
"""
import csv
import json
import sys


def main():
    path, name, warmup, steps = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    d = []
    for r in csv.DictReader(open(path)):
        if name in r['Kernel_Name']:
            d.append((int(r['Dispatch_Id']), (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-6))
    d.sort()
    ms = [x[1] for x in d]
    timed = ms[warmup:warmup + steps]
    out = {'source': path, 'kernel': name, 'dispatches': len(ms), 'warmup': warmup, 'steps': steps,
           'warmup_ms': [round(x, 3) for x in ms[:warmup]],
           'timed_avg_ms': round(sum(timed) / len(timed), 3) if timed else None,
           'timed_min_ms': round(min(timed), 3) if timed else None,
           'timed_max_ms': round(max(timed), 3) if timed else None,
           'after_ms': [round(x, 3) for x in ms[warmup + steps:]],
           'all_avg_ms': round(sum(ms) / len(ms), 3) if ms else None}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
