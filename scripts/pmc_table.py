"""Per-kernel table of the SQ counter passes (gpurun_out/pmc_sq*/): counter
sums over the kernel's dispatches and the kernel's traced duration."""
import csv
import glob
import os
import sys
from collections import defaultdict

src = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out'
val = defaultdict(lambda: defaultdict(float))
dur = defaultdict(float)
for d in sorted(glob.glob(os.path.join(src, 'pmc_sq*'))):
    if not os.path.isdir(d):
        continue
    seen = set()
    with open(os.path.join(d, 'run_counter_collection.csv')) as f:
        for r in csv.DictReader(f):
            k = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('lte::', '')
            val[k][r['Counter_Name']] += float(r['Counter_Value'])
            if d.endswith('1') and (r['Dispatch_Id']) not in seen:
                seen.add(r['Dispatch_Id'])
                dur[k] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-6
cols = sorted({c for v in val.values() for c in v})
print('kernel'.ljust(28), 'ms'.rjust(8), *[c.replace('SQ_', '')[:14].rjust(15) for c in cols])
for k in sorted(val, key=lambda k: -dur.get(k, 0)):
    if dur.get(k, 0) < 0.2:
        continue
    print(k[:28].ljust(28), f'{dur[k]:8.2f}', *[f'{val[k].get(c, 0):15.4g}' for c in cols])
