"""Summarise the round-4 PMC passes of scripts/gpu_r4.sh `pmc:<config>` into one
JSON per config: per kernel its traced duration, SQ instruction counts per
frame, VALU / LDS / VMEM shares of active issue, LDS bank-conflict cycles per
LDS instruction, and HBM bytes per frame (FETCH_SIZE x 2 -- the gfx950
correction of MI355X_MICROARCH.md for wide streaming reads, an upper bound for
narrower ones -- plus WRITE_SIZE; both counters in KB).

usage: python scripts/pmc_r4_summary.py gpurun_out/r4d c4__frames_8192 8192 > profiles/r4_pmc_c4.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    val = defaultdict(lambda: defaultdict(float))
    dur = defaultdict(float)
    calls = defaultdict(set)
    f = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    if not f:
        return val, dur, calls
    for r in csv.DictReader(open(f[0])):
        k = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('lte::', '')
        val[k][r['Counter_Name']] += float(r['Counter_Value'])
        if r['Dispatch_Id'] not in calls[k]:
            calls[k].add(r['Dispatch_Id'])
            if 'End_Timestamp' in r and r['End_Timestamp']:
                dur[k] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-6
    return val, dur, calls


def main():
    root, tag, frames = sys.argv[1], sys.argv[2], int(sys.argv[3])
    passes = [load(os.path.join(root, f'pmc_{tag}_p{i}')) for i in range(1, 5)]
    kernels = set()
    for v, _, _ in passes:
        kernels |= set(v)
    out = {}
    for k in sorted(kernels):
        c = {}
        for v, _, _ in passes:
            c.update(v.get(k, {}))
        ms = passes[0][1].get(k, 0.0)
        if ms < 0.001:   # (round 6: was 0.05; config 4's merged noise-power kernels take ~4 us)
            continue
        e = {'ms': round(ms, 3), 'dispatches': len(passes[0][2].get(k, ()))}
        waves = c.get('SQ_WAVES', 0)
        for n in ('SQ_INSTS_VALU', 'SQ_INSTS_SALU', 'SQ_INSTS_LDS', 'SQ_INSTS_VMEM_RD', 'SQ_INSTS_VMEM_WR'):
            if n in c:
                e[n.replace('SQ_INSTS_', '').lower() + '_wave_instr_per_frame'] = round(c[n] / frames, 1)
        act = c.get('SQ_ACTIVE_INST_ANY', 0)
        if act:
            e['share_of_active_issue'] = {u: round(c.get(f'SQ_ACTIVE_INST_{u.upper()}', 0) / act, 3)
                                          for u in ('valu', 'lds', 'vmem')}
        if c.get('SQ_WAVE_CYCLES'):
            wc = c['SQ_WAVE_CYCLES']
            e['wave_cycles'] = {'active': round(act / wc, 3), 'wait_any': round(c.get('SQ_WAIT_ANY', 0) / wc, 3),
                                'wait_inst_any': round(c.get('SQ_WAIT_INST_ANY', 0) / wc, 3)}
        if c.get('SQ_INSTS_LDS'):
            e['lds_conflict_cycles_per_lds_instr'] = round(c.get('SQ_LDS_BANK_CONFLICT', 0) / c['SQ_INSTS_LDS'], 3)
        if 'FETCH_SIZE' in c or 'WRITE_SIZE' in c:
            rd = 2 * c.get('FETCH_SIZE', 0) * 1024 / frames
            wr = c.get('WRITE_SIZE', 0) * 1024 / frames
            e['hbm_bytes_per_frame'] = round(rd + wr)
            e['hbm_read_bytes_per_frame'] = round(rd)
            e['hbm_write_bytes_per_frame'] = round(wr)
            if ms:
                e['hbm_GBs'] = round((rd + wr) * frames / (ms * 1e-3) / 1e9, 1)
        if waves:
            e['waves'] = int(waves)
        out[k] = e
    print(json.dumps({'source': f'scripts/gpu_r4.sh pmc:{tag} (rocprofv3 --pmc, one pass per counter group, '
                                f'one bench step of {frames} frames); scripts/pmc_r4_summary.py',
                      'frames': frames, 'kernels': out}, indent=1))


if __name__ == '__main__':
    main()
