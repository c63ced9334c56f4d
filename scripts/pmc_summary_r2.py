"""Summarise the PMC passes of scripts/gpu_pmc_r2.sh (one bench step of F
frames) per kernel: HBM bytes per frame (FETCH_SIZE x 2 x 1024 for reads --
MI355X_MICROARCH.md's gfx950 correction for wide streaming reads -- and
WRITE_SIZE x 1024 for writes), SQ instruction / wait counters per frame, and
derived VALU / LDS / VMEM shares.  Writes

  profiles/<tag>_pmc_<prec>.json         every kernel (tag r2 by default)
  profiles/pmc_turbo_traffic_<prec>.json  the decoder's bytes (bench.py roofline.traffic)
  profiles/pmc_turbo_sq_<prec>.json       the decoder's VALU instruction count

usage: python scripts/pmc_summary_r2.py [prec] [frames] [src_dir] [tag: output profiles/<tag>_pmc_<prec>.json]
"""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STEPS, PASSES = 27919, 17   # sum(K+3) over the 5 CBs of TB 27760; 8 iterations x 2 + final


def kname(s):
    """'void lte::k_rx_data<double, 1, 6, false, 2048>(...)' -> 'k_rx_data'."""
    s = s[5:] if s.startswith('void ') else s
    return s.split('(')[0].split('<')[0].strip().replace('lte::', '')


def per_kernel(path):
    """{kernel: {counter: value summed over dispatches}} and dispatch counts."""
    tot = defaultdict(lambda: defaultdict(float))
    n = defaultdict(set)
    with open(path) as f:
        for r in csv.DictReader(f):
            k = kname(r['Kernel_Name'])
            tot[k][r['Counter_Name']] += float(r['Counter_Value'])
            n[k].add(r['Dispatch_Id'])
    return tot, {k: len(v) for k, v in n.items()}


def kernel_time(path):
    t = defaultdict(float)
    with open(path) as f:
        for r in csv.DictReader(f):
            k = kname(r['Kernel_Name'])
            t[k] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9
    return t


def main(prec='f64', frames=8192, src=os.path.join(ROOT, 'gpurun_out'), tag='r2'):
    frames = int(frames)
    d = lambda n: os.path.join(src, f'pmc_{prec}_{n}')   # noqa: E731
    fk, _ = per_kernel(os.path.join(d('FETCH_SIZE'), 'run_counter_collection.csv'))
    wk, _ = per_kernel(os.path.join(d('WRITE_SIZE'), 'run_counter_collection.csv'))
    s1, _ = per_kernel(os.path.join(d('sq1'), 'run_counter_collection.csv'))
    s2, _ = per_kernel(os.path.join(d('sq2'), 'run_counter_collection.csv'))
    tk = kernel_time(os.path.join(d('sq1'), 'run_kernel_trace.csv'))
    out = {}
    for k in sorted(fk):
        if k.startswith('__amd'):
            continue
        rd = 2.0 * fk[k].get('FETCH_SIZE', 0.0) * 1024
        wr = wk.get(k, {}).get('WRITE_SIZE', 0.0) * 1024
        sq = dict(s1.get(k, {}))
        sq.update(s2.get(k, {}))
        e = {'read_bytes_per_frame': rd / frames, 'write_bytes_per_frame': wr / frames,
             'hbm_bytes_per_frame': (rd + wr) / frames,
             'sq_per_frame': {c: v / frames for c, v in sorted(sq.items())}}
        if sq.get('SQ_ACTIVE_INST_ANY'):
            a = sq['SQ_ACTIVE_INST_ANY']
            e['share_of_active_issue'] = {c.replace('SQ_ACTIVE_INST_', '').lower(): round(sq.get(c, 0) / a, 3)
                                          for c in ('SQ_ACTIVE_INST_VALU', 'SQ_ACTIVE_INST_LDS', 'SQ_ACTIVE_INST_VMEM')}
        if sq.get('SQ_WAVE_CYCLES'):
            e['wait_share_of_wave_cycles'] = round(sq.get('SQ_WAIT_ANY', 0) / sq['SQ_WAVE_CYCLES'], 3)
            e['lds_wait_share_of_wave_cycles'] = round(sq.get('SQ_WAIT_INST_LDS', 0) / sq['SQ_WAVE_CYCLES'], 3)
        if sq.get('SQ_INSTS_LDS'):
            e['lds_bank_conflict_cycles_per_lds_instr'] = round(sq.get('SQ_LDS_BANK_CONFLICT', 0) / sq['SQ_INSTS_LDS'], 3)
        if tk.get(k):
            e['profiled_s'] = tk[k]
        out[k] = e
    meta = {'precision': prec, 'frames_per_launch': frames,
            'command': f'rocprofv3 --pmc <C> --kernel-trace --output-format csv -- python3 bench.py --frames {frames} '
                       f'--steps 1 --warmup 0 --no-cpu --precision {prec} (scripts/gpu_pmc_r2.sh: one pass per '
                       'FETCH_SIZE / WRITE_SIZE, two 8-counter SQ passes)',
            'correction': 'MI355X_MICROARCH.md HBM section: gfx950 FETCH_SIZE reports 1/2 of wide streaming-read '
                          'bytes -> read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE x 1024 exact',
            'kernels': out}
    with open(os.path.join(ROOT, 'profiles', f'{tag}_pmc_{prec}.json'), 'w') as f:
        json.dump(meta, f, indent=1)
    tk_name = 'k_turbo64' if prec == 'f64' else 'k_turbo'
    t = out[tk_name]
    esz = 8 if prec == 'f64' else 4
    # checkpoint rows stored (and loaded) per step: 8 (f64) / 7 (f32) states per
    # super-window of 24 (f64, LTE_TURBO64_SUB = 3) / 16 (f32) steps
    ckrows = (8 / 24.0) if prec == 'f64' else (7 / 16.0)
    model = STEPS * PASSES * esz * (6 + 1 + 2 * ckrows)
    with open(os.path.join(ROOT, 'profiles', f'pmc_turbo_traffic_{prec}.json'), 'w') as f:
        json.dump({'kernel': tk_name, 'frames_per_launch': frames, 'command': meta['command'],
                   'correction': meta['correction'],
                   'read_bytes_per_frame': t['read_bytes_per_frame'], 'write_bytes_per_frame': t['write_bytes_per_frame'],
                   'bytes_per_frame': t['hbm_bytes_per_frame'],
                   'model_bytes_per_frame': round(model),
                   'model_note': f'per code-block step per pass: fwd 3 + bwd 3 row loads, 1 extrinsic store, '
                                 f'{ckrows:.4f} checkpoint rows stored + loaded, {esz} B each; x {STEPS} steps x '
                                 f'{PASSES} passes (first pass skips the a-priori loads)'}, f, indent=1)
    sq = t['sq_per_frame']
    with open(os.path.join(ROOT, 'profiles', f'pmc_turbo_sq_{prec}.json'), 'w') as f:
        json.dump({'kernel': tk_name, 'frames_per_launch': frames, 'command': meta['command'],
                   'valu_wave_instr_per_frame': sq.get('SQ_INSTS_VALU'),
                   'vmem_wave_instr_per_frame': sq.get('SQ_INSTS_VMEM_RD', 0) + sq.get('SQ_INSTS_VMEM_WR', 0),
                   'valu_instr_per_cb_step_pass': sq.get('SQ_INSTS_VALU', 0) / (STEPS * PASSES / 64),
                   # issue cycles of one wave64 VALU instruction on a SIMD-32: 2 (f32), 4 (f64 adds / max:
                   # 16 lanes per cycle, profiles/r2_valu_peak_microbench.jsonl)
                   'issue_cycles_per_instr': 4 if prec == 'f64' else 2,
                   'counters_per_frame': sq}, f, indent=1)
    for k, e in out.items():
        print(f"{k:24s} {e['hbm_bytes_per_frame'] / 1e3:10.1f} KB/frame  "
              f"{e.get('profiled_s', 0) * 1e3:8.2f} ms  {e.get('share_of_active_issue', '')} "
              f"wait {e.get('wait_share_of_wave_cycles', '')} lds-wait {e.get('lds_wait_share_of_wave_cycles', '')} "
              f"bank {e.get('lds_bank_conflict_cycles_per_lds_instr', '')}")
    print(f"{tk_name}: {t['hbm_bytes_per_frame'] / 1e6:.2f} MB/frame measured, {model / 1e6:.2f} MB/frame model")


if __name__ == '__main__':
    main(*sys.argv[1:])
