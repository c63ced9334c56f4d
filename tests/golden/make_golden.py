"""Generate golden vectors by running the REFERENCE (Darioxavierl/OFDM-LTE at
/root/reference) in this container.  Output: tests/golden/golden_*.npz + a
manifest.  Data only (inputs and expected outputs) -- no reference source is
copied.  The GPU box never runs this (the reference does not exist there).

usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--slow]
"""
import contextlib
import hashlib
import io
import json
import os
import sys
import time

import numpy as np

REF = '/root/reference'
OUT = os.path.dirname(os.path.abspath(__file__))


def h(a):
    a = np.ascontiguousarray(a)
    return hashlib.sha256(a.tobytes()).hexdigest()


def packbits(b):
    return np.packbits(np.asarray(b).astype(np.uint8))


def quiet():
    return contextlib.redirect_stdout(io.StringIO())


def main():
    if not os.path.isdir(REF):
        sys.exit('make_golden.py needs the reference at /root/reference (survey container only)')
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    slow = '--slow' in sys.argv
    from config import LTEConfig
    from core.resource_mapper import LTEResourceGrid, PilotPattern
    from core.modulator import QAMModulator, OFDMModulator
    from core.rayleighchannel import RayleighChannel
    from core.lte_receiver import LTEChannelEstimator, LTEEqualizerZF
    from core.ofdm_core import OFDMSimulator
    from core.channel_coding import crc, segmentation, turbo_encoder, rate_matching, turbo_decoder

    man = {}
    G = {}

    # G1/G2 numerology + index tables
    for bw in [1.25, 2.5, 5.0, 10.0, 15.0, 20.0]:
        for cpt in ['normal', 'extended']:
            c = LTEConfig(bandwidth=bw, modulation='QPSK', cp_type=cpt)
            g = LTEResourceGrid(c.N, c.Nc)
            key = f'num_{bw}_{cpt}'
            G[key + '_scalars'] = np.array([c.N, c.Nc, c.fs, c.cp_length, c.samples_per_ofdm_symbol], dtype=np.float64)
            G[key + '_data'] = g.get_data_indices().astype(np.int32)
            G[key + '_pilot'] = g.get_pilot_indices().astype(np.int32)

    # G3 pilots
    for cell in range(4):
        G[f'pilots_cell{cell}'] = PilotPattern(cell).generate_pilots(200)

    # G4 QAM
    rs = np.random.RandomState(7)
    for mod in ['QPSK', '16-QAM', '64-QAM']:
        q = QAMModulator(mod)
        bps = {'QPSK': 2, '16-QAM': 4, '64-QAM': 6}[mod]
        bits = rs.randint(0, 2, 600 * bps + 1)          # odd length exercises padding
        G[f'qam_{mod}_bits'] = bits.astype(np.uint8)
        G[f'qam_{mod}_syms'] = q.bits_to_symbols(bits)
        pts = (rs.randn(2048) + 1j * rs.randn(2048)) * 0.8
        grid = np.round(rs.uniform(-8, 8, 512)) / {'QPSK': np.sqrt(2), '16-QAM': np.sqrt(10), '64-QAM': np.sqrt(42)}[mod]
        pts = np.concatenate([pts, grid + 1j * rs.randn(512) * 0.5, rs.randn(512) + 1j * grid])
        G[f'qam_{mod}_pts'] = pts
        G[f'qam_{mod}_hard'] = q.symbols_to_bits(pts).astype(np.uint8)

    # G5 OFDM modulation (config 1 full stream)
    c1 = LTEConfig(bandwidth=1.25, modulation='QPSK')
    bits = np.random.RandomState(0).randint(0, 2, 14 * 62 * 2)
    with quiet():
        sig, syms, _ = OFDMModulator(c1, mode='lte').modulate_stream(bits)
    G['mod_c1_bits'] = bits.astype(np.uint8)
    G['mod_c1_signal'] = sig

    # G6 Jakes + filter
    for fD in [0.0, 5.5555555556, 55.555555556]:
        ch = RayleighChannel(1.92e6, fD, [0.0, 0.11e-6 * 10, 0.41e-6 * 10], 10 ** (np.array([0.0, -9.7, -22.8]) / 20))
        np.random.seed(123)
        x = (np.random.randn(1024) + 1j * np.random.randn(1024))
        np.random.seed(321)
        y = ch.filter(x)
        G[f'jakes_fD{fD:.3f}_x'] = x
        G[f'jakes_fD{fD:.3f}_y'] = y

    # G8 estimation + ZF (config 2 grid, random channel)
    c2 = LTEConfig(bandwidth=20.0, modulation='64-QAM')
    est = LTEChannelEstimator(c2, 0)
    rs = np.random.RandomState(5)
    Y = rs.randn(c2.N) + 1j * rs.randn(c2.N)
    with quiet():
        info = est.estimate_channel(Y)
    G['chest_Y'] = Y
    G['chest_H'] = info['channel_estimate']
    G['chest_snr_db'] = np.array([info['pilot_snr_db']])
    G['zf_out'] = LTEEqualizerZF(c2).equalize(Y, info['channel_estimate'])

    # G9 LLRs
    sim = OFDMSimulator(LTEConfig(bandwidth=1.25, modulation='QPSK'))
    rs = np.random.RandomState(9)
    pts = (rs.randn(1024) + 1j * rs.randn(1024)) * 0.7
    nv = np.abs(rs.randn(1024)) * 0.3 + 1e-3
    G['llr_pts'] = pts
    G['llr_nv'] = nv
    G['llr_QPSK'] = sim._calculate_llrs_qpsk(pts, nv)
    G['llr_16-QAM'] = sim._calculate_llrs_16qam(pts, nv)
    G['llr_64-QAM'] = sim._calculate_llrs_64qam(pts, nv)

    # G10 CRC
    rs = np.random.RandomState(10)
    vecs = {'zeros40': np.zeros(40, np.uint8), 'ones40': np.ones(40, np.uint8),
            'alt40': np.array([i % 2 for i in range(40)], np.uint8),
            'rand27760': rs.randint(0, 2, 27760).astype(np.uint8)}
    for k, v in vecs.items():
        G[f'crc_{k}_in'] = v
        G[f'crc_{k}_24a'] = crc.calculate_crc24a(v)
        G[f'crc_{k}_24b'] = crc.calculate_crc24b(v)
        G[f'crc_{k}_16'] = crc.calculate_crc16(v)

    # G11 segmentation
    for B in [40, 6144, 6145, 9232, 27784]:
        tb = np.random.RandomState(B).randint(0, 2, B).astype(np.uint8)
        with quiet():
            blocks, meta = segmentation.segment_code_blocks(tb)
        G[f'seg_{B}_tb'] = packbits(tb)
        G[f'seg_{B}_sizes'] = np.array(meta['block_sizes'], np.int32)
        G[f'seg_{B}_blocks'] = packbits(np.concatenate(blocks))

    # G12/G13 turbo encode + rate matching (+ dematch round trip)
    for K in [40, 1024, 5568, 5632, 6144]:
        cb = np.random.RandomState(K).randint(0, 2, K).astype(np.uint8)
        enc = turbo_encoder.turbo_encode(cb)
        G[f'enc_{K}_in'] = packbits(cb)
        G[f'enc_{K}_out'] = packbits(enc)
        E = 3 * K + 12
        rm = rate_matching.rate_match_turbo(enc, E, K, 0)
        G[f'rm_{K}_out'] = packbits(rm)
        llr = np.random.RandomState(K + 1).randn(E) * 3
        G[f'dm_{K}_in'] = llr
        G[f'dm_{K}_out'] = rate_matching.rate_dematching_turbo(llr, K, 0)
        for E2 in [K + 17, 4 * K]:
            G[f'rm_{K}_E{E2}'] = packbits(rate_matching.rate_match_turbo(enc, E2, K, 2))
            l2 = np.random.RandomState(E2).randn(E2)
            G[f'dm_{K}_E{E2}_in'] = l2
            G[f'dm_{K}_E{E2}_out'] = rate_matching.rate_dematching_turbo(l2, K, 2)

    # G14 turbo decode on noisy LLRs
    for K, its, snr in [(40, 8, 0.0), (1024, 1, 1.0), (1024, 8, -0.5), (5568, 2, 0.5)]:
        if K == 5568 and not slow:
            continue
        cb = np.random.RandomState(K * 3).randint(0, 2, K).astype(np.uint8)
        enc = turbo_encoder.turbo_encode(cb)
        rs = np.random.RandomState(K * 7 + its)
        s = 1 - 2.0 * enc
        sigma2 = 10 ** (-snr / 10)
        llr = 2 * (s + np.sqrt(sigma2) * rs.randn(len(s))) / sigma2
        t = time.time()
        dec = turbo_decoder.turbo_decode(llr, K, num_iterations=its)
        G[f'td_{K}_{its}_llr'] = llr
        G[f'td_{K}_{its}_cb'] = packbits(cb)
        G[f'td_{K}_{its}_dec'] = packbits(dec)
        print(f'turbo K={K} it={its}: {time.time()-t:.1f}s errors={int(np.sum(dec != cb))}')
        # one BCJR pass (a-posteriori) for kernel-level parity
        if K == 1024 and its == 1:
            d = turbo_decoder.LogMAPDecoder()
            ls = np.concatenate([llr[0:3 * K:3], llr[3 * K:3 * K + 3]])
            lp = np.concatenate([llr[1:3 * K:3], llr[3 * K + 3:3 * K + 6]])
            la = rs.randn(K + 3) * 2
            la[K:] = 0
            _, app = d.decode(ls, lp, la, return_extrinsic=False)
            G['bcjr_ls'], G['bcjr_lp'], G['bcjr_la'], G['bcjr_app'] = ls, lp, la, app

    # G17 end-to-end simulate_* (frozen RNG: these ARE the reference's outputs)
    def e2e(name, bw, mod, chan, n_bits, snrs, fn='siso', num_rx=1, full=False):
        c = LTEConfig(bandwidth=bw, modulation=mod)
        with quiet():
            s = OFDMSimulator(c, channel_type=chan)
        bits = np.random.RandomState(0).randint(0, 2, n_bits)
        G[f'{name}_bits'] = packbits(bits)
        G[f'{name}_nbits'] = np.array([n_bits])
        for snr in snrs:
            t = time.time()
            with quiet():
                if fn == 'siso':
                    r = s.simulate_siso(bits, snr)
                elif fn == 'simo':
                    r = s.simulate_simo(bits, snr, num_rx=num_rx, parallel=False)
                else:
                    r = s.simulate_siso_coded(bits, snr)
            k = f'{name}_snr{snr}'
            G[k + '_errors'] = np.array([r['bit_errors']])
            G[k + '_rx'] = packbits(r['bits_received_array'])
            G[k + '_papr'] = np.array([r['papr_db']])
            G[k + '_state'] = np.array(np.random.get_state()[1][:8], dtype=np.uint32)
            if fn == 'coded':
                G[k + '_crc'] = np.array([int(r['crc_pass'])])
                G[k + '_chsnr'] = np.array([r['channel_snr_db']])
                G[k + '_nvmean'] = np.array([r['noise_var_mean']])
                man[k + '_symbols_rx_sha'] = h(r['symbols_rx'])
            if fn == 'simo':
                man[k + '_comb_sha'] = h(r['symbols_rx_combined'])
                if full:
                    G[k + '_comb'] = r['symbols_rx_combined']
            else:
                man[k + '_sigrx_sha'] = h(r['signal_rx'])
                if full:
                    G[k + '_sigrx'] = r['signal_rx']
                    G[k + '_symrx'] = r['symbols_rx']
            man[k + '_sigtx_sha'] = h(r['signal_tx'])
            print(f'{k}: errors={r["bit_errors"]} ber={r["ber"]:.4e} ({time.time()-t:.1f}s)')

    e2e('e2e_c1', 1.25, 'QPSK', 'awgn', 14 * 62 * 2, [0, 5, 10], full=True)
    e2e('e2e_c1odd', 1.25, 'QPSK', 'awgn', 1001, [3], full=True)
    e2e('e2e_c2', 20.0, '64-QAM', 'rayleigh_mp', 14 * 999 * 6, [0, 10, 20, 30])
    e2e('e2e_c2awgn', 20.0, '16-QAM', 'awgn', 5000, [12])
    e2e('e2e_c3', 10.0, '16-QAM', 'rayleigh_mp', 14 * 499 * 4, [5, 15], fn='simo', num_rx=4)
    e2e('e2e_c1simo', 1.25, 'QPSK', 'awgn', 14 * 62 * 2, [2], fn='simo', num_rx=2, full=True)
    e2e('e2e_cod_small', 1.25, 'QPSK', 'awgn', 200, [0, 6], fn='coded')
    e2e('e2e_cod_c2s', 20.0, '64-QAM', 'rayleigh_mp', 2000, [8, 20], fn='coded')
    if slow:
        e2e('e2e_cod_c2', 20.0, '64-QAM', 'rayleigh_mp', 27760, [20], fn='coded')

    np.savez_compressed(os.path.join(OUT, 'golden.npz'), **G)
    man['generated_by'] = 'tests/golden/make_golden.py (reference snapshot 2026-02-13, numpy ' + np.__version__ + ')'
    man['slow'] = slow
    with open(os.path.join(OUT, 'golden_manifest.json'), 'w') as f:
        json.dump(man, f, indent=1, sort_keys=True)
    sz = os.path.getsize(os.path.join(OUT, 'golden.npz'))
    print(f'wrote golden.npz ({sz/1e6:.2f} MB), {len(G)} arrays')


if __name__ == '__main__':
    main()
