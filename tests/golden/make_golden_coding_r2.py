"""Round-2 channel-coding goldens from the REFERENCE (/root/reference, this
container only): the core.channel_coding names the drop-in gained in round 2.
Output tests/golden/golden_coding_r2.npz (+ _meta.json: segmentation
metadata dicts).  Data only.

  * segment_code_blocks metadata for B in {40, 6144, 6145, 9232, 27784}
    (segmentation.py:74-263) and get_segmentation_info (:362-420)
  * sub_block_interleaver / sub_block_deinterleaver (rate_matching.py:25-190)
  * qpp_interleave / qpp_deinterleave (turbo_encoder.py:76-134)
  * LogMAPDecoder.decode, extrinsic and a-posteriori (turbo_decoder.py:181-278)
  * exact log-MAP (set_decoder_mode(False)): LogMAPDecoder.decode and
    turbo_decode on the round-1 td_40_8 / td_1024_1 inputs
  * rate_dematching_turbo with repetition E = 3 N_cb + 5 (rate_matching.py:433-436)

usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_coding_r2.py
"""
import contextlib
import io
import json
import os
import sys

import numpy as np

REF = '/root/reference'
OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    if not os.path.isdir(REF):
        sys.exit('needs the reference at /root/reference (survey container only)')
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    from core.channel_coding import segmentation, rate_matching, turbo_encoder, turbo_decoder
    g1 = np.load(os.path.join(OUT, 'golden.npz'))
    G, meta = {}, {}
    rs = np.random.RandomState(2024)
    for B in [40, 6144, 6145, 9232, 27784]:
        tb = rs.randint(0, 2, B)
        with contextlib.redirect_stdout(io.StringIO()):
            blocks, md = segmentation.segment_code_blocks(tb)
            back = segmentation.desegment_code_blocks(blocks, md)
        G[f'seg{B}_tb'] = tb.astype(np.uint8)
        G[f'seg{B}_blocks'] = np.concatenate(blocks).astype(np.uint8)
        G[f'seg{B}_back'] = np.asarray(back).astype(np.uint8)
        meta[f'seg{B}'] = {k: (v if not isinstance(v, np.integer) else int(v)) for k, v in md.items()}
        meta[f'info{B}'] = {k: (v if not isinstance(v, np.integer) else int(v))
                            for k, v in segmentation.get_segmentation_info(B).items()}
    for n in [1, 31, 32, 33, 1030, 5574]:
        x = rs.randint(0, 2, n)
        v = rate_matching.sub_block_interleaver(x)
        G[f'sbi{n}_in'] = x.astype(np.uint8)
        G[f'sbi{n}_out'] = v
        G[f'sbi{n}_back'] = rate_matching.sub_block_deinterleaver(v, n)
    for K in [40, 1024, 6144]:
        x = rs.randn(K)
        G[f'qpp{K}_in'] = x
        G[f'qpp{K}_il'] = turbo_encoder.qpp_interleave(x, K)
        G[f'qpp{K}_dil'] = turbo_encoder.qpp_deinterleave(x, K)
    # LogMAPDecoder on a noisy codeword, both modes
    K = 256
    cb = rs.randint(0, 2, K)
    s = 1 - 2.0 * turbo_encoder.turbo_encode(cb)
    llr = 2 * (s + 0.8 * rs.randn(len(s))) / 0.64
    ls = np.concatenate([llr[0:3 * K:3], llr[3 * K:3 * K + 3]])
    lp = np.concatenate([llr[1:3 * K:3], llr[3 * K + 3:3 * K + 6]])
    la = np.concatenate([rs.randn(K) * 1.5, np.zeros(3)])
    G['lmd_ls'], G['lmd_lp'], G['lmd_la'] = ls, lp, la
    with contextlib.redirect_stdout(io.StringIO()):
        for mode, name in [(True, 'maxlog'), (False, 'logmap')]:
            turbo_decoder.set_decoder_mode(mode)
            d = turbo_decoder.LogMAPDecoder()
            b, ext = d.decode(ls, lp, la, return_extrinsic=True)
            _, app = d.decode(ls, lp, la, return_extrinsic=False)
            G[f'lmd_{name}_bits'], G[f'lmd_{name}_ext'], G[f'lmd_{name}_app'] = b, ext, app
        turbo_decoder.set_decoder_mode(False)
        for key, its in [('td_40_8', 8), ('td_1024_1', 1)]:
            Kk = int(key.split('_')[1])
            G[f'{key}_logmap_dec'] = turbo_decoder.turbo_decode(g1[key + '_llr'], Kk, num_iterations=its)
        turbo_decoder.set_decoder_mode(True)
    # rate dematching with repetition
    for K in [40, 1024]:
        Ncb = 3 * (K + 6)
        E = 3 * Ncb + 5
        x = rs.randn(E)
        G[f'dmrep{K}_in'] = x
        G[f'dmrep{K}_out'] = rate_matching.rate_dematching_turbo(x, K, rv_idx=1)
    np.savez_compressed(os.path.join(OUT, 'golden_coding_r2.npz'), **G)
    with open(os.path.join(OUT, 'golden_coding_r2_meta.json'), 'w') as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(f'wrote golden_coding_r2.npz ({len(G)} arrays)')


if __name__ == '__main__':
    main()
