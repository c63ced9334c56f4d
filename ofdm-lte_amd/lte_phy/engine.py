"""Plan cache and batch runner over the C ABI (lte_plan_create / lte_run).

A plan is one device workspace for one configuration (numerology, chain,
channel, payload size, capacity).  `Plan.run` executes the whole
TX -> channel -> RX (-> turbo) chain for a batch of frames on the GPU and
returns counters and any requested host captures.
"""
from __future__ import annotations

import ctypes
from collections import OrderedDict

import numpy as np

from . import _capi as C


class Plan:
    def __init__(self, *, N, Nc, cp_len, bps, n_sym, chain, channel, num_rx=1, delays=(), gains=(), fD=0.0,
                 fs=0.0, n_bits, turbo_iters=8, max_frames=1, cell_id=0, num_tx=1, rank=0, detector=0,
                 precoder=(), sc_fdm=0, bf_adaptive=0, no_equalization=0, precision=None):
        C.device_init()
        d = C.PlanDesc()
        d.N, d.Nc, d.cp_len, d.bps, d.n_sym = N, Nc, cp_len, bps, n_sym
        d.chain, d.channel, d.num_rx = chain, channel, num_rx
        d.n_paths = len(delays)
        if d.n_paths > C.MAX_PATHS:
            raise ValueError('too many multipath taps')
        for i, (dl, g) in enumerate(zip(delays, gains)):
            d.delays[i] = int(dl)
            d.gains[i] = float(g)
        d.fD, d.fs = float(fD), float(fs)
        d.n_bits, d.turbo_iters, d.max_frames, d.cell_id = int(n_bits), int(turbo_iters), int(max_frames), cell_id
        d.num_tx = int(num_tx)
        d.rank, d.detector, d.sc_fdm, d.bf_adaptive = int(rank), int(detector), int(sc_fdm), int(bf_adaptive)
        d.no_equalization = int(no_equalization)
        # float64 (the reference's arithmetic) unless 'f32' is asked for
        d.precision = C.PREC_F64 if C.precision_of(precision) == 'f64' else C.PREC_F32
        if rank and num_tx <= 4 and rank <= 4:   # W [num_tx][rank] -> the [4][4] table of lte_plan_desc.precoder
            #                                    (larger arrays: lte_plan_create rejects them, LTE_EUNSUP)
            W = np.asarray(precoder, dtype=np.complex128).reshape(int(num_tx), int(rank))
            for t in range(W.shape[0]):
                for c in range(W.shape[1]):
                    d.precoder[(t * 4 + c) * 2] = float(W[t, c].real)
                    d.precoder[(t * 4 + c) * 2 + 1] = float(W[t, c].imag)
        self.desc = d
        h = ctypes.c_void_p()
        C.check(C.load().lte_plan_create(ctypes.byref(d), ctypes.byref(h)))
        self.h = h
        info = np.zeros(8, dtype=np.int64)
        C.check(C.load().lte_plan_info(h, C.ptr(info, C.c_i64)))
        self.L, self.n_sym, self.Nd, self.Np, self.n_grp, self.n_cb, self.coded_bits, self.n_re_bits = \
            (int(v) for v in info)
        self.precision = 'f64' if C.load().lte_plan_precision(h) == C.PREC_F64 else 'f32'
        # element types of in_signal and the real / complex captures
        self.cdt = np.complex128 if self.precision == 'f64' else np.complex64
        self.rdt = np.float64 if self.precision == 'f64' else np.float32
        self.num_rx, self.N, self.bps, self.n_bits, self.max_frames = num_rx, N, bps, int(n_bits), int(max_frames)
        self.chain = chain
        self.num_tx = int(num_tx)
        self.coded = chain in (C.CHAIN_CODED, C.CHAIN_SFBC_CODED)
        self.bf = chain == C.CHAIN_BEAMFORMING
        self.mimo = chain >= C.CHAIN_SFBC and not self.bf
        sfbc = chain in (C.CHAIN_SFBC, C.CHAIN_SFBC_CODED)
        # multi-antenna geometry (lte_capi.hip lte_plan_create): REs per OFDM symbol,
        # data SCs carrying data, channel estimates per frame
        self.res = (self.Nd & ~1) if sfbc else self.Nd
        self.rank = int(rank) if rank else self.num_tx
        self.n_dsc = self.res if sfbc else -(-self.Nd // max(1, self.rank))
        self.n_est = self.n_grp if sfbc else self.n_sym
        # per-TX CRS subsets pilots[t::step], step = min(num_tx, 4) (lte_capi.hip
        # plan_mimo_tables, core/mimo_channel_estimator_periodic.py:75-107): the
        # largest subset is what the spatial receiver hands the detector per
        # (RX, estimate, TX) on the pilot-estimate path (LTE_SPATIAL_HP)
        self.cp_len, self.channel = int(cp_len), int(channel)
        self.n_paths, self.max_delay = len(delays), int(max(delays)) if len(delays) else 0
        self.pilots_per_tx = -(-self.Np // min(max(1, self.num_tx), 4))

    def __del__(self):
        try:
            if getattr(self, 'h', None):
                C.load().lte_plan_destroy(self.h)
                self.h = None
        except Exception:
            pass

    # ------------------------------------------------------------------
    def run(self, snr_db, *, snr_index=None, n_snr=1, seed=0, frame_ids=None, frame_id0=0, bits=None,
            bits_broadcast=False, phases=None, phases_broadcast=False, noise=None, noise_broadcast=False,
            stages=C.STAGE_ALL, in_signal=None, capture=(), link_noise=None, link_h=None, link_broadcast=False):
        snr = np.ascontiguousarray(np.atleast_1d(snr_db), dtype=np.float64)   # float64 as the reference (ABI 3)
        B = len(snr)
        a = C.RunArgs()
        a.n_frames = B
        a.snr_db = C.ptr(snr, C.F64)
        keep = [snr]
        if snr_index is not None:
            si = np.ascontiguousarray(snr_index, dtype=np.int32)
            keep.append(si)
            a.snr_index = C.ptr(si, C.I32)
        a.n_snr = int(n_snr)
        a.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        if frame_ids is not None:
            fi = np.ascontiguousarray(frame_ids, dtype=np.uint64)
            keep.append(fi)
            a.frame_ids = C.ptr(fi, C.U64)
        a.frame_id0 = int(frame_id0)
        if bits is not None:
            b = np.ascontiguousarray(bits, dtype=np.uint8)
            keep.append(b)
            a.bits = C.ptr(b, C.U8)
            a.bits_stride = 0 if bits_broadcast else self.n_bits
        if phases is not None:
            ph = np.ascontiguousarray(phases, dtype=np.float64)
            keep.append(ph)
            a.phases = C.ptr(ph, C.F64)
            a.phases_stride = 0 if phases_broadcast else ph.size // B
        if noise is not None:
            z = np.ascontiguousarray(noise, dtype=np.float64)
            keep.append(z)
            a.noise = C.ptr(z, C.F64)
            a.noise_stride = 0 if noise_broadcast else z.size // B
        if link_noise is not None:
            lz = np.ascontiguousarray(link_noise, dtype=np.float64)
            keep.append(lz)
            a.link_noise = C.ptr(lz, C.F64)
            a.link_noise_stride = 0 if link_broadcast else lz.size // B
        if link_h is not None:
            lh = np.ascontiguousarray(link_h, dtype=np.float64)
            keep.append(lh)
            a.link_h = C.ptr(lh, C.F64)
            a.link_h_stride = 0 if link_broadcast else lh.size // B
        counts = np.zeros((max(1, n_snr), 4), dtype=np.uint64)
        a.counts = C.ptr(counts, C.U64)
        out = {'counts': counts}
        ferr = np.zeros(B, dtype=np.uint32)
        a.frame_errors = C.ptr(ferr, C.U32)
        out['frame_errors'] = ferr
        if self.coded:
            crc = np.zeros(B, dtype=np.uint8)
            a.frame_crc_ok = C.ptr(crc, C.U8)
            out['crc_ok'] = crc
        a.stages = int(stages)
        cdt, rdt = self.cdt, self.rdt
        if in_signal is not None:
            xs = np.ascontiguousarray(in_signal, dtype=cdt).reshape(-1, self.L)
            keep.append(xs)
            a.in_signal = xs.ctypes.data
            a.in_signal_stride = 0 if xs.shape[0] == 1 else 2 * self.L
        shapes = {
            'signal_tx': ((B, self.L), cdt, 'cap_signal_tx', None),
            'signal_rx': ((B, self.num_rx, self.L), cdt, 'cap_signal_rx', None),
            'data_syms': ((B, self.n_sym * self.Nd), cdt, 'cap_data_syms', None),
            'H': ((B, self.num_rx, self.n_grp, self.N), cdt, 'cap_H', None),
            'pilot_stats': ((B, self.num_rx, self.n_grp, 2), rdt, 'cap_pilot_stats', None),
            'bits_rx': ((B, self.n_bits), np.uint8, 'cap_bits_rx', C.U8),
            'llr': ((B, self.n_re_bits), rdt, 'cap_llr', None),
            'noise_power': ((B, self.num_rx), rdt, 'cap_noise_power', None),
            'tx_syms': ((B, self.n_sym * self.Nd), cdt, 'cap_tx_syms', None),
        }
        if self.mimo:
            shapes.update({
                'signal_tx': ((B, self.num_tx, self.L), cdt, 'cap_signal_tx', None),
                'data_syms': ((B, self.n_sym * self.res), cdt, 'cap_data_syms', None),
                'H': ((B, self.num_rx, self.n_est, self.num_tx, self.n_dsc), cdt, 'cap_H', None),
                'link_stats': ((B, self.num_rx, self.num_tx, 4), rdt, 'cap_link_stats', None)})
            shapes.pop('pilot_stats')
            shapes.pop('tx_syms')
        if self.bf:
            shapes.update({'H': ((B, self.num_rx, self.num_tx), cdt, 'cap_H', None),
                           'pmi': ((B,), np.int32, 'cap_pmi', C.I32),
                           'bf_gain': ((B,), np.float64, 'cap_bf_gain', C.F64)})
            for k in ('pilot_stats', 'tx_syms', 'signal_tx', 'signal_rx', 'llr', 'noise_power'):
                shapes.pop(k)
        for name in capture:
            shp, dt, field, ct = shapes[name]
            arr = np.zeros(shp, dtype=dt)
            # void* fields take the address; typed fields a ctypes pointer
            setattr(a, field, arr.ctypes.data if ct is None else C.ptr(arr, ct))
            out[name] = arr
        C.check(C.load().lte_run(self.h, ctypes.byref(a)))
        del keep
        return out

    # ------------------------------------------------------------------
    def timing(self, on=True):
        C.check(C.load().lte_timing_enable(self.h, 1 if on else 0))

    def timing_reset(self):
        C.check(C.load().lte_timing_reset(self.h))

    def timing_read(self):
        names = ctypes.create_string_buffer(512)
        ms = np.zeros(32, dtype=np.float64)
        nl = np.zeros(32, dtype=np.int64)
        n = C.check(C.load().lte_timing_read(self.h, names, 512, C.ptr(ms, C.F64), C.ptr(nl, C.c_i64), 32))
        keys = names.value.decode().split(',')
        return {k: (float(ms[i]), int(nl[i])) for i, k in enumerate(keys[:n])}


_CACHE: "OrderedDict[tuple, Plan]" = OrderedDict()
_CACHE_MAX = 8


def get_plan(**kw):
    kw['precision'] = C.precision_of(kw.get('precision'))   # resolved now: part of the cache key
    key = tuple(sorted((k, tuple(v) if isinstance(v, (list, tuple, np.ndarray)) else v) for k, v in kw.items()))
    p = _CACHE.get(key)
    if p is None:
        p = Plan(**kw)
        _CACHE[key] = p
        while len(_CACHE) > _CACHE_MAX:
            _CACHE.popitem(last=False)
    else:
        _CACHE.move_to_end(key)
    return p


def clear_cache():
    _CACHE.clear()
