"""Drop-in mirror of core/mimo_channel_estimator_periodic.py:
MIMOChannelEstimatorPeriodic.  The CRS estimate of every (RX, TX) link is
the GPU estimator (lte_chest_host64: LS at TX t's pilot subset, linear
interpolation, edges held), one call per TX for all RX; FFTs on the GPU too.

The reference's estimate_channel_periodic unpacks three values from
estimate_channel_from_grid, which returns two (core/mimo_channel_estimator_
periodic.py:219), so it and demodulate_and_estimate_mimo always raise that
ValueError; the mirror raises it at the same point (after the first slot's
estimate and its pilot reseeds).  The simulators' SFBC chains carry the
fixed estimator instead."""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np

from . import _capi as C
from .lte_receiver import LTEChannelEstimator, chest
from .resource_mapper import LTEResourceGrid, PilotPattern


class MIMOChannelEstimatorPeriodic:
    """MIMOChannelEstimatorPeriodic (core/mimo_channel_estimator_periodic.py:16-273)."""

    def __init__(self, config, num_tx: int = 2, num_rx: int = 2, slot_size: int = 14):
        self.config = config
        self.num_tx = num_tx
        self.num_rx = num_rx
        self.slot_size = slot_size
        if num_tx not in [2, 4, 8]:
            raise ValueError(f"num_tx debe ser 2, 4 o 8, recibido: {num_tx}")
        self.estimators = [LTEChannelEstimator(config, cell_id=t % 4) for t in range(num_tx)]
        self.pilot_patterns = [PilotPattern(cell_id=t % 4) for t in range(num_tx)]
        self.resource_grid = LTEResourceGrid(config.N, config.Nc)

    def get_orthogonal_pilot_indices(self) -> List[np.ndarray]:
        """TX t: pilots[t % step :: step], step = min(num_tx, 4) (:75-106)."""
        allp = self.resource_grid.get_pilot_indices()
        step = self.num_tx if self.num_tx <= 4 else 4
        return [allp[t % step::step] for t in range(self.num_tx)]

    def estimate_channel_from_grid(self, grid_rx: np.ndarray, return_full_freq: bool = True) -> Tuple[np.ndarray, Dict]:
        """H [num_rx, num_tx, N] (or the per-link mean of the pilot LS values)
        from one received grid per RX (:108-185)."""
        grids = np.asarray(grid_rx, dtype=np.complex128)
        grids = grids.reshape(1, -1) if grids.ndim == 1 else grids
        nr, N = grids.shape
        pidx_tx = self.get_orthogonal_pilot_indices()
        H = np.zeros((nr, self.num_tx, N) if return_full_freq else (nr, self.num_tx), dtype=complex)
        for t in range(self.num_tx):
            pidx = pidx_tx[t]
            # the reference draws TX t's pilots once per RX (each call reseeds the global RNG)
            for _ in range(nr):
                known = self.pilot_patterns[t].generate_pilots(len(pidx))
            Ht, hp, _ = chest(grids, pidx, known, stats=False)
            if return_full_freq:
                H[:, t, :] = Ht
            else:
                H[:, t] = np.mean(hp, axis=-1)
        info = {'num_pilots_per_tx': [len(p) for p in pidx_tx], 'pilot_indices': pidx_tx, 'num_rx': nr,
                'num_tx': self.num_tx, 'N': N}
        return H, info

    def estimate_channel_periodic(self, all_received_grids: List[np.ndarray]) -> Tuple[List[np.ndarray],
                                                                                       List[np.ndarray], float]:
        if len(all_received_grids) == 0:
            return [], [], 0.0
        res = self.estimate_channel_from_grid(all_received_grids[0])
        if len(res) != 3:
            raise ValueError(f"not enough values to unpack (expected 3, got {len(res)})")
        raise AssertionError("unreachable")   # pragma: no cover

    def demodulate_and_estimate_mimo(self, signal_rx: np.ndarray, cp_length: int) -> Tuple[List[np.ndarray],
                                                                                              List[np.ndarray],
                                                                                              List[np.ndarray]]:
        """Whole symbols only, CP removed, FFT / sqrt(N) on the GPU, then the
        periodic estimate (:234-273)."""
        N = self.config.N
        sl = N + cp_length
        x = np.asarray(signal_rx, dtype=np.complex128)
        n = len(x) // sl
        grids = (list(C.fft(x[:n * sl].reshape(n, sl)[:, cp_length:], inverse=False, precision='f64'))
                 if n else [])
        H0, H1, _ = self.estimate_channel_periodic(grids)
        return grids, H0, H1
