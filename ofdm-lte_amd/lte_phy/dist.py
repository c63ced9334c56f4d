"""Multi-GPU plumbing for Monte-Carlo sweeps.

Units are independent (SNR point, trial) frames, so the work shards with no
data-path collective: rank r of W runs global frame ids (k*W + r)*F + [0, F) at
step k.  All randomness is Philox keyed by the global id, so results do not
depend on W.  After the timed region the per-SNR counters
[bit_err, bits, blk_err, blks] are summed with one all-reduce (512 B for 16
SNR points) and the elapsed time is max-reduced.

Backend-agnostic: 'nccl' (RCCL over xGMI on ROCm) reduces on the GPU, 'gloo'
on the CPU (the CPU test suite runs world_size 2 with gloo).
"""
from __future__ import annotations

import numpy as np


def frame_ids(step: int, rank: int, world: int, frames: int) -> np.ndarray:
    """Global frame ids of this rank's batch at `step` (disjoint over ranks and steps)."""
    base = np.uint64((int(step) * int(world) + int(rank)) * int(frames))
    return base + np.arange(frames, dtype=np.uint64)


def snr_index(ids: np.ndarray, n_snr: int) -> np.ndarray:
    """SNR row of each frame: cycles the grid so every rank sees every SNR point."""
    return (ids % np.uint64(n_snr)).astype(np.int32)


def trial_shard(num_trials: int, rank: int, world: int) -> range:
    """Trials a rank owns in run_grid: t = rank, rank + W, ... (balanced per SNR)."""
    return range(rank, int(num_trials), int(world))


def _device(dist):
    import torch
    return torch.device('cuda', torch.cuda.current_device()) if dist.get_backend() == 'nccl' else torch.device('cpu')


def allreduce_counts(counts: np.ndarray, dist=None) -> np.ndarray:
    """Sum uint64 counters over ranks (one collective).  No-op without a process group."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return counts
    import torch
    t = torch.tensor(np.asarray(counts, dtype=np.int64), device=_device(dist))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy().astype(np.uint64)


def allreduce_max(x: float, dist=None) -> float:
    """Max of a scalar over ranks (the slowest rank's elapsed time)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(x)
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64, device=_device(dist))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
