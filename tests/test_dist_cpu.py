"""CPU: the multi-GPU path of bench.py / run_grid (lte_phy/dist.py) under
torch.distributed gloo, world_size 2: disjoint and complete frame-id shards,
SNR coverage on every rank, counter SUM and time MAX reductions."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip('torch')
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from lte_phy import dist as D
    F, S, steps = 96, 16, 3
    ids = np.concatenate([D.frame_ids(k, rank, world, F) for k in range(steps)])
    si = D.snr_index(ids, S)
    counts = np.zeros((S, 4), dtype=np.uint64)
    np.add.at(counts[:, 0], si, ids % np.uint64(7))          # any per-frame statistic
    np.add.at(counts[:, 3], si, np.uint64(1))
    tot = D.allreduce_counts(counts, dist)
    el = D.allreduce_max(0.5 + rank, dist)
    trials = list(D.trial_shard(10, rank, world))
    q.put((rank, ids.tolist(), tot.tolist(), el, trials))
    dist.barrier()
    dist.destroy_process_group()


def test_world2_gloo_shards_and_reductions():
    world, port = 2, _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ids0, ids1 = set(res[0][1]), set(res[1][1])
    assert not ids0 & ids1                                    # disjoint
    assert ids0 | ids1 == set(range(2 * 96 * 3))              # complete: same frames as 1 GPU x 2x steps
    allids = np.array(sorted(ids0 | ids1), dtype=np.uint64)
    ref = np.zeros((16, 4), dtype=np.uint64)
    np.add.at(ref[:, 0], (allids % np.uint64(16)).astype(int), allids % np.uint64(7))
    np.add.at(ref[:, 3], (allids % np.uint64(16)).astype(int), np.uint64(1))
    for r in range(world):
        assert np.array_equal(np.array(res[r][2], dtype=np.uint64), ref)   # SUM on every rank
        assert res[r][3] == 1.5                                            # MAX of elapsed
    assert sorted(res[0][4] + res[1][4]) == list(range(10))               # run_grid trial shards


def test_single_process_reductions_are_identity():
    from lte_phy import dist as D
    c = np.arange(8, dtype=np.uint64).reshape(2, 4)
    assert D.allreduce_counts(c) is c
    assert D.allreduce_max(3.0) == 3.0
