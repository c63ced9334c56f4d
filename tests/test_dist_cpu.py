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


def _bench(args, env=None):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(root, 'bench.py')] + args, env=e, capture_output=True,
                          text=True, timeout=300)


def test_bench_self_launches_ranks_dry_run():
    """`bench.py --gpus 2` with no launcher starts 2 ranks itself (torch.distributed.run,
    gloo in --dry-run), shards frames by global id and reports the distinct
    devices (here: ranks) and the summed counters of both ranks."""
    import json
    from lte_phy import dist as D
    F, steps = 64, 2
    r = _bench(['--gpus', '2', '--dry-run', '--steps', str(steps), '--warmup', '0', '--frames', str(F),
                '--cpu-seconds', '0.5'])
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(line) == 1, r.stdout          # one JSON line, rank 0 only
    out = json.loads(line[0])
    assert out['n_gpus'] == 2 and out['config']['ranks'] == 2 and out['config']['global_batch'] == 2 * F
    ids = np.concatenate([D.frame_ids(k, rk, 2, F) for k in range(steps) for rk in range(2)])
    si = D.snr_index(ids, 16)
    ref = np.zeros((16, 4), dtype=np.uint64)
    np.add.at(ref[:, 0], si, ids % np.uint64(7))
    np.add.at(ref[:, 1], si, np.uint64(27760))
    np.add.at(ref[:, 2], si, (ids % np.uint64(3) == 0).astype(np.uint64))
    np.add.at(ref[:, 3], si, np.uint64(1))
    assert np.array_equal(np.array(out['counts'], dtype=np.uint64), ref)
    # the N > 1 line carries the CPU baseline (timed by the launching parent,
    # before any rank starts) and a roofline priced on the slowest rank's timers
    cpu = out['cpu_baseline']
    assert cpu and cpu['value'] > 0 and cpu['cores'] >= 1 and cpu['kind'] == 'port'
    # BASELINE.md's CPU timing: 1 process, the GPU's share, all cores (extrapolated)
    assert cpu['single_process']['cores'] == 1 and cpu['single_process']['value'] > 0
    assert cpu['gpu_share']['value'] == cpu['value'] and cpu['all_cores']['cores'] == os.cpu_count()
    roof = out['roofline']
    # bound = the measured limiter (the exact recursion's HBM row stream), with
    # SURVEY §8(d)'s K7 VALU figure beside it
    assert roof['bound'] == roof['measured_limiter']
    assert (roof['unit'], roof['peak']) == (('GB/s', 8000.0) if roof['bound'] == 'hbm' else ('Top/s', 39.32))
    assert roof['valu']['unit'] == 'Top/s' and roof['valu']['peak'] == 39.32 and roof['valu_frac'] > 0
    for k in ('achieved', 'frac', 'traffic', 'hbm_frac', 'avg_launch_ms', 'hbm_row_stream', 'stage_bytes',
              'measured_limiter', 'front_end'):
        assert k in roof, k
    assert set(roof['front_end']) >= {'ofdm_tx', 'rx_data', 'dematch'}
    assert roof['hbm_row_stream']['peak_GBs'] == 8000.0 and 'store_cost' in roof['hbm_row_stream']
    # the BER-match sample comes from the CPU baseline's oracle frames; no device here
    assert out['ber_match'] is None and 'frames' not in cpu
    # rank 1's synthetic timer is 1 % slower: the merged timer is the max
    assert abs(roof['avg_launch_ms'] - 0.87 * out['ms_per_step'] * 1.01) < 0.05 * out['ms_per_step']


@pytest.mark.parametrize('config', [4, 5])
def test_bench_other_configs_dry_run_world2(config):
    """`bench.py --config 4|5 --gpus 2 --dry-run`: config 5 is the config
    BASELINE names for the 8-GPU sharded grid.  The line sums both ranks'
    counters (each config's own payload size), carries a roofline priced on
    the slowest rank (config 4: the decoder's K7 view; config 5: the dominant
    stage against HBM with the plan's stage bytes) and a cpu_baseline whose
    note states the cores actually used."""
    import json
    from lte_phy import dist as D
    F, steps = 64, 2
    r = _bench(['--config', str(config), '--gpus', '2', '--dry-run', '--steps', str(steps), '--warmup', '0',
                '--frames', str(F), '--cpu-seconds', '0.3'])
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(line) == 1, r.stdout
    out = json.loads(line[0])
    nb = {4: 27760, 5: 14 * 999 * 6}[config]
    ids = np.concatenate([D.frame_ids(k, rk, 2, F) for k in range(steps) for rk in range(2)])
    si = D.snr_index(ids, 16)
    ref = np.zeros((16, 4), dtype=np.uint64)
    np.add.at(ref[:, 0], si, ids % np.uint64(7))
    np.add.at(ref[:, 1], si, np.uint64(nb))
    np.add.at(ref[:, 2], si, (ids % np.uint64(3) == 0).astype(np.uint64))
    np.add.at(ref[:, 3], si, np.uint64(1))
    assert np.array_equal(np.array(out['counts'], dtype=np.uint64), ref)
    assert out['config']['bench_config'] == config and out['n_gpus'] == 2
    roof = out['roofline']
    assert roof is not None
    if config == 4:
        assert roof['kernel'] == 'k_turbo64' and roof['frac'] > 0 and 'hbm_row_stream' in roof
    else:
        # rx_chest (k_rx_fft_mimo) is the largest synthetic stage: the RX streams
        # (no CP) in, the data-SC values + LS pilot estimates out per frame
        assert roof['bound'] == 'hbm' and roof['stage'] == 'rx_chest' and roof['unit'] == 'GB/s'
        c = 16
        assert roof['alg_bytes_per_frame'] == 4 * 14 * 2048 * c + 14 * 4 * 250 * c + 4 * 14 * 4 * 50 * c
        assert roof['traffic'] and roof['hbm_frac'] is not None
        assert set(roof['other_stages']) == {'ofdm_tx', 'fading', 'channel', 'rx_data'}
    cpu = out['cpu_baseline']
    assert cpu['cores'] == min(32, os.cpu_count())
    assert cpu['note'].startswith(f"{cpu['cores']} single-threaded worker processes")
    assert f"{os.cpu_count()} CPUs visible" in cpu['note']


def test_merge_timers_takes_slowest_rank():
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location('bench_mod', os.path.join(root, 'bench.py'))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    m = b.merge_timers([{'turbo': (10.0, 5), 'dematch': (1.0, 5)}, {'turbo': (12.0, 5), 'dematch': (0.5, 5)}, None])
    assert m == {'turbo': (12.0, 5), 'dematch': (1.0, 5)}
    # the exact decoder's row model: 116 rows of 8 B per step over 8 iterations
    assert b.decoder_row_bytes(5568, 8, 8) == 5568 * 116 * 8 + 3 * 2 * 17 * 8 + 5568 / 8


def test_bench_rejects_world_size_mismatch():
    r = _bench(['--gpus', '2', '--dry-run', '--steps', '1', '--warmup', '0'], env={'WORLD_SIZE': '1'})
    assert r.returncode == 2 and 'WORLD_SIZE' in r.stderr
