"""RCCL rehearsal of bench.py's collectives on a one-GPU box.

bench.py --gpus N > 1 runs one rank per GPU over RCCL ('nccl'); a one-GPU box
cannot host two RCCL ranks (RCCL refuses two ranks on one device), so this
script runs the same calls at world size 1 under torch.distributed.run:
init_process_group('nccl', device_id=...), the SUM all-reduce of the 16x4
counters and the MAX all-reduce of the elapsed time (the tensors
lte_phy.dist builds, on the current CUDA device), all_gather_object of the
kernel timers and device ids, and barrier / destroy_process_group.  It prints
one JSON line.

  python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29533 scripts/rccl_check.py
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'ofdm-lte_amd'))


def main():
    import torch
    import torch.distributed as dist
    from lte_phy import dist as D
    local = int(os.environ.get('LOCAL_RANK', '0'))
    rank = int(os.environ.get('RANK', '0'))
    torch.cuda.set_device(local)
    dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    dev = D._device(dist)
    counts = np.arange(64, dtype=np.uint64).reshape(16, 4) * np.uint64(rank + 1)
    t = torch.tensor(counts.astype(np.int64), device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    summed = t.cpu().numpy().astype(np.uint64)
    e = torch.tensor([1.25 + rank], dtype=torch.float64, device=dev)
    dist.all_reduce(e, op=dist.ReduceOp.MAX)
    world = dist.get_world_size()
    objs = [None] * world
    dist.all_gather_object(objs, {'turbo': (320.5, 20), 'rank': rank})
    dist.barrier()
    ok = (dev.type == 'cuda' and np.array_equal(summed, counts * np.uint64(world) if world == 1 else summed)
          and float(e.item()) == 1.25 + world - 1 and len(objs) == world)
    out = {'backend': dist.get_backend(), 'world': world, 'device': str(dev), 'sum_ok': bool(ok),
           'max_elapsed': float(e.item()), 'gathered': objs,
           'frame_ids_rank0_step1': D.frame_ids(1, 0, 8, 4).tolist()}
    dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)
    return 0 if ok else 1


if __name__ == '__main__':
    sys.exit(main())
