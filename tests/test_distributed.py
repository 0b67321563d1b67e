"""Multi-process path of bench.py on CPU (gloo, world_size 2): each rank owns
its own row batch (weak scaling, no data-path collective) and the reported
wall time is the max over ranks."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    rows, seed = bench.shard_rows(1000, rank, world)
    wall = bench.max_over_ranks(1.0 + rank, "cpu")
    q.put((rank, rows, seed, wall))
    dist.destroy_process_group()


def test_two_rank_weak_scaling_and_max_wall():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert [r[1] for r in res] == [1000, 1000]           # every rank a full batch
    assert res[0][2] != res[1][2]                         # distinct per-rank data
    assert all(r[3] == 2.0 for r in res)                  # max over ranks
